# SPDX-License-Identifier: BSD-2-Clause
"""tests/hostmem.py: the buffers GPU tests register start on a page of their
own and own every page they touch (no other object shares one)."""
import numpy as np

from hostmem import PAGE, _KEEP, page_buffer


def test_page_buffer_owns_its_pages():
    for count, dtype in ((1, np.uint8), (4097, np.uint8), (100, np.dtype([("a", "<u8"), ("b", "<u8")]))):
        a = page_buffer(count, dtype)
        assert a.ctypes.data % PAGE == 0
        assert len(a) == count and (a.view(np.uint8) == 0).all()
        m = _KEEP[-1]  # the mapping behind it: whole pages, kept for the process
        assert len(m) % PAGE == 0 and len(m) >= a.nbytes
        a.view(np.uint8)[:] = 7  # writable
