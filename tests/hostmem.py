# SPDX-License-Identifier: BSD-2-Clause
"""Host buffers the GPU tests register with the device (hipHostRegister,
through oo_gpu_rx_host_register or the poll shim): whole pages of their own
from an anonymous mmap -- no other object of the process shares a page with
a registered range -- kept for the life of the process, so a range once
registered is never handed to a pageable buffer that torch later copies
(the faults)."""
import mmap

import numpy as np

PAGE = mmap.PAGESIZE
_KEEP = []


def whole_pages(nbytes: int) -> int:
    """nbytes rounded up to whole pages (a registration's size)."""
    return -(-int(nbytes) // PAGE) * PAGE


def page_buffer(count: int, dtype=np.uint8) -> np.ndarray:
    """A zeroed array of `count` items on pages of its own."""
    nbytes = max(1, int(count) * np.dtype(dtype).itemsize)
    m = mmap.mmap(-1, (nbytes + PAGE - 1) // PAGE * PAGE)
    _KEEP.append(m)
    return np.frombuffer(m, dtype=np.uint8, count=nbytes).view(dtype)
