# SPDX-License-Identifier: BSD-2-Clause
"""oo_gpu_rx_host_register's contract, enforced by the library
(include/oo_gpu_rx.h; DESIGN.md §5 round 6, the registration faults), on
host-only contexts -- they keep the same books as device contexts, so every
return here is the one a device context gives:

* whole pages only: a start or a length that is not a page multiple is
  -EINVAL;
* no page in two registrations, across every context of the process:
  -EINVAL, adjacent ranges are fine;
* a context holding registrations does not close (-EBUSY) and stays usable;
  after the caller unregisters, it closes; the same pages can then be
  registered again;
* unregister of an address that is not a registered base of the context:
  -ENOENT; a group with a member holding registrations does not close."""
import ctypes
import errno
import mmap

import numpy as np
import pytest

from hostmem import PAGE
from onload_amd import _abi
from onload_amd.group import GpuRxGroup
from onload_amd.rx import GpuRxStack


@pytest.fixture()
def pages():
    """Eight pages of their own (unmapped when the last view goes)."""
    return np.frombuffer(mmap.mmap(-1, 8 * PAGE), np.uint8)


def _reg(stack, addr, nbytes):
    lib = stack._lib
    d = ctypes.c_void_p()
    rc = lib.oo_gpu_rx_host_register(stack._ctx, ctypes.c_void_p(addr), nbytes, ctypes.byref(d))
    return rc, d.value


def _unreg(stack, addr):
    return stack._lib.oo_gpu_rx_host_unregister(stack._ctx, ctypes.c_void_p(addr))


def test_whole_pages_only(pages):
    s = GpuRxStack(device=-1)
    base = pages.ctypes.data
    assert base % PAGE == 0
    for addr, nbytes in ((base + 64, PAGE), (base, PAGE + 1), (base, PAGE - 64), (base, 0),
                         (base + PAGE // 2, 2 * PAGE)):
        assert _reg(s, addr, nbytes)[0] == -errno.EINVAL, (addr - base, nbytes)
    rc, d = _reg(s, base, 2 * PAGE)
    assert rc == 0 and d == base  # a host-only context's "device" address is p
    assert s.host_registered() == 1
    assert _unreg(s, base) == 0 and s.host_registered() == 0
    s.close()


def test_no_page_in_two_registrations(pages):
    a = GpuRxStack(device=-1)
    b = GpuRxStack(device=-1)
    base = pages.ctypes.data
    assert _reg(a, base + 2 * PAGE, 2 * PAGE)[0] == 0
    for st in (a, b):  # the same context or another one
        for addr, nbytes in ((base + 2 * PAGE, 2 * PAGE), (base + PAGE, 2 * PAGE),
                             (base + 3 * PAGE, 2 * PAGE), (base, 8 * PAGE),
                             (base + 3 * PAGE, PAGE)):
            assert _reg(st, addr, nbytes)[0] == -errno.EINVAL, (addr - base, nbytes)
    # adjacent on both sides: fine
    assert _reg(b, base + PAGE, PAGE)[0] == 0
    assert _reg(b, base + 4 * PAGE, 4 * PAGE)[0] == 0
    # b cannot unregister a's range; a can
    assert _unreg(b, base + 2 * PAGE) == -errno.ENOENT
    assert _unreg(a, base + 2 * PAGE) == 0
    assert _unreg(a, base + 2 * PAGE) == -errno.ENOENT  # already gone
    assert _reg(a, base + 2 * PAGE, 2 * PAGE)[0] == 0  # the pages are free again
    for st, addr in ((a, base + 2 * PAGE), (b, base + PAGE), (b, base + 4 * PAGE)):
        assert _unreg(st, addr) == 0
    a.close()
    b.close()


def test_close_refuses_while_registered(pages):
    s = GpuRxStack(device=-1)
    base = pages.ctypes.data
    assert s.host_register(pages[:PAGE]) == base  # the Python mirror: whole pages
    assert s.host_registered() == 1
    assert s._lib.oo_gpu_rx_close(s._ctx) == -errno.EBUSY
    with pytest.raises(OSError) as e:
        s.close()
    assert e.value.errno == errno.EBUSY
    # still open and usable
    assert s.filter_insert(1, 4, "10.0.0.1", 80, None, 0, 6) == 0
    assert s.table_gen() == 1
    s.host_unregister(pages[:PAGE])
    s.close()
    assert s._ctx is None


def test_python_mirror_registers_the_arrays_pages(pages):
    s = GpuRxStack(device=-1)
    with pytest.raises(OSError) as e:  # not the start of a page
        s.host_register(pages[100:200])
    assert e.value.errno == errno.EINVAL
    assert s.host_register(pages[:100]) == pages.ctypes.data  # its page, whole
    with pytest.raises(OSError) as e:  # the same page again
        s.host_register(pages[:PAGE])
    assert e.value.errno == errno.EINVAL
    s.host_unregister(pages[:100])
    s.close()


def test_group_close_refuses_while_a_member_holds_registrations(pages):
    g = GpuRxGroup(devices=[-1, -1])
    m = g.members[1]
    assert m.host_register(pages[:PAGE]) == pages.ctypes.data
    assert g._lib.oo_gpu_rx_group_close(g._g) == -errno.EBUSY
    with pytest.raises(OSError):
        g.close()
    m.host_unregister(pages[:PAGE])
    g.close()


def test_abi_close_signatures():
    lib = _abi.load_library()
    assert lib.oo_gpu_rx_close(None) == 0
    assert lib.oo_gpu_rx_group_close(None) == 0
    assert lib.oo_gpu_rx_host_registered(None) == -errno.EINVAL
