# SPDX-License-Identifier: BSD-2-Clause
"""The join shape's collectives (oo_gpu_rx_group_share_tables / _share_ops /
_gather_rccl / _sum_counters, onload_amd/csrc/oo_gpu_rx_group.cpp) run
without a GPU: two host-only members joined over a transport whose ranks are
threads (tests/group_xport.py), so the same sequencing code RCCL drives runs
here with failures injected on one rank.

What is held: every rank enters the same collectives in the same order,
whatever failed locally (no thread is left waiting: a hang fails the test);
a failure that would leave one rank out of the next collective is agreed on
first and returned by every rank; a count mismatch in the gather is -EINVAL
on every rank and moves nothing; a replica never imports a stale image.
(the RCCL form: tests/test_gpu_group_rccl.py.)"""
import ctypes
import errno

import numpy as np
import pytest

from group_xport import ThreadXport, run_ranks
from onload_amd import _abi, pktgen
from onload_amd.group import GpuRxGroup

N = 2


def _join(x, rank, **kw):
    kw.setdefault("max_socks", 8192)
    return GpuRxGroup.join_transport(rank, N, x.transport(rank), **kw)


def _groups(x, **kw):
    return run_ranks(lambda r: _join(x, r, **kw), N)


def _images(gs):
    return [g.members[0].image_host().tobytes() for g in gs]


def _errno(res):
    return res.errno if isinstance(res, OSError) else res


def _world_on_rank0(g):
    filters, socks = pktgen.world(5)
    g.load_world(filters[:400], socks)
    return filters


def test_tables_and_ops_replicate_over_the_transport():
    x = ThreadXport(N)
    gs = _groups(x)
    assert [g.uses_rccl for g in gs] == [False, False]
    filters = _world_on_rank0(gs[0])
    assert run_ranks(lambda r: gs[r].share_tables(), N) == [None, None]
    a, b = _images(gs)
    assert a == b
    # changes on rank 0 only (-EPERM elsewhere), then shared in order
    f = filters[0]
    assert gs[1].filter_remove_raw(f.sock, f.af, bytes(f.laddr)[:4 if f.af == 4 else 16],
                                   f.lport_be, None, f.rport_be, f.proto) == -errno.EPERM
    for f in filters[:50]:
        ra = None if f.raddr_any else bytes(f.raddr)[:4 if f.af == 4 else 16]
        assert gs[0].filter_remove_raw(f.sock, f.af, bytes(f.laddr)[:4 if f.af == 4 else 16],
                                       f.lport_be, ra, f.rport_be, f.proto) == 0
    assert run_ranks(lambda r: gs[r].share_ops(), N) == [50, 50]
    a, b = _images(gs)
    assert a == b
    assert x.calls[0] == x.calls[1]  # the same collectives, in the same order
    for g in gs:
        g.close()


def test_share_ops_header_failure_on_one_rank_is_agreed():
    """Rank 1's copy of the header fails (the old code returned there while
    rank 0 went on into the body broadcasts alone): every rank returns -EIO,
    nobody hangs, rank 0 keeps its ops, and the next share_ops delivers them."""
    x = ThreadXport(N)
    gs = _groups(x)
    _world_on_rank0(gs[0])
    assert run_ranks(lambda r: gs[r].share_tables(), N) == [None, None]
    filters, socks = pktgen.world(4)
    for i, f in enumerate(filters[:20]):
        ra = None if f.raddr_any else bytes(f.raddr)[:4 if f.af == 4 else 16]
        gs[0].filter_insert_raw(7000 + i, f.af, bytes(f.laddr)[:4 if f.af == 4 else 16],
                                f.lport_be, ra, f.rport_be, f.proto)
    x.fail[(1, "bcast", x.count[1].get("bcast", 0))] = True
    res = run_ranks(lambda r: gs[r].share_ops(), N)
    assert [_errno(e) for e in res] == [errno.EIO, errno.EIO]
    assert x.timeouts == 0
    assert x.calls[0] == x.calls[1]
    assert run_ranks(lambda r: gs[r].share_ops(), N) == [20, 20]
    a, b = _images(gs)
    assert a == b
    for g in gs:
        g.close()


def test_share_ops_body_failure_reported_after_the_last_broadcast():
    """A failed body chunk on rank 1 (of a share that needs two chunks):
    rank 1 still enters the second chunk's broadcast, and reports -EIO after
    it; rank 0 succeeds."""
    x = ThreadXport(N)
    gs = _groups(x, max_socks=16384, ip4_log2=17)
    assert run_ranks(lambda r: gs[r].share_tables(), N) == [None, None]
    s = _abi.Sock()
    for i in range(9000):  # > one 8192-op chunk
        assert gs[0].sock_set(i, s) == 0
    x.fail[(1, "bcast", x.count[1].get("bcast", 0) + 1)] = True  # the first body chunk
    res = run_ranks(lambda r: gs[r].share_ops(), N)
    assert res[0] == 9000 and _errno(res[1]) == errno.EIO
    assert x.timeouts == 0 and x.calls[0] == x.calls[1]
    for g in gs:
        g.close()


def test_share_tables_never_imports_a_stale_image():
    """Rank 1 misses the image broadcast (its staging still holds the last
    share's image, which would pass the import's checks: ADVICE r5): every
    rank returns an error and rank 1's tables are unchanged."""
    x = ThreadXport(N)
    gs = _groups(x)
    _world_on_rank0(gs[0])
    assert run_ranks(lambda r: gs[r].share_tables(), N) == [None, None]
    before = _images(gs)[1]
    for i, f in enumerate(pktgen.world(3)[0][:30]):
        ra = None if f.raddr_any else bytes(f.raddr)[:4 if f.af == 4 else 16]
        gs[0].filter_insert_raw(6000 + i, f.af, bytes(f.laddr)[:4 if f.af == 4 else 16],
                                f.lport_be, ra, f.rport_be, f.proto)
    x.fail[(1, "bcast", x.count[1].get("bcast", 0))] = True
    res = run_ranks(lambda r: gs[r].share_tables(), N)
    assert [_errno(e) for e in res] == [errno.EIO, errno.EIO]
    assert _images(gs)[1] == before
    assert run_ranks(lambda r: gs[r].share_tables(), N) == [None, None]
    a, b = _images(gs)
    assert a == b != before
    for g in gs:
        g.close()


def _records(n, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, n * 32, dtype=np.uint8)


@pytest.mark.parametrize("n0,n1", [(100, 37), (0, 5), (6, 0)])
def test_gather_moves_every_ranks_records(n0, n1):
    x = ThreadXport(N)
    gs = _groups(x)
    recs = [_records(n0, 1), _records(n1, 2)]
    dst = np.zeros((n0 + n1) * 32, np.uint8)

    def run(r):
        d = dst.ctypes.data if r == 0 else 0
        gs[r].gather_rccl(recs[r].ctypes.data, (n0, n1)[r], d, [n0, n1] if r == 0 else None)
    assert run_ranks(run, N) == [None, None]
    assert dst.tobytes() == recs[0].tobytes() + recs[1].tobytes()
    for g in gs:
        g.close()


@pytest.mark.parametrize("case", ["count", "no_dst", "no_counts"])
def test_gather_mismatch_is_einval_on_every_rank(case):
    """Rank 0's counts disagree with rank 1's n (or rank 0 gives no
    destination / counts): -EINVAL on every rank, nothing moved, no hang."""
    x = ThreadXport(N)
    gs = _groups(x)
    recs = [_records(10, 1), _records(20, 2)]
    dst = np.zeros(64 * 32, np.uint8)
    counts = [10, 19 if case == "count" else 20]

    def run(r):
        d = dst.ctypes.data if (r == 0 and case != "no_dst") else 0
        c = counts if (r == 0 and case != "no_counts") else None
        gs[r].gather_rccl(recs[r].ctypes.data, (10, 20)[r], d, c)
    res = run_ranks(run, N)
    assert [_errno(e) for e in res] == [errno.EINVAL, errno.EINVAL]
    assert not dst.any() and x.count[0].get("gather", 0) == 0 == x.count[1].get("gather", 0)
    assert x.timeouts == 0
    for g in gs:
        g.close()


def test_sum_counters_over_the_transport():
    x = ThreadXport(N)
    gs = _groups(x)
    c = [np.arange(_abi.R_COUNT, dtype=np.uint32) * (r + 1) for r in range(N)]
    assert run_ranks(lambda r: gs[r].sum_counters(c[r].ctypes.data), N) == [None, None]
    for r in range(N):
        np.testing.assert_array_equal(c[r], np.arange(_abi.R_COUNT, dtype=np.uint32) * 3)
    for g in gs:
        g.close()


def test_join_transport_rejects_device_members_and_missing_calls():
    x = ThreadXport(1)
    lib = _abi.load_library()
    from onload_amd.group import _cfg
    g = ctypes.c_void_p()
    t = x.transport(0)
    for dev, tt in ((0, t), (-1, None)):
        cfg = _cfg(dev, 64, 16, 14, (0,))
        rc = lib.oo_gpu_rx_group_join_transport(ctypes.byref(g), ctypes.byref(cfg), 0, 1,
                                                None if tt is None else ctypes.byref(tt))
        assert rc == -errno.EINVAL
    # a transport group of one rank: its collectives are its own
    g1 = GpuRxGroup.join_transport(0, 1, t, max_socks=64)
    g1.share_tables()
    assert g1.share_ops() == 0
    g1.close()
