# SPDX-License-Identifier: BSD-2-Clause
"""The key index (oo_rx_device.h, DESIGN.md "The key index") against the
oracle's walks: keys that pile into one bucket (lookups past full buckets,
misses that scan them), an overflow that turns the index off, a socket
whose fields change under its filter (a PREFERRED entry its key no longer
hashes to: the index turns off), lanes that fall back to the walks
(multicast, bind2dev), mixed IPv4 / IPv6 waves, and the walks alone
(tuning `walks`) on the edge corpus and every configuration's sample."""
import os

import numpy as np
import pytest

from frames import L4A, L6A, PEER4, PEER6, _sock, edge_frames, edge_world, eth, install, ipv4, \
    ipv6, pack, tcp, udp
from gpu_util import diff_report, run_dev
from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack, htons
from oracle_lib import OracleStack, counters_of

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)
HWPORTS = (0, 1, 3, 2, 5)
NB4 = 1 << 16  # buckets per protocol region for a 2^16-slot IPv4 table
NE6 = 1 << 17  # IPv6 entries for a 2^14-slot IPv6 table (OO_KX_V6_MUL 8)


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _mix(h):
    h = h ^ (h >> np.uint32(16))
    h = h * np.uint32(0x7FEB352D)
    h = h ^ (h >> np.uint32(15))
    h = h * np.uint32(0x846CA68B)
    return h ^ (h >> np.uint32(16))


_C = [0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D, 0x27D4EB2F, 0x165667B1, 0xD3A2646D, 0xFD7046C5,
      0xB55A4F09, 0x2545F491, 0x9E3779B9]


def kx_hash(words):
    """oo_rx_device.h kx_hash over ten uint32 arrays (la[4], ra[4], ports, pw):
    each word folded (w ^ w >> 16), weighted, summed, mixed."""
    with np.errstate(over="ignore"):
        acc = np.zeros(np.broadcast(*words).shape, dtype=np.uint32)
        for w, c in zip(words, _C):
            w = np.asarray(w, dtype=np.uint32)
            acc = acc + (w ^ (w >> np.uint32(16))) * np.uint32(c)
        return _mix(acc)


def _le(b: bytes) -> int:
    return int.from_bytes(b, "little")


def colliding_v4(n, lport0=20000, nports=256):
    """n UDP (laddr, lport) keys of 10.0.x.y in one IPv4 bucket."""
    la = (np.arange(1 << 16, dtype=np.uint32) << np.uint32(16)) | np.uint32(10)  # 10.0.hi.lo
    ports = np.array([htons(lport0 + k) for k in range(nports)], dtype=np.uint32)
    z = np.uint32(0)
    b = kx_hash([la[:, None], z, z, z, z, z, z, z, ports[None, :], z]) & np.uint32(NB4 - 1)
    target = np.bincount(b.ravel(), minlength=NB4).argmax()
    ia, ip_ = np.nonzero(b == target)
    assert len(ia) >= n, len(ia)
    return [(int(la[i]).to_bytes(4, "little"), lport0 + int(p)) for i, p in zip(ia[:n], ip_[:n])]


def colliding_v6(n, lport=21000):
    """n IPv6 UDP wildcard keys (fd00::x:y, lport) in one IPv6 index entry run."""
    lo = np.arange(1 << 23, dtype=np.uint32)
    base = L6A[:12]
    w = [np.uint32(_le(base[4 * i:4 * i + 4])) for i in range(3)]
    la3 = lo.byteswap()  # the last word as the frame holds it (network order)
    z = np.uint32(0)
    b = kx_hash([w[0], w[1], w[2], la3, z, z, z, z, np.uint32(htons(lport)),
                 np.uint32(17 | 0x100)]) & np.uint32(NE6 - 1)
    target = np.bincount(b, minlength=NE6).argmax()
    idx = np.nonzero(b == target)[0]
    assert len(idx) >= n, len(idx)
    return [base + int(lo[i]).to_bytes(4, "big") for i in idx[:n]]


def _pair(**kw):
    return GpuRxStack(device=0, **kw), OracleStack(**kw)


def _check(g, o, buf, desc):
    got, ctr = run_dev(g, buf, desc)
    want = o.handle_rx_batch(buf, desc, nthreads=NTHREADS)
    assert got.tobytes() == want.tobytes(), diff_report(got, want, desc)
    np.testing.assert_array_equal(ctr, counters_of(want))
    return got


def _u4(dst, dport, src=PEER4, sport=40001, pay=b"x" * 18):
    return eth(ipv4(src, dst, 17, udp(4, src, dst, sport, dport, pay)), 0x0800)


def _u6(dst, dport, src=PEER6, sport=40001, pay=b"y" * 18):
    return eth(ipv6(src, dst, 17, udp(6, src, dst, sport, dport, pay)), 0x86DD)


def _t4(dst, dport, src=PEER4, sport=40001):
    return eth(ipv4(src, dst, 6, tcp(4, src, dst, sport, dport, b"z" * 10)), 0x0800)


def _world_frames(keys4, keys6):
    """Frames to every key (installed or not: the keys past the installed
    ones miss after scanning the full buckets of their own), a TCP listener's
    and a connected socket's traffic, in mixed order."""
    fr = []
    for la, lp in keys4:
        fr.append(_u4(la, lp))
        fr.append(_u4(la, lp, sport=50000 + lp % 97))
    for la6 in keys6:
        fr.append(_u6(la6, 21000))
    fr.append(_t4(L4A, 80))
    fr.append(_t4(L4A, 80, sport=40000))
    rng = np.random.default_rng(5)
    return [(fr[i], 0) for i in rng.permutation(len(fr))]


def _install_keys(stacks, keys4, keys6, first_id=100):
    sid = first_id
    for la, lp in keys4:
        for s in stacks:
            assert s.sock_set(sid, _sock(17, lp)) == 0
            assert s.filter_insert(sid, 4, la, lp, None, 0, 17) == 0
        sid += 1
    for la6 in keys6:
        for s in stacks:
            assert s.sock_set(sid, _sock(17, 21000)) == 0
            assert s.filter_insert(sid, 6, la6, 21000, None, 0, 17) == 0
        sid += 1
    for s in stacks:  # a listener and a connected socket on port 80
        assert s.sock_set(sid, _sock(6, 80)) == 0
        assert s.filter_insert(sid, 4, L4A, 80, None, 0, 6) == 0
        assert s.sock_set(sid + 1, _sock(6, 80, PEER4, 40000, flags=_abi.SOCK_CONNECTED)) == 0
        assert s.filter_insert(sid + 1, 4, L4A, 80, PEER4, 40000, 6) == 0


@pytest.mark.parametrize("kernel", ["0", "1", "2", "3"])
def test_keys_past_full_buckets(cuda, kernel, monkeypatch):
    """40 IPv4 keys in one bucket (20 full buckets to pass), 40 IPv6 keys in
    one entry run, 8 more of each that miss after scanning them, IPv4 and
    IPv6 lanes in one wave."""
    if kernel != "0":
        monkeypatch.setenv("OO_RX_KERNEL", kernel)
    keys4, keys6 = colliding_v4(48), colliding_v6(48)
    g, o = _pair()
    _install_keys((g, o), keys4[:40], keys6[:40])
    buf, desc = pack(_world_frames(keys4, keys6))
    got = _check(g, o, buf, desc)
    assert (got["reason"] == _abi.R_DELIVER).sum() >= 2 * 40 + 40
    g.close()


def test_overflow_turns_the_index_off(cuda):
    """More keys in one bucket than the overflow room holds: the index is
    turned off and every lookup walks (same records)."""
    keys4 = colliding_v4(200)
    g, o = _pair()
    _install_keys((g, o), keys4, [])
    buf, desc = pack(_world_frames(keys4, []))
    assert len(desc) > 400
    _check(g, o, buf, desc)
    # removing most of them brings the index back (rebuilt at the change)
    for i, (la, lp) in enumerate(keys4[20:]):
        for s in (g, o):
            s.filter_remove(120 + i, 4, la, lp, None, 0, 17)
    _check(g, o, buf, desc)
    g.close()


def test_socket_fields_changed_under_a_filter(cuda):
    """A socket connected after its filter went in (its entry stays where the
    old tuple hashed): the index turns off, the walks give the reference's
    answer; re-inserting the filter restores it."""
    g, o = _pair()
    install(g, edge_world())
    install(o, edge_world())
    frames = [(_u4(L4A, 5001), 0), (_u4(L4A, 5001, sport=7002), 0), (_u4(L4A, 5003), 0)]
    buf, desc = pack(frames + [(f, i) for f, i in edge_frames()[:64]])
    _check(g, o, buf, desc)
    for s in (g, o):
        assert s.sock_set(1, _sock(17, 5001, PEER4, 40001, flags=_abi.SOCK_CONNECTED)) == 0
    _check(g, o, buf, desc)
    for s in (g, o):
        s.filter_remove(1, 4, L4A, 5001, None, 0, 17)
        assert s.filter_insert(1, 4, L4A, 5001, PEER4, 40001, 17) == 0
    _check(g, o, buf, desc)
    g.close()


@pytest.mark.parametrize("kernel", ["1", "2", "3"])
def test_walks_alone(cuda, kernel, monkeypatch):
    """Tuning `walks`: no key index, every lookup walks the tables."""
    monkeypatch.setenv("OO_RX_KERNEL", kernel)
    monkeypatch.setenv("OO_RX_WALKS", "1")
    g, o = _pair(intf_hwport=HWPORTS)
    install(g, edge_world())
    install(o, edge_world())
    for shift in (0, 3):
        buf, desc = pack(edge_frames(), align=64 if shift % 2 == 0 else 16, shift=shift)
        _check(g, o, buf, desc)
    g.close()
    for config, n in ((3, 1 << 16), (4, 1 << 14), (5, 1 << 16)):
        filters, socks = pktgen.world(config)
        g, o = _pair()
        g.load_world(filters, socks)
        o.load_world(filters, socks)
        buf, desc = pktgen.generate(config, n, first=4242 * config, nthreads=NTHREADS)
        _check(g, o, buf, desc)
        g.close()


def _churn_ops(stacks, filters, idx, remove):
    for i in idx:
        f = filters[i]
        n = 4 if f.af == 4 else 16
        ra = None if f.raddr_any else bytes(f.raddr)[:n]
        for s in stacks:
            fn = s.filter_remove_raw if remove else s.filter_insert_raw
            rc = fn(f.sock, f.af, bytes(f.laddr)[:n], f.lport_be, ra, f.rport_be, f.proto)
            assert rc == 0 or remove, rc


@pytest.mark.parametrize("kernel", ["0", "3"])
def test_incremental_index_under_churn(cuda, kernel, monkeypatch):
    """Small flushes of filter removes and re-inserts (no socket change)
    update the index for the flushed keys only (oo_gpu_rx_get_table_stats:
    index_updates, no rebuild): keys that lost their last match stay as dead
    entries that walk, re-inserted keys take their new first slot, and the
    records equal the oracle's walks after every flush -- IPv4 and IPv6, TCP
    and UDP (config 5's world), and keys in one full IPv4 bucket."""
    if kernel != "0":
        monkeypatch.setenv("OO_RX_KERNEL", kernel)
    filters, socks = pktgen.world(5)
    g, o = _pair()
    g.load_world(filters, socks)
    o.load_world(filters, socks)
    keys4 = colliding_v4(40)
    _install_keys((g, o), keys4, [], first_id=6000)
    buf, desc = pktgen.generate(5, 1 << 15, first=777, nthreads=NTHREADS)
    kbuf, kdesc = pack(_world_frames(keys4, []))
    _check(g, o, buf, desc)
    st0 = g.table_stats()
    assert st0["index_on"] == 1
    rng = np.random.default_rng(9)
    removed = set()
    for r in range(6):
        out = rng.choice(len(filters), 60, replace=False)
        out = [i for i in out if i not in removed]
        _churn_ops((g, o), filters, out, remove=True)
        removed.update(out)
        back = rng.choice(sorted(removed), min(len(removed), 40), replace=False)
        _churn_ops((g, o), filters, back, remove=False)
        removed.difference_update(back)
        # keys of the full bucket: some go, some come back
        for j, (la, lp) in enumerate(keys4):
            if (j + r) % 3 == 0:
                for s in (g, o):
                    s.filter_remove(6000 + j, 4, la, lp, None, 0, 17)
            elif (j + r) % 3 == 1:
                for s in (g, o):
                    s.filter_remove(6000 + j, 4, la, lp, None, 0, 17)
                    assert s.filter_insert(6000 + j, 4, la, lp, None, 0, 17) == 0
        _check(g, o, buf, desc)
        _check(g, o, kbuf, kdesc)
    st = g.table_stats()
    assert st["index_updates"] - st0["index_updates"] >= 6, st  # (a flush a round)
    assert st["index_rebuilds"] == st0["index_rebuilds"], st
    assert st["index_on"] == 1
    g.close()


def test_incremental_index_falls_back_to_rebuild(cuda):
    """A socket change in a flush, or an op whose tuple is not its socket's,
    rebuilds the index.  An index that is off (a socket connected under its
    filter: a PREFERRED entry its key no longer hashes to) cannot be updated:
    the next filter-only flush finds it off and asks for a rebuild, which the
    flush after it does; fixing the filter brings the index back."""
    g, o = _pair()
    install(g, edge_world())
    install(o, edge_world())
    for s in (g, o):
        assert s.sock_set(7000, _sock(17, 6001)) == 0
    frames = [(_u4(L4A, 5001), 0), (_u4(L4A, 5001, sport=7002), 0), (_u4(L4A, 6001), 0)]
    buf, desc = pack(frames + [(f, i) for f, i in edge_frames()[:96]])
    _check(g, o, buf, desc)

    def step(expect, on):
        before = g.table_stats()
        _check(g, o, buf, desc)
        st = g.table_stats()
        got = "rebuild" if st["index_rebuilds"] > before["index_rebuilds"] else \
            "update" if st["index_updates"] > before["index_updates"] else "none"
        assert (got, st["index_on"]) == (expect, on), (before, st)

    for s in (g, o):  # a socket change: rebuild
        assert s.sock_set(1, _sock(17, 5001)) == 0
    step("rebuild", 1)
    for s in (g, o):  # a filter op of a consistent socket: update
        assert s.filter_insert(7000, 4, L4A, 6001, None, 0, 17) == 0
    step("update", 1)
    for s in (g, o):  # socket 1 connected under its filter: rebuild, off
        assert s.sock_set(1, _sock(17, 5001, PEER4, 40001, flags=_abi.SOCK_CONNECTED)) == 0
    step("rebuild", 0)
    for s in (g, o):  # filter-only flush: finds the index off, asks for a rebuild
        assert s.filter_remove(7000, 4, L4A, 6001, None, 0, 17) == 0
    step("update", 0)
    # no table change: the requested rebuild runs before the next batch all
    # the same (still off: socket 1's entry is misplaced) -- ADVICE r5
    step("rebuild", 0)
    step("none", 0)
    for s in (g, o):  # a filter-only flush finds it off again and asks
        assert s.filter_insert(7000, 4, L4A, 6001, None, 0, 17) == 0
    step("update", 0)
    for s in (g, o):  # socket 1's filter re-inserted under its tuple: rebuild, on
        s.filter_remove(1, 4, L4A, 5001, None, 0, 17)
        assert s.filter_insert(1, 4, L4A, 5001, PEER4, 40001, 17) == 0
    step("rebuild", 1)
    for s in (g, o):
        assert s.filter_remove(7000, 4, L4A, 6001, None, 0, 17) == 0
    step("update", 1)
    g.close()


def test_index_rebuilt_after_many_incremental_updates(cuda):
    """Incremental updates leave KX_DEAD entries behind (a key that lost its
    last match walks); after 256 of them in a row the index is rebuilt from
    the tables before the next batch, table ops queued or not (oo_gpu_rx.cpp
    kKxIncMax), once.  Records equal the oracle's throughout."""
    g, o = _pair()
    install(g, edge_world())
    install(o, edge_world())
    frames = [(_u4(L4A, 5001), 0), (_u4(L4A, 6001), 0)]
    buf, desc = pack(frames + [(f, i) for f, i in edge_frames()[:30]])
    for s in (g, o):
        assert s.sock_set(7000, _sock(17, 6001)) == 0
    _check(g, o, buf, desc)  # (the socket change: a rebuild)
    st0 = g.table_stats()
    for k in range(256):
        for s in (g, o):
            if k % 2 == 0:
                assert s.filter_insert(7000, 4, L4A, 6001, None, 0, 17) == 0
            else:
                assert s.filter_remove(7000, 4, L4A, 6001, None, 0, 17) == 0
        if k % 64 == 63:
            _check(g, o, buf, desc)
        else:
            g.sync()
    st = g.table_stats()
    assert st["index_updates"] - st0["index_updates"] == 256, (st0, st)
    assert st["index_rebuilds"] == st0["index_rebuilds"] and st["index_on"] == 1
    _check(g, o, buf, desc)  # nothing queued, but the rebuild is due: it runs first
    st = g.table_stats()
    assert st["index_rebuilds"] == st0["index_rebuilds"] + 1 and st["index_on"] == 1, (st0, st)
    _check(g, o, buf, desc)  # and only once
    assert g.table_stats()["index_rebuilds"] == st["index_rebuilds"]
    for s in (g, o):
        assert s.filter_remove(7000, 4, L4A, 6001, None, 0, 17) == 0
    _check(g, o, buf, desc)
    assert g.table_stats()["index_updates"] == st["index_updates"] + 1  # updates again
    g.close()
