# SPDX-License-Identifier: BSD-2-Clause
"""The batched ci_netif_poll_evq RX branch (src/shim/oo_rx_poll.c) on the
GPU, driven with a fake callback table (tests/poll_util.py Recorder) over the
edge corpus: for every event, the dispatch decision (release / handle_rx_pkt
/ post-future with the future's fields / full handler / the loop's own
branch), the record each callback receives (bit-exact with the oracle) and
the counter deltas, against the restatement of netif_event.c:1709-1742,
:1131-1191, :1014-1128, tcp_rx.c:4814-4835 and the future helpers in
poll_util.expect."""
import numpy as np
import pytest

from frames import edge_frames, edge_world, install, pack
from hostmem import page_buffer
from onload_amd import _abi, poll
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack
from poll_util import Recorder, events_for, expect, onload_stats, transformed

pytestmark = pytest.mark.gpu

HWPORTS = (0, 1, 3, 2, 5)
BUF = 16384  # jumbo frames of the corpus fit one buffer


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _oracle_records(frames, evs, pool, sw_verify):
    """The oracle's records of the events the transform takes, in order, and
    the oracle (its tables hold the edge world)."""
    sel = [(frames[int(e["rq_id"])][0], int(e["intf_i"])) for e in evs
           if transformed(e, sw_verify, BUF, pool.nbytes)]
    o = OracleStack(intf_hwport=HWPORTS)
    install(o, edge_world())
    if not sel:
        return np.zeros(0, _abi.RESULT_DTYPE), o
    buf, desc = pack(sel)
    return o.handle_rx_batch(buf, desc), o


@pytest.mark.parametrize("sw_verify,evs_per_poll,seed", [(1, 64, 1), (1, 1000, 2), (0, 64, 3),
                                                         (1, 1, 4), (1, 200, 5)])
def test_poll_dispatch_and_counters(cuda, sw_verify, evs_per_poll, seed):
    # (chunks of 64 and 200: 8-packet tiles -- the poll instance in a library
    # built with it; 1000: rx_kernel's 64-packet tiles)
    rng = np.random.default_rng(seed)
    frames = edge_frames(seed=seed)
    if evs_per_poll == 1:
        frames = frames[:200]
    pool, evs = events_for(frames, BUF, rng)
    # a recvq that is full for some sockets' packets: the future is declined
    decline = lambda i: i % 7 == 3  # noqa: E731
    g = GpuRxStack(device=0, intf_hwport=HWPORTS, host_stage_bytes=64 << 20,
                   host_stage_pkts=65536)
    install(g, edge_world())
    rec = Recorder(decline)
    p = poll.RxPoll(g, pool, BUF, evs_per_poll, bool(sw_verify), rec)
    assert p.poll(evs) == len(evs)
    want_recs, o = _oracle_records(frames, evs, pool, sw_verify)
    calls, want = expect(evs, want_recs, pool, BUF, sw_verify, decline, o)
    # the records the callbacks saw are the oracle's, bit for bit
    got = np.array([tuple(r[k] for k in _abi.RESULT_DTYPE.names) for r in rec.recs],
                   dtype=_abi.RESULT_DTYPE)
    assert got.tobytes() == want_recs.tobytes()
    assert len(rec.calls) == len(calls)
    for k, (a, b) in enumerate(zip(rec.calls, calls)):
        assert a == b, (k, a, b)
    st = p.stats.as_dict()
    assert onload_stats(st) == want
    if evs_per_poll <= 256 and st["n_batches"]:  # a poll's batch: the poll instance
        assert g.last_path() == 5
    ntrans = len(want_recs)
    assert st["n_batches"] == (0 if ntrans == 0 else
                               sum(1 for s in range(0, len(evs), evs_per_poll)
                                   if any(transformed(e, sw_verify, BUF, pool.nbytes)
                                          for e in evs[s:s + evs_per_poll])))
    # every edge-corpus outcome reached the shim (sw_verify: all of them)
    if sw_verify and evs_per_poll == 64:
        kinds = {c[0] for c in calls}
        assert kinds == {"release", "pkt", "future", "declined", "full", "other"}
        assert set(want_recs["reason"]) >= {0, 1, 2, 3, 4, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25}
    p.close()
    g.close()


def test_poll_stage_routing(cuda):
    """TCP decided in stage 2 or 3 and IPv6 go to the full handler; TCP
    stage 1 and single-match IPv4 UDP go through the future (tcp_rx.c:
    4814-4835, tcp_rx.h:150-214, udp_internal.h:41-134)."""
    import cases
    socks, filters = cases.order_world()
    g = GpuRxStack(device=0, host_stage_bytes=1 << 20, host_stage_pkts=1024)
    install(g, (socks, filters))
    f = cases.order_frame()
    pool = page_buffer(4 * 2048)
    pool[192:192 + len(f)] = np.frombuffer(f, np.uint8)
    ev = np.zeros(1, poll.EV_DTYPE)
    ev[0] = (0, 192, len(f), poll.EV_SOP, 0, 0, 0)
    seen = []
    for stage in (1, 2, 3):
        rec = Recorder()
        p = poll.RxPoll(g, pool, 2048, 64, True, rec)
        assert p.poll(ev) == 1
        seen.append(rec.calls[0][0])
        assert rec.recs[0]["stage"] == stage
        if stage == 1:
            assert rec.calls[0][3] == rec.recs[0]["hash3"]  # rxp.hash
            assert p.stats.tcp_in_segs == 1
        else:
            assert p.stats.tcp_in_segs == 0  # ci_tcp_handle_rx counts it itself
        p.close()
        g.filter_remove(*filters[stage - 1])
    assert seen == ["future", "full", "full"]
    g.close()


# The per-record counters the shim keeps (src/shim/oo_rx_poll.c count_drop /
# dispatch) -> the reference counter whose per-frame changes they replace.
SHIM_DROP = {"in_hdr_errs": "ip.in_hdr_errs", "in6_hdr_errs": "ip.in6_hdr_errs",
             "udp_in_errs": "udp.udp_in_errs"}
SHIM_HANDLED = {"in_recvs": "ip.in_recvs", "in_delivers": "ip.in_delivers",
                "in6_recvs": "ip.in6_recvs", "in6_delivers": "ip.in6_delivers",
                "ip_options": "ni.ip_options"}
SHIM_FUTURE = {"tcp_in_segs": "tcp.tcp_in_segs", "udp_in_dgrams": "udp.udp_in_dgrams"}


@pytest.mark.parametrize("name", ("edge", "edge99", "c2", "c4", "c5"))
def test_poll_counters_match_reference_run(cuda, name):
    """The shim's per-record stack counters against the reference's own run
    of the same frames (tests/golden/ref_l4_golden.npz: every counter
    handle_rx_csum_bad, handle_rx_pkt and the handlers changed, per frame):
    the drop counters over the dropped frames, handle_rx_pkt's over the
    frames an L4 handler took (the slow-path ones go to ops->pkt_handler,
    which is handle_rx_pkt and counts for itself), the handlers' in_segs /
    in_dgrams over the frames whose future resolved (the post-future helpers
    count them, tcp_rx.h:182, udp_internal.h:99; the full handlers count
    the rest themselves).  rx_evs / rx_discard_* / rx_sw_csum_pass belong to
    the poll loop around handle_rx_csum_bad (netif_event.c:1164-1191,
    :1718), which the harness does not run: test_poll_dispatch_and_counters
    checks them."""
    import l4_ref
    from test_oracle_l4_ref import GOLDEN
    golden = np.load(GOLDEN)
    out, sha = l4_ref.load(golden, name)
    obs, stats = l4_ref.load_stats(golden, name)
    socks, filters, hwports, frames = l4_ref.corpus(name)
    assert l4_ref.frames_sha(frames) == sha
    g = GpuRxStack(device=0, intf_hwport=hwports, host_stage_bytes=64 << 20,
                   host_stage_pkts=65536)
    for i, s in socks.items():
        assert g.sock_set(i, s) == 0
    for (i, af, la, lp, ra, rp, proto) in filters:
        assert g.filter_insert_raw(i, af, la, lp, ra, rp, proto) == 0
    pool, evs = events_for(frames, BUF, np.random.default_rng(5), discard_mix=False)
    rec = Recorder()
    p = poll.RxPoll(g, pool, BUF, 64, True, rec)
    assert p.poll(evs) == len(evs)
    st = p.stats.as_dict()
    c = {k: out[:, i] for i, k in enumerate(l4_ref.COLS)}
    dropped = c["handled"] == 0
    took = (c["handled"] == 1) & (c["entry"] != 0)
    fut = took & (c["fut"] >= 0)
    want = {}
    for k, ref in SHIM_DROP.items():
        want[k] = sum(stats[i].get(ref, 0) for i in np.flatnonzero(dropped))
    for k, ref in SHIM_HANDLED.items():
        want[k] = sum(stats[i].get(ref, 0) for i in np.flatnonzero(took))
    for k, ref in SHIM_FUTURE.items():
        want[k] = sum(stats[i].get(ref, 0) for i in np.flatnonzero(fut))
    got = {k: st[k] for k in want}
    assert got == want
    assert st["n_future"] == int(fut.sum())
    assert st["n_pkt_handler"] == int(((c["handled"] == 1) & (c["entry"] == 0)).sum())
    p.close()
    g.close()


@pytest.mark.parametrize("evs_per_poll", (16, 64))
def test_poll_table_change_in_a_callback(cuda, evs_per_poll):
    """A callback that changes the tables (a filter removed as its socket
    closes, next to ci_netif_filter_remove) while the rest of its chunk and
    the next chunk are already transformed: the packets after it see the new
    tables, as the reference's one-event-at-a-time loop would --
    the shim transforms both again."""
    import cases
    socks, filters = cases.order_world()
    g = GpuRxStack(device=0, host_stage_bytes=16 << 20, host_stage_pkts=4096)
    install(g, (socks, filters))
    f = cases.order_frame()
    n = 4 * evs_per_poll
    pool = page_buffer(n * 2048)
    evs = np.zeros(n, poll.EV_DTYPE)
    for i in range(n):
        pool[i * 2048 + 192:i * 2048 + 192 + len(f)] = np.frombuffer(f, np.uint8)
        evs[i] = (i, 192, len(f), poll.EV_SOP, 0, 0, 0)
    cut = evs_per_poll + 3  # inside the second chunk: the third is in flight

    class Closer(Recorder):
        def post_future(self, i, r, fu):
            if i == cut:
                assert g.filter_remove(*filters[0]) == 0  # stage 1's socket closes
            return super().post_future(i, r, fu)

        def full_handler(self, i, r):
            if i == cut:
                assert g.filter_remove(*filters[0]) == 0
            super().full_handler(i, r)

    rec = Closer()
    p = poll.RxPoll(g, pool, 2048, evs_per_poll, True, rec)
    assert p.poll(evs) == n
    stages = [int(r["stage"]) for r in rec.recs]
    assert stages == [1] * (cut + 1) + [2] * (n - cut - 1)
    assert p.stats.n_resubmit == 2  # the chunk's rest, then the next chunk
    assert p.stats.n_batches == n // evs_per_poll + 1  # + the rest (the next chunk: replaced)
    p.close()
    g.close()


@pytest.mark.parametrize("zero_copy", (False, True))
def test_poll_crossover(cuda, zero_copy):
    """OO_RX_POLL_CROSSOVER (oo_rx_poll.c gpu_pays): a chunk the cost model
    prices below the device batch goes back whole, in order, through
    other_ev (the call site runs it through the per-event loop), counted only
    in n_handback and n_other (every event other_ev receives); a chunk it
    prices above runs exactly as without the flag.
    Chunks of one poll are priced one by one: with evs_per_poll 64 and a
    model whose fixed cost 40 frames of the corpus repay, the short last
    chunk goes back and the full ones do not."""
    rng = np.random.default_rng(11)
    frames = edge_frames(seed=11)
    pool, evs = events_for(frames, BUF, rng)
    n = len(evs)

    def run(crossover, epp=64):
        g = GpuRxStack(device=0, intf_hwport=HWPORTS, host_stage_bytes=64 << 20,
                       host_stage_pkts=65536)
        install(g, edge_world())
        rec = Recorder()
        p = poll.RxPoll(g, pool, BUF, epp, True, rec, zero_copy=zero_copy, crossover=crossover)
        assert p.zero_copy == zero_copy
        assert p.poll(evs) == n
        st = p.stats.as_dict()
        p.close()
        g.close()
        return rec, st

    base_rec, base_st = run(None)
    # never pays: everything handed back, nothing else counted
    rec, st = run({"gpu_fixed_ns": 1 << 30})
    assert rec.calls == [("other", int(e["rq_id"])) for e in evs]
    assert st["n_handback"] == n and st["n_other"] == n and st["n_batches"] == 0
    assert all(v == 0 for k, v in st.items() if k not in ("n_handback", "n_other")), st
    # always pays: the same calls, records and counters as without the flag
    rec, st = run({"cpu_pkt_ps": 1 << 30})
    assert rec.calls == base_rec.calls
    assert [r.tobytes() if hasattr(r, "tobytes") else r for r in rec.recs] == \
        [r.tobytes() if hasattr(r, "tobytes") else r for r in base_rec.recs]
    assert st == base_st
    # per chunk: fixed = 40 frames' worth of the CPU's per-frame saving (the
    # per-byte terms 1 ps each: 0 would take the defaults)
    per = {"cpu_pkt_ps": 20000, "cpu_byte_ps": 1, "gpu_pkt_ps": 10000, "gpu_byte_ps": 1,
           "gpu_fixed_ns": 400}
    rec, st = run(per)
    cut = (n // 64) * 64
    if n - cut < 40:
        tail = [("other", int(e["rq_id"])) for e in evs[cut:]]
        assert rec.calls[len(rec.calls) - len(tail):] == tail
        assert st["n_handback"] == n - cut
    assert st["n_batches"] >= (cut // 64) - 1


def test_poll_table_change_then_rest_handed_back(cuda):
    """A callback changes the tables mid-chunk with OO_RX_POLL_CROSSOVER set,
    and the model prices the re-transformed rest of the chunk below the
    device batch: the rest goes to other_ev, and none of it is counted by
    the shim -- rx_evs and the discard class counters hold only
    the events the shim itself handled."""
    import cases
    socks, filters = cases.order_world()
    g = GpuRxStack(device=0, host_stage_bytes=16 << 20, host_stage_pkts=4096)
    install(g, (socks, filters))
    f = cases.order_frame()
    epp = 64
    n = 3 * epp
    pool = page_buffer(n * 2048)
    evs = np.zeros(n, poll.EV_DTYPE)
    for i in range(n):
        pool[i * 2048 + 192:i * 2048 + 192 + len(f)] = np.frombuffer(f, np.uint8)
        # every 5th event a bad-FCS discard: released, counted in its class
        evs[i] = (i, 192, len(f), poll.EV_SOP, poll.DISCARD_ETH_FCS_ERR if i % 5 == 4 else 0, 0, 0)
    cut = 30  # the rest of chunk 0 (33 events) is re-priced and loses
    removed = []

    class Closer(Recorder):
        def post_future(self, i, r, fu):
            if i == cut and not removed:
                removed.append(g.filter_remove(*filters[0]))
            return super().post_future(i, r, fu)

        def full_handler(self, i, r):
            if i == cut and not removed:
                removed.append(g.filter_remove(*filters[0]))
            super().full_handler(i, r)

    # per chunk: fixed = 40 frames' worth of the CPU's per-frame saving (the
    # per-byte terms 1 ps each: 0 would take the defaults)
    per = {"cpu_pkt_ps": 20000, "cpu_byte_ps": 1, "gpu_pkt_ps": 10000, "gpu_byte_ps": 1,
           "gpu_fixed_ns": 400}
    rec = Closer()
    p = poll.RxPoll(g, pool, 2048, epp, True, rec, crossover=per)
    assert p.poll(evs) == n
    assert removed == [0]
    st = p.stats.as_dict()
    rest = set(range(cut + 1, epp))
    assert [c for c in rec.calls if c[0] == "other"] == [("other", i) for i in sorted(rest)]
    assert st["n_handback"] == len(rest) and st["n_other"] == len(rest)
    fcs = [i for i in range(n) if i % 5 == 4]
    assert st["rx_discard_crc_bad"] == len([i for i in fcs if i not in rest])
    assert st["rx_evs"] == len([i for i in range(n) if i % 5 != 4 and i not in rest])
    p.close()
    g.close()


@pytest.mark.parametrize("zero_copy", (False, True))
def test_frames_flush_with_pool_page_ends(cuda, zero_copy):
    """Every frame ends at its 2048-B buffer's last byte -- every second one
    at a page's, the last at the registered pool's -- read in place (zero
    copy) or gathered: the shim's batches never read past a frame's lines,
    and the records the callbacks see are the oracle's."""
    frames = [(f, i) for f, i in edge_frames(seed=11) if 0 < len(f) <= 2048]
    frames = frames[:len(frames) & ~1]  # the pool whole pages (two buffers a page)
    n = len(frames)
    pool = page_buffer(n * 2048)
    evs = np.zeros(n, poll.EV_DTYPE)
    for i, (f, intf) in enumerate(frames):
        ofs = 2048 - len(f)
        pool[i * 2048 + ofs:(i + 1) * 2048] = np.frombuffer(f, np.uint8)
        evs[i] = (i, ofs, len(f), poll.EV_SOP, 0, intf, 0)
    g = GpuRxStack(device=0, intf_hwport=HWPORTS, host_stage_bytes=16 << 20,
                   host_stage_pkts=4096)
    install(g, edge_world())
    rec = Recorder(lambda i: False)
    p = poll.RxPoll(g, pool, 2048, 64, True, rec, zero_copy=zero_copy)
    assert p.zero_copy == zero_copy
    assert p.poll(evs) == n
    o = OracleStack(intf_hwport=HWPORTS)
    install(o, edge_world())
    sel = [frames[i] for i in range(n) if transformed(evs[i], True, 2048, pool.nbytes)]
    buf, desc = pack(sel)
    want = o.handle_rx_batch(buf, desc)
    got = np.array([tuple(r[k] for k in _abi.RESULT_DTYPE.names) for r in rec.recs],
                   dtype=_abi.RESULT_DTYPE)
    assert len(sel) > 100 and got.tobytes() == want.tobytes()
    p.close()
    g.close()
