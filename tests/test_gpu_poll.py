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
                                                         (1, 1, 4)])
def test_poll_dispatch_and_counters(cuda, sw_verify, evs_per_poll, seed):
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
    pool = np.zeros(4 * 2048, np.uint8)
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
