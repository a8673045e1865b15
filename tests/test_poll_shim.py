# SPDX-License-Identifier: BSD-2-Clause
"""The batched RX branch (include/oo_rx_poll.h) without a GPU: the shim
library loads against liboo_gpu_rx.so and exports what its header declares;
events the transform does not take are classified, counted and dispatched
as the reference loop does (tests/poll_util.py); and a batch the device
cannot run (host-only context: -ENODEV) runs no callback and adds no
counter, so the caller still owns every event."""
import ctypes
import os
import re

import numpy as np
import pytest

from onload_amd import poll
from onload_amd.rx import GpuRxStack
from poll_util import Recorder, events_for, expect, onload_stats, transformed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_every_declared_symbol():
    lib = poll.load_poll()
    hdr = open(os.path.join(ROOT, "include", "oo_rx_poll.h")).read()
    names = set(re.findall(r"\b(oo_rx_poll_\w+)\s*\(", hdr))
    assert names == set(poll.POLL_SYMBOLS)
    for n in names:
        assert hasattr(lib, n)


def test_layouts_match_header():
    assert ctypes.sizeof(poll.Stats) == 8 * len(poll.STAT_NAMES) == 200
    assert ctypes.sizeof(poll.Ops) == 6 * 8
    assert ctypes.sizeof(poll.PollCfg) == 56
    assert poll.EV_DTYPE.itemsize == 16 and ctypes.sizeof(poll.Future) == 24


def test_open_rejects_bad_cfg():
    st = GpuRxStack(device=-1)
    pool = np.zeros(4096, np.uint8)
    for bs, n in ((3000, 64), (2048, 0), (2048, poll.MAX_EVS + 1)):
        with pytest.raises(OSError):
            poll.RxPoll(st, pool, bs, n, True, Recorder())
    st.close()


def _untransformed_events(rng, n=400, bs=2048):
    frames = [(bytes(rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8)), 0)
              for _ in range(n)]
    pool, evs = events_for(frames, bs, rng)
    # keep only events the transform would not take
    keep = [not transformed(e, True, bs, pool.nbytes) for e in evs]
    return pool, evs[np.array(keep)]


def test_untransformed_events_follow_the_loop():
    rng = np.random.default_rng(7)
    pool, evs = _untransformed_events(rng)
    assert len(evs) > 50
    st = GpuRxStack(device=-1)
    rec = Recorder()
    p = poll.RxPoll(st, pool, 2048, 64, True, rec)
    assert p.poll(evs) == len(evs)
    calls, want = expect(evs, [], pool, 2048, True, lambda i: False, None)
    assert rec.calls == calls
    assert onload_stats(p.stats.as_dict()) == want
    assert p.stats.n_batches == 0
    p.close()
    st.close()


def test_device_failure_runs_no_callback():
    rng = np.random.default_rng(8)
    frames = [(bytes(64), 0)] * 10
    pool, evs = events_for(frames, 2048, rng, discard_mix=False)
    st = GpuRxStack(device=-1)
    rec = Recorder()
    p = poll.RxPoll(st, pool, 2048, 4, True, rec)
    assert p.poll(evs) == -19  # -ENODEV: the first batch could not run
    assert rec.calls == [] and p.stats.as_dict() == {k: 0 for k in poll.STAT_NAMES}
    # with sw_verify off the same plain events are the loop's own business
    q = poll.RxPoll(st, pool, 2048, 4, False, rec)
    assert q.poll(evs) == len(evs)
    # ... and their rx_evs is the loop's to count (not twice)
    assert rec.calls == [("other", i) for i in range(10)] and q.stats.rx_evs == 0
    p.close()
    q.close()
    st.close()


def test_failure_after_a_handled_chunk_returns_the_handled_count():
    """Chunks of 4: the first holds only events the transform does not take
    (its callbacks run, its counters land), the second needs the device,
    which fails: the call returns 4 and the caller still owns events 4.."""
    rng = np.random.default_rng(9)
    pool, evs = events_for([(bytes(80), 0)] * 8, 2048, rng, discard_mix=False)
    evs["flags"][:4] = poll.EV_SOP | poll.EV_CONT  # multi-buffer: the loop's own
    evs["discard"][2] = poll.DISCARD_ETH_FCS_ERR    # a discard outside the csum class
    st = GpuRxStack(device=-1)
    rec = Recorder()
    p = poll.RxPoll(st, pool, 2048, 4, True, rec)
    assert p.poll(evs) == 4
    assert rec.calls == [("other", 0), ("other", 1), ("release", 2, None), ("other", 3)]
    d = p.stats.as_dict()
    assert d["rx_discard_crc_bad"] == 1 and d["n_other"] == 3 and d["rx_evs"] == 0
    p.close()
    st.close()


def test_frame_past_its_buffer_is_not_taken():
    """an event whose frame runs past the end of its buffer (ofs +
    len > buf_size) is not the shim's: a plain event goes back to the loop,
    a checksum-class discard is released -- never copied into a gather slot."""
    pool = np.zeros(8 * 2048, np.uint8)
    evs = np.zeros(3, poll.EV_DTYPE)
    evs[0] = (0, 1000, 1100, poll.EV_SOP, 0, 0, 0)                          # 2100 > 2048
    evs[1] = (1, 2047, 2, poll.EV_SOP, poll.DISCARD_L4_CSUM_ERR, 0, 0)     # 2049 > 2048
    evs[2] = (2, 192, 1856, poll.EV_SOP, 0, 0, 0)                           # 2048: fits
    st = GpuRxStack(device=-1)
    rec = Recorder()
    p = poll.RxPoll(st, pool, 2048, 64, True, rec)
    # event 2 fits its buffer exactly and needs the device: the host-only
    # context fails that batch, so only a call over the first two completes
    assert p.poll(evs[:2]) == 2
    assert rec.calls == [("other", 0), ("release", 1, None)]
    assert p.poll(evs[2:]) == -19
    p.close()
    st.close()


@pytest.mark.skipif(not os.path.exists("/root/reference/src/lib/transport/ip/netif_event.c"),
                    reason="the reference tree is only in the build container")
def test_integration_compiles_against_reference():
    """integration/netif_event_gpu.c binds the callback table to the real
    post-future helpers, handlers and stats of the reference tree: it must
    compile there warning-free (check-only, not shipped)."""
    import subprocess
    r = subprocess.run(["make", "-C", ROOT, "check-integration"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
