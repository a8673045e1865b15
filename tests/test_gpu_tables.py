# SPDX-License-Identifier: BSD-2-Clause
"""Device-side filter-table maintenance: filter
inserts/removes and socket changes between batches are applied to the HBM
tables by the table_ops kernel on the batch stream (oo_table_kernel.hip), not
uploaded from the host.  After every script the device image equals, byte for
byte, the image of a host-only context fed the same calls (whose slots the
CPU tests pin to the oracle's restatement of netif_table.c), and the records
of every batch equal the oracle's -- including a batch still running on
another stream while the change is queued."""
import ctypes

import numpy as np
import pytest

from gpu_util import diff_report, to_dev
from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack, counters_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _device_image(torch, g, stream=None):
    img = torch.zeros(g.image_bytes(), dtype=torch.uint8, device="cuda")
    s = stream or torch.cuda.current_stream()
    g.table_export(img.data_ptr(), img.numel(), s.cuda_stream)
    torch.cuda.synchronize()
    return img.cpu().numpy()


def _copy_sock(s):
    c = _abi.Sock()
    ctypes.memmove(ctypes.byref(c), ctypes.byref(s), ctypes.sizeof(s))
    return c


def _raw(f):
    la = bytes(f.laddr)[: 4 if f.af == 4 else 16]
    ra = None if f.raddr_any else bytes(f.raddr)[: 4 if f.af == 4 else 16]
    return (f.sock, f.af, la, f.lport_be, ra, f.rport_be, f.proto)


def _script(rng, filters, socks, live, n_rm, n_add, n_sock):
    """Calls for one round: removes of live world filters, re-inserts of
    removed ones, socket changes (connect flag, bind2dev) and raw inserts of
    extra entries for spare socket ids (route counts, tombstones)."""
    calls = []
    live_idx = np.nonzero(live)[0]
    for i in rng.choice(live_idx, size=min(n_rm, len(live_idx)), replace=False):
        calls.append(("rm", _raw(filters[i])))
        live[i] = False
    dead = np.nonzero(~live)[0]
    for i in rng.choice(dead, size=min(n_add, len(dead)), replace=False):
        calls.append(("ins", _raw(filters[i])))
        live[i] = True
    for k in rng.choice(len(socks), size=n_sock, replace=False):
        s = _copy_sock(socks[k])
        if rng.random() < 0.5:
            s.flags |= _abi.SOCK_BIND2DEV
            s.bind2dev_hwports = int(rng.integers(0, 4))
            s.bind2dev_vlan = 0
        else:
            s.flags &= ~_abi.SOCK_BIND2DEV
        socks[k] = s
        calls.append(("sock", (int(k), s)))
    for j in range(n_add // 2):
        sid = 8000 + int(rng.integers(0, 190))
        la = bytes([10, 0, 0, 1])
        calls.append(("ins", (sid, 4, la, int(rng.integers(0, 65536)), None, 0, 17)))
    return calls


def _apply(stacks, calls):
    for kind, args in calls:
        rcs = set()
        for st in stacks:
            if kind == "ins":
                rcs.add(st.filter_insert_raw(*args))
            elif kind == "rm":
                rcs.add(st.filter_remove_raw(*args))
            else:
                rcs.add(st.sock_set(*args))
        assert len(rcs) == 1, (kind, args, rcs)


def test_device_tables_follow_ops_between_batches(cuda):
    torch = cuda
    filters, socks = pktgen.world(5)
    socks = list(socks)
    kw = dict(intf_hwport=(0, 1, 2, 3))
    g = GpuRxStack(device=0, **kw)
    h = GpuRxStack(device=-1, **kw)
    o = OracleStack(**kw)
    for st in (g, h, o):
        st.load_world(filters, socks)
    n = 1 << 16
    buf, desc = pktgen.generate(5, n, first=5151)
    desc["intf_i"] = np.arange(n) % 4
    fr, de = to_dev(buf), to_dev(desc)
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(_abi.R_COUNT, dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    rng = np.random.default_rng(2024)
    live = np.ones(len(filters), bool)
    for rnd in range(6):
        _apply((g, h, o), _script(rng, filters, socks, live, 400, 250, 60))
        s = streams[rnd % 2]
        ctr.zero_()
        torch.cuda.synchronize()
        g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, out.data_ptr(),
                              ctr.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
        want = o.handle_rx_batch(buf, desc, nthreads=8)
        assert got.tobytes() == want.tobytes(), f"round {rnd}: " + diff_report(got, want, desc)
        np.testing.assert_array_equal(ctr.cpu().numpy().astype(np.uint32), counters_of(want))
        img = _device_image(torch, g, streams[(rnd + 1) % 2])
        ref = h.image_host()
        bad = np.nonzero(img != ref)[0]
        assert len(bad) == 0, f"round {rnd}: {len(bad)} image bytes differ, first {bad[:8]}"
    assert (got["stage"][got["reason"] == 0] == 1).any()


def test_change_queued_while_batch_runs_on_other_stream(cuda):
    """Batch 1 (old tables) is enqueued on stream A; the filters of every
    UDP socket are then removed and batch 2 enqueued on stream B at once.
    Batch 1 must see none of the removal, batch 2 all of it."""
    torch = cuda
    filters, socks = pktgen.world(2)
    g = GpuRxStack(device=0)
    o_old, o_new = OracleStack(), OracleStack()
    for st in (g, o_old, o_new):
        st.load_world(filters, socks)
    n = 1 << 18
    buf, desc = pktgen.generate(2, n, first=77)
    fr, de = to_dev(buf), to_dev(desc)
    out1 = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    out2 = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):  # several back to back: batch 1 is still running below
        g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, out1.data_ptr(), 0,
                              a.cuda_stream)
    for f in filters[: len(filters) // 2]:
        for st in (g, o_new):
            assert st.filter_remove_raw(*_raw(f)) == 0
    g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, out2.data_ptr(), 0,
                          b.cuda_stream)
    torch.cuda.synchronize()
    got1 = out1.cpu().numpy().view(_abi.RESULT_DTYPE)
    got2 = out2.cpu().numpy().view(_abi.RESULT_DTYPE)
    want1 = o_old.handle_rx_batch(buf, desc, nthreads=8)
    want2 = o_new.handle_rx_batch(buf, desc, nthreads=8)
    assert got1.tobytes() == want1.tobytes(), diff_report(got1, want1, desc)
    assert got2.tobytes() == want2.tobytes(), diff_report(got2, want2, desc)
    assert (want2["reason"] == _abi.R_NO_MATCH).sum() > (want1["reason"] == _abi.R_NO_MATCH).sum()


def test_import_replicates_tables(cuda):
    """The image of a host-only stack, imported into a device stack from HBM
    (what a broadcast delivers), gives the same records as the tables built
    by calls; the device's own export equals the imported image."""
    torch = cuda
    filters, socks = pktgen.world(4)
    h = GpuRxStack(device=-1)
    o = OracleStack()
    for st in (h, o):
        st.load_world(filters, socks)
    for f in filters[::5]:  # tombstones and route counts in the image
        for st in (h, o):
            assert st.filter_remove_raw(*_raw(f)) == 0
    img = h.image_host()
    g = GpuRxStack(device=0)
    dimg = torch.from_numpy(img).to("cuda")
    g.table_import(dimg.data_ptr(), dimg.numel(), torch.cuda.current_stream().cuda_stream)
    assert np.array_equal(_device_image(torch, g), img)
    buf, desc = pktgen.generate(4, 1 << 14, first=99)
    from gpu_util import run_dev
    got, ctr = run_dev(g, buf, desc)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    assert got.tobytes() == want.tobytes(), diff_report(got, want, desc)
    # The imported mirror answers lookups and keeps placing entries right.
    for f in filters[::7][:50]:
        a = _raw(f)[1:]
        assert g.filter_lookup_raw(*a) == o.filter_lookup_raw(*a)


def _run_streams(torch, nstreams, nlaunch, cfg, n, done_every=0):
    filters, socks = pktgen.world(cfg)
    g = GpuRxStack(device=0)
    o = OracleStack()
    for st in (g, o):
        st.load_world(filters, socks)
    buf, desc = pktgen.generate(cfg, n, first=31)
    fr, de = to_dev(buf), to_dev(desc)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    outs = [torch.full((n * 32,), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(nlaunch)]
    torch.cuda.synchronize()
    for i in range(nlaunch):
        s = streams[i % nstreams]
        g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, outs[i].data_ptr(), 0,
                              s.cuda_stream)
        if done_every and i % done_every == done_every - 1:
            g.stream_done(s.cuda_stream)
            streams[i % nstreams] = torch.cuda.Stream()
    torch.cuda.synchronize()
    for i, out in enumerate(outs):
        got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
        assert got.tobytes() == want.tobytes(), f"launch {i}: " + diff_report(got, want, desc)
    g.close()


def test_launches_on_three_streams_share_no_claim_counters(cuda):
    """24 launches queued round-robin on three streams run
    concurrently; each stream has its own tile-claim counters, so every launch
    claims every tile exactly once (short frames: many claims per us)."""
    _run_streams(cuda, 3, 24, 3, 1 << 18)


def test_more_streams_than_tracked_entries(cuda):
    """Eleven streams through the context's eight tracked entries (a reused
    entry's new stream waits for the old one), with streams given up by
    oo_gpu_rx_stream_done and replaced as they go."""
    _run_streams(cuda, 11, 33, 2, 1 << 16, done_every=5)


def test_table_changes_across_destroyed_and_recreated_streams(cuda):
    """a table flush runs on stream A, the caller gives A up
    (oo_gpu_rx_stream_done) and destroys it, and a new stream -- often with
    the same handle -- runs the next batch after another change: that batch
    must wait for the flush (the context forgets A's handle at stream_done)
    and see the new tables.  Raw HIP streams (torch pools its own, so its
    handles never die); no synchronisation between the rounds."""
    import ctypes
    torch = cuda
    # the HIP runtime this process already runs (torch's), never a second copy
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(path)
    filters, socks = pktgen.world(2)
    g = GpuRxStack(device=0)
    o = OracleStack()
    for st in (g, o):
        st.load_world(filters, socks)
    n = 1 << 14
    buf, desc = pktgen.generate(2, n, first=5)
    fr, de = to_dev(buf), to_dev(desc)
    victims = filters[:8]
    outs, wants = [], []
    torch.cuda.synchronize()
    for r in range(16):
        f = victims[r % len(victims)]
        for st in (g, o):  # remove on even rounds, put back on odd ones
            rc = (st.filter_remove_raw if r % 2 == 0 else st.filter_insert_raw)(*_raw(f))
            assert rc == 0
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        out = torch.full((n * 32,), 0xAB, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # (the output's fill, on torch's stream)
        g.handle_rx_batch_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), n, out.data_ptr(), 0,
                              s.value)
        g.stream_done(s.value)
        assert hip.hipStreamDestroy(s) == 0
        outs.append(out)
        wants.append(o.handle_rx_batch(buf, desc, nthreads=8))
    torch.cuda.synchronize()
    for r, (out, want) in enumerate(zip(outs, wants)):
        got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
        assert got.tobytes() == want.tobytes(), f"round {r}: " + diff_report(got, want, desc)
    g.close()
