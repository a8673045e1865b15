# SPDX-License-Identifier: BSD-2-Clause
"""Per-wave phase timeline of one rx_kernel launch (diagnostic).

Needs a library built with -DOO_RX_STAMPS (``make variants
VARIANTS="st:-DOO_RX_EXPERIMENTS,-DOO_RX_STAMPS"``), selected with OO_RX_LIB.  Prints where a
wave's time goes per tile (header wait, parse, body stream, record) and how
the waves' finish times spread.

    OO_RX_LIB=build/var_st.so python tools/stamps.py --config 2
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def oo_waves_per_block(lib) -> int:
    try:
        return int(lib.oo_rx_waves_per_block())
    except AttributeError:
        return 2


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--raw", default="", help="also save the per-wave stamps (npz) here")
    args = ap.parse_args()
    import torch

    from bench import DEFAULT_N
    from onload_amd import pktgen
    from onload_amd.rx import GpuRxStack

    # The stamps come from rx_kernel's tile loop: its instance for the
    # configuration (the split transform's kernels write none).
    os.environ.setdefault("OO_RX_KERNEL", "2" if args.config in (3, 5) else "1")
    dev = torch.device("cuda", 0)
    n = args.n or DEFAULT_N[args.config]
    filters, socks = pktgen.world(args.config)
    buf, desc = pktgen.generate(args.config, n)
    g = GpuRxStack(device=0)
    g.load_world(filters, socks)
    lib = g._lib
    lib.oo_gpu_rx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.oo_gpu_rx_debug_grid.argtypes = [ctypes.c_void_p]
    grid = lib.oo_gpu_rx_debug_grid(g._ctx)
    frames = torch.from_numpy(buf).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    waves = grid * 4  # upper bound on waves per block
    st = torch.zeros(waves * 128 * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    g.sync(s)
    for _ in range(3):
        g.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                              out.data_ptr(), 0, s)
    lib.oo_gpu_rx_debug_stamps(g._ctx, ctypes.c_void_p(st.data_ptr()))
    torch.cuda.synchronize(dev)
    g.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                          out.data_ptr(), 0, s)
    torch.cuda.synchronize(dev)
    a = st.cpu().numpy().reshape(waves, 128, 16)
    used = a[:, :, 0] != 0
    if args.raw:
        kmax = int(used.sum(1).max())
        np.savez_compressed(args.raw, stamps=a[:, :kmax, :8], grid=grid,
                            waves_per_block=oo_waves_per_block(lib))
    t0 = a[:, :, 0][used].min()
    ns = 10.0  # s_memrealtime is 100 MHz
    rows = []
    for w in range(waves):
        k = int(used[w].sum())
        if k == 0:
            continue
        rows.append((w, k, (a[w, k - 1, 5] - t0) * ns, (a[w, 0, 0] - t0) * ns))
    rows = np.array(rows)
    ph = a[used]
    d = lambda i, j: (ph[:, j] - ph[:, i]) * ns  # noqa: E731
    res = {
        "waves": int(len(rows)), "grid_blocks": grid,
        "tiles_per_wave": {str(int(k)): int((rows[:, 1] == k).sum()) for k in np.unique(rows[:, 1])},
        "kernel_span_us": float(rows[:, 2].max() / 1e3),
        "wave_end_us_pct": [float(np.percentile(rows[:, 2], q) / 1e3) for q in (0, 10, 50, 90, 100)],
        "wave_start_us_max": float(rows[:, 3].max() / 1e3),
        "per_tile_us_mean": {
            "hdr_wait": float(d(0, 1).mean() / 1e3), "parse": float(d(1, 2).mean() / 1e3),
            "demux": float(d(2, 3).mean() / 1e3),
            "stream": float(d(3, 4).mean() / 1e3),
            "record": float(d(4, 5).mean() / 1e3), "total": float(d(0, 5).mean() / 1e3),
            "gap_to_next": float(np.mean([(a[w, i + 1, 0] - a[w, i, 5]) * ns
                                          for w in range(waves) for i in range(int(used[w].sum()) - 1)]) / 1e3),
        },
        "rounds_mean": float(ph[:, 7].mean()),
        "stream_ns_per_round": float((d(3, 4) / np.maximum(ph[:, 7], 1)).mean()),
    }
    # Inside the demux (slots 8-12, when the build stamps them): first-probe
    # occupancy words landed, first records issued, stages walked (11, 12:
    # after the first and the second stage).
    dm = ph[:, 8] != 0
    if dm.any():
        q = ph[dm]

        def phase(i, j):
            # a phase whose start or end stamp is missing (0: the build or
            # the tile did not reach it) is reported as missing, never as a
            # difference against zero
            ok = (q[:, i] != 0) & (q[:, j] != 0)
            if not ok.any():
                return {"us": None, "tiles": 0, "missing": int(len(q))}
            return {"us": float(((q[ok, j] - q[ok, i]) * ns).mean() / 1e3), "tiles": int(ok.sum()),
                    "missing": int((~ok).sum())}
        res["demux_us_mean"] = {"occ_words": phase(2, 8), "to_walks": phase(8, 9),
                                "walks": phase(9, 10), "after_walks": phase(10, 3)}
        # The state-machine walk stamps its step count in slot 11 (+1e6).
        fsm = dm & (ph[:, 11] >= 1000000) & (ph[:, 11] < 2000000)
        if fsm.any():
            res["fsm_steps_mean"] = float((ph[fsm, 11] - 1000000).mean())
            res["fsm_steps_hist"] = np.bincount((ph[fsm, 11] - 1000000).astype(np.int64)).tolist()
        # Per stage (slots 11, 12: after the first and second stage walks).
        st = dm & (ph[:, 11] < 1000000) & (ph[:, 9] != 0) & (ph[:, 10] != 0) & (ph[:, 11] != 0) & (ph[:, 12] != 0)
        if st.any():
            q = ph[st]
            res["walk_stage_us_mean"] = [float(((q[:, 11] - q[:, 9]) * ns).mean() / 1e3),
                                         float(((q[:, 12] - q[:, 11]) * ns).mean() / 1e3),
                                         float(((q[:, 10] - q[:, 12]) * ns).mean() / 1e3)]
    # The demux as a chain of its stamps (2 -> 8 -> 9 -> 10 -> 11 -> 12 -> 3),
    # over the tiles that have them all (builds that stamp the key index's
    # levels: 9 before, 10 after the first, 11 after the last; 12 before the
    # record's assembly).
    # (builds that stamp the index's level count as 4000000 + levels in slot 11)
    lvm = (ph[:, 11] >= 4000000) & (ph[:, 11] < 5000000)
    if lvm.any():
        res["kx_levels_hist"] = np.bincount((ph[lvm, 11] - 4000000).astype(np.int64)).tolist()
    res["slot_nonzero_frac"] = [round(float((ph[:, j] != 0).mean()), 3) for j in range(16)]
    chain = [2, 8, 9, 10, 11, 12, 3]
    cm = np.all(ph[:, chain] != 0, axis=1) & ~((ph[:, 11] >= 1000000) & (ph[:, 11] < 2000000))
    if cm.any():
        q = ph[cm]
        res["demux_chain_us"] = {f"{i}->{j}": float(((q[:, j] - q[:, i]) * ns).mean() / 1e3)
                                 for i, j in zip(chain, chain[1:])}
        res["demux_chain_tiles"] = int(cm.sum())
    # Inside the parse (slots 13-15, when the build stamps them): the cells
    # read and the IPv4 fixed-format parse, the IPv6 one, the general walk.
    pm = (ph[:, 13] != 0) & (ph[:, 14] != 0) & (ph[:, 15] != 0)
    if pm.any():
        q = ph[pm]
        res["parse_us_mean"] = {
            "cells_fixed4": float(((q[:, 13] - q[:, 1]) * ns).mean() / 1e3),
            "fixed6": float(((q[:, 14] - q[:, 13]) * ns).mean() / 1e3),
            "general": float(((q[:, 15] - q[:, 14]) * ns).mean() / 1e3),
            "to_stamp2": float(((q[:, 2] - q[:, 15]) * ns).mean() / 1e3),
            "tiles": int(pm.sum())}
        gm = pm & (ph[:, 9] != 0) & (ph[:, 12] != 0) & (ph[:, 10] != 0) & (ph[:, 11] != 0)
        if gm.any():
            q = ph[gm]
            res["general_us_mean"] = {
                "l2_l3": float(((q[:, 9] - q[:, 14]) * ns).mean() / 1e3),
                "l4_pseudo": float(((q[:, 10] - q[:, 9]) * ns).mean() / 1e3),
                "sums": float(((q[:, 11] - q[:, 10]) * ns).mean() / 1e3),
                "verdict_fields_options": float(((q[:, 12] - q[:, 11]) * ns).mean() / 1e3),
                "to_end": float(((q[:, 15] - q[:, 12]) * ns).mean() / 1e3),
                "tiles": int(gm.sum())}
    # Phase concurrency over time: the fraction of live waves streaming a
    # body (stamps 3 -> 4) vs in the header phases (0 -> 3), in 1-us bins --
    # synchronised header phases show as dips in the streaming fraction.
    span = int(rows[:, 2].max() / 1e3) + 1
    bins = np.arange(0, span + 1, 1.0)
    strm = np.zeros(len(bins) - 1)
    head = np.zeros(len(bins) - 1)
    for w in range(waves):
        for i in range(int(used[w].sum())):
            t = (a[w, i, :6] - t0) * ns / 1e3
            strm += np.histogram(np.linspace(t[3], t[4], 64), bins)[0] * ((t[4] - t[3]) / 64)
            head += np.histogram(np.linspace(t[0], t[3], 16), bins)[0] * ((t[3] - t[0]) / 16)
    live = strm + head
    frac = np.where(live > 0, strm / np.maximum(live, 1e-9), 0)
    res["stream_frac_by_us"] = {"min": float(frac[5:-40].min()) if span > 60 else None,
                                "mean": float(frac[5:-40].mean()) if span > 60 else None,
                                "first_12us": [round(float(x), 2) for x in frac[:12]],
                                "p10_p90": [float(np.percentile(frac[5:-40], 10)),
                                            float(np.percentile(frac[5:-40], 90))] if span > 60 else None}
    # The launch's end: live and streaming waves and the body bytes streamed
    # (each tile's rounds x 1 KiB spread evenly over its stream phase), in
    # 2-us bins over the last 40 us, against the mean rate of the middle.
    kb = np.zeros(len(bins) - 1)
    for w in range(waves):
        for i in range(int(used[w].sum())):
            t = (a[w, i, :6] - t0) * ns / 1e3
            kb += np.histogram(np.linspace(t[3], t[4], 64), bins)[0] * (float(a[w, i, 7]) / 64)
    if span > 60:
        tail = slice(span - 40, span)
        pair = lambda x: [round(float(x[tail][j:j + 2].sum() / 2), 2) for j in range(0, 40, 2)]  # noqa: E731
        res["end_40us"] = {"live_waves": pair(live), "streaming_waves": pair(strm),
                           "body_GBps": [round(v * 1.024, 0) for v in pair(kb)],
                           "body_GBps_mid_mean": round(float(kb[20:span - 40].mean()) * 1.024, 0)}
    res["per_tile_k_us"] = {str(k): [round(float(np.mean((a[used[:, k], k, j + 1] - a[used[:, k], k, j]) * ns / 1e3)), 2)
                                     for j in range(5)]
                            for k in range(min(int(used.sum(1).max()), 8)) if used[:, k].any()}
    # per-XCD view: blocks are dealt round-robin to the 8 XCDs
    wpb = oo_waves_per_block(lib)
    ends = {}
    for w, k, e, _ in rows:
        ends.setdefault(int(w) // wpb % 8, []).append(e / 1e3)
    res["end_us_by_xcd(block%8)"] = {x: round(float(np.mean(v)), 1) for x, v in sorted(ends.items())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
