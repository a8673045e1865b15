# SPDX-License-Identifier: BSD-2-Clause
"""Device-resident throughput of Onload's RX transform (checksum verify +
header parse + 4-tuple demux) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

A "step" is one pass of the transform over one batch: BASELINE.json config 2
(2^20 x 1514 B IPv4/UDP) per GPU by default.  Frames, descriptors and the
filter tables are resident in HBM before the timed region; results (32 B per
frame) are written to HBM.  For N > 1 (torchrun, one rank per GPU) every rank
owns an independent shard of the packet stream (weak scaling, no data-path
collective); the timed region is bracketed by a barrier + device sync, the
max over ranks is taken, and rank 0 prints one JSON line.

Extra objects on that line:
  roofline      algorithmic HBM bytes of one launch / its average duration
                (HIP events on the launch stream) against the 8 TB/s peak;
                traffic = PMC-measured HBM bytes per launch from
                profiles/pmc_<config>.json when that file exists, else null.
  cpu_baseline  the CPU oracle (the reference path restated in C, fixture
                pinned) on host threads over the same frames (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
DESC_B, RESULT_B = 16, 32
DEFAULT_N = {2: 1 << 20, 3: 1 << 24, 4: 1 << 22, 5: 1 << 24}
WORKLOAD = {
    2: "config 2: 2^20 x 1514 B IPv4/UDP per GPU, device-resident csum+parse+demux",
    3: "config 3: 2^24 x 64 B IPv4/UDP per GPU, device-resident csum+parse+demux",
    4: "config 4: 2^22 mixed IPv4/TCP 64-9014 B with IP+TCP options per GPU",
    5: "config 5: 2^24 IMIX TCP+UDP IPv4+IPv6 per GPU (8 shards = 2^27 at 8 GPUs)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5))
    ap.add_argument("--n", type=int, default=0, help="packets per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--scatter", action="store_true",
                    help="N>1: also time an RCCL scatter of every shard from rank 0's GPU")
    ap.add_argument("--tx", action="store_true",
                    help="also time the TX checksum fill (oo_gpu_tx_fill_dev) on the same frames")
    ap.add_argument("--xdp", action="store_true",
                    help="also time the AF_XDP ring path (oo_gpu_rx_xdp_dev): the same frames in "
                         "a UMEM of 2048-B buffers at 256 B headroom, struct xdp_desc ring entries")
    ap.add_argument("--host-path", action="store_true",
                    help="also time pinned H2D + transform + D2H (printed to stderr)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from onload_amd import pktgen
    from onload_amd.rx import GpuRxStack

    cfg = args.config
    n = args.n or DEFAULT_N[cfg]
    seed = pktgen.default_seed(cfg)
    t0 = time.time()
    filters, socks = pktgen.world(cfg)
    from shard import shard_range
    first, _ = shard_range(n * world, rank, world)  # weak scaling: n per rank
    buf, desc = pktgen.generate(cfg, n, seed=seed, first=first)
    log(f"[rank {rank}] generated {n} frames ({buf.nbytes / 1e9:.2f} GB) in {time.time() - t0:.1f}s")

    stack = GpuRxStack(device=local)
    stack.load_world(filters, socks)
    frames = torch.from_numpy(buf).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    out = torch.empty(n * RESULT_B, dtype=torch.uint8, device=dev)
    ctr = torch.zeros(32, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    stack.sync(sh)

    def step():
        stack.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                                  out.data_ptr(), 0, sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_end = time.perf_counter()
    local_ms = (t_end - t_start) * 1e3 / args.steps
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    if world > 1:
        t = torch.tensor([local_ms, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_step, kern_ms_max = float(t[0]), float(t[1])
    else:
        ms_step, kern_ms_max = local_ms, kern_ms

    # Correctness of what was timed: counters of one more pass.
    stack.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                              out.data_ptr(), ctr.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    counts = ctr.cpu().numpy()
    assert counts.sum() == n, counts

    mean_len = float(desc["len"].astype(np.float64).mean())
    alg_bytes_pkt = mean_len + DESC_B + RESULT_B
    launch_bytes = alg_bytes_pkt * n
    achieved = launch_bytes / (kern_ms * 1e-3) / 1e9  # GB/s, this rank's kernel
    total_pkts = n * world
    mpps = total_pkts / (ms_step * 1e-3) / 1e6
    gbs = total_pkts * alg_bytes_pkt / (ms_step * 1e-3) / 1e9

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_config{cfg}.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if int(pm.get("packets_per_launch", -1)) == n:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    scatter = None
    if args.scatter and world > 1:
        scatter = time_scatter(torch, dist, cfg, seed, n, rank, world, dev, buf)
        if rank == 0:
            log(f"[rank 0] rccl scatter: {json.dumps(scatter)}")

    host_path = None
    if args.host_path:
        host_path = time_host_path(torch, stack, buf, desc, dev)
        log(f"[rank {rank}] host path: {json.dumps(host_path)}")

    tx = None
    if args.tx:
        tx = time_tx_fill(torch, stack, frames, d_desc, n, mean_len, sh, args.steps, args.warmup)
        log(f"[rank {rank}] tx fill: {json.dumps(tx)}")

    xdp = None
    if args.xdp:
        xdp = time_xdp(torch, stack, buf, desc, out, dev, sh, args.steps, args.warmup)
        log(f"[rank {rank}] xdp ring: {json.dumps(xdp)}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(filters, socks, buf, desc, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "Mpkt/s + GB/s device-resident csum+parse+demux, 1500B IPv4/UDP; % HBM roofline",
            "value": round(mpps, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/u16 integer (one's-complement sums in u32)",
            "data": "synthetic (seeded generator, onload_amd/csrc/oo_pktgen.c)",
            "config": {"workload": WORKLOAD[cfg], "packets_per_gpu": n,
                       "mean_frame_bytes": round(mean_len, 1), "sockets": len(socks),
                       "filters": len(filters), "parallelism": f"shard{world}"},
            "gbps": round(gbs, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel_ms": round(kern_ms, 5),
                         "kernel_ms_max_rank": round(kern_ms_max, 5),
                         "bytes_per_pkt": round(alg_bytes_pkt, 1)},
            "cpu_baseline": cpu,
            "outcomes": {k: int(v) for k, v in enumerate(counts) if v},
        }
        if host_path is not None:
            line["host_path"] = host_path
        if tx is not None:
            line["tx_fill"] = tx
        if xdp is not None:
            line["xdp_ring"] = xdp
        if scatter is not None:
            line["rccl_scatter"] = scatter
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def time_scatter(torch, dist, cfg, seed, n, rank, world, dev, my_buf, reps: int = 3):
    """Frames of all shards start on rank 0's GPU and are scattered over
    RCCL/xGMI (one 16-B-padded slab per rank); timed on its own, outside the
    device-resident metric.  Each rank checks it received its own shard."""
    from onload_amd import pktgen
    from shard import shard_range
    size = torch.tensor([my_buf.nbytes], dtype=torch.int64, device=dev)
    dist.all_reduce(size, op=dist.ReduceOp.MAX)
    slab = int(size.item() + 15) // 16 * 16
    recv = torch.empty(slab, dtype=torch.uint8, device=dev)
    send = None
    if rank == 0:
        send = []
        for r in range(world):
            first, _ = shard_range(n * world, r, world)
            b, _ = pktgen.generate(cfg, n, seed=seed, first=first)
            t = torch.zeros(slab, dtype=torch.uint8, device=dev)
            t[: b.nbytes] = torch.from_numpy(b).to(dev)
            send.append(t)
    times = []
    for r in range(reps + 1):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        dist.scatter(recv, send if rank == 0 else None, src=0)
        torch.cuda.synchronize(dev)
        dist.barrier()
        if r:
            times.append(time.perf_counter() - t0)
    ok = bool(torch.equal(recv[: my_buf.nbytes].cpu(), torch.from_numpy(my_buf)))
    okt = torch.tensor([1 if ok else 0], device=dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    s = float(np.median(times))
    return {"ms": round(s * 1e3, 3), "bytes_per_peer": slab,
            "GBps_from_root": round(slab * (world - 1) / s / 1e9, 1), "verified": bool(okt.item())}


def time_tx_fill(torch, stack, frames, d_desc, n, mean_len, sh, steps, warmup):
    """The TX checksum fill over the same HBM-resident frames (in place; a
    fill of already-filled frames rewrites the same values).  Algorithmic
    bytes: the frame read, the descriptor, the 4 check-field bytes written."""
    for _ in range(warmup):
        stack.tx_fill_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n, sh)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        stack.tx_fill_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n, sh)
        e.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    bpp = mean_len + DESC_B + 4
    gbs = n * bpp / (ms * 1e-3) / 1e9
    return {"kernel_ms": round(ms, 5), "mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "achieved_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "bytes_per_pkt": round(bpp, 1)}


def time_xdp(torch, stack, buf, desc, ref_out, dev, sh, steps, warmup, headroom=256):
    """The transform straight off an AF_XDP RX ring: the same frames laid out
    as AF_XDP delivers them (each in its own 2048-B UMEM buffer at `headroom`,
    a longer frame running on into the next buffers), the ring holding the
    entries from a consumer index just below 2^32 so the ring and the u32
    index both wrap.  Records must equal the descriptor path's (ref_out).
    Algorithmic bytes as the main line's: frame + 16-B entry + 32-B record."""
    from onload_amd import _abi
    n = len(desc)
    lens = desc["len"].astype(np.int64)
    nch = (headroom + lens + 2047) // 2048
    addr = (np.concatenate(([0], np.cumsum(nch)[:-1])) * 2048 + headroom).astype(np.uint64)
    umem = np.zeros(int(nch.sum()) * 2048, dtype=np.uint8)
    offs = desc["frame_off"].astype(np.int64)
    for L in np.unique(lens):  # vectorised per frame length, in bounded pieces
        idx = np.nonzero(lens == L)[0]
        step = max(1, (1 << 24) // max(int(L), 1))
        col = np.arange(int(L), dtype=np.int64)
        for i in range(0, len(idx), step):
            j = idx[i:i + step]
            umem[addr[j].astype(np.int64)[:, None] + col] = buf[offs[j][:, None] + col]
    log2 = max(1, (n - 1).bit_length())
    cons = (1 << 32) - n // 2
    ring = np.zeros(1 << log2, dtype=_abi.XDP_DESC_DTYPE)
    at = (cons + np.arange(n, dtype=np.uint64)) & np.uint64((1 << log2) - 1)
    ring["addr"][at] = addr
    ring["len"][at] = lens.astype(np.uint32)
    d_umem = torch.from_numpy(umem).to(dev)
    d_ring = torch.from_numpy(ring.view(np.uint8)).to(dev)
    del umem
    out = torch.empty_like(ref_out)
    intf = int(desc["intf_i"][0]) if n else 0

    def run():
        stack.xdp_dev(d_umem.data_ptr(), d_umem.numel(), d_ring.data_ptr(), (1 << log2) - 1,
                      cons, n, intf, out.data_ptr(), 0, sh)
    for _ in range(warmup):
        run()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        run()
        e.record(stream)
    torch.cuda.synchronize()
    same = bool(torch.equal(out, ref_out)) and bool((desc["intf_i"] == intf).all())
    ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    bpp = float(lens.mean()) + DESC_B + RESULT_B
    gbs = n * bpp / (ms * 1e-3) / 1e9
    return {"kernel_ms": round(ms, 5), "mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "achieved_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "umem_bytes": int(d_umem.numel()), "headroom": headroom,
            "records_equal_descriptor_path": same}


def time_host_path(torch, stack, buf, desc, dev, reps: int = 5):
    """Pinned host frames -> H2D -> transform -> D2H results, one stream."""
    n = len(desc)
    h_frames = torch.from_numpy(buf).pin_memory()
    h_desc = torch.from_numpy(desc.view(np.uint8)).pin_memory()
    h_out = torch.empty(n * RESULT_B, dtype=torch.uint8).pin_memory()
    d_frames = torch.empty_like(h_frames, device=dev)
    d_desc = torch.empty_like(h_desc, device=dev)
    d_out = torch.empty(n * RESULT_B, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    times = []
    for r in range(reps + 1):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        d_frames.copy_(h_frames, non_blocking=True)
        d_desc.copy_(h_desc, non_blocking=True)
        stack.handle_rx_batch_dev(d_frames.data_ptr(), d_frames.numel(), d_desc.data_ptr(), n,
                                  d_out.data_ptr(), 0, stream.cuda_stream)
        h_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize(dev)
        if r:
            times.append(time.perf_counter() - t)
    s = float(np.median(times))
    byt = buf.nbytes + desc.nbytes + n * RESULT_B
    return {"mpps": round(n / s / 1e6, 2), "gbs_pcie": round(byt / s / 1e9, 2),
            "ms": round(s * 1e3, 3)}


def cpu_baseline(filters, socks, buf, desc, seconds):
    """The oracle (reference CPU path restated in C, pinned by tests/golden)
    on host threads over the same frames."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import OracleStack
    threads = min(16, os.cpu_count() or 1)
    o = OracleStack()
    o.load_world(filters, socks)
    sample = min(len(desc), 1 << 18)
    d = desc[:sample]
    o.handle_rx_batch(buf, d[:1024], nthreads=threads)  # warm
    done, t = 0, time.perf_counter()
    while True:
        o.handle_rx_batch(buf, d, nthreads=threads)
        done += sample
        el = time.perf_counter() - t
        if el >= seconds:
            break
    return {"value": round(done / el / 1e6, 3), "unit": "Mpkt/s", "cores": threads,
            "kind": "port",
            "sample": f"first {sample} frames of the same workload, repeated for {el:.1f}s "
                      f"({threads} threads, contiguous shards)"}


if __name__ == "__main__":
    main()
