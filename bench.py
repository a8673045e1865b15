# SPDX-License-Identifier: BSD-2-Clause
"""Device-resident throughput of Onload's RX transform (checksum verify +
header parse + 4-tuple demux) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

A "step" is one pass of the transform over one batch: BASELINE.json config 2
(2^20 x 1514 B IPv4/UDP) per GPU by default.  Frames, descriptors and the
filter tables are resident in HBM before the timed region; results (32 B per
frame) are written to HBM.

N > 1: one process per GPU.  Under torchrun (WORLD_SIZE set) --gpus must
equal WORLD_SIZE; run directly, bench.py starts the N ranks itself (child
processes, before anything touches a GPU) and exits with the worst rank's
status.  Each rank owns a contiguous shard of the packet stream (weak
scaling: N x the per-GPU packets; byte-balanced for the mixed-size configs,
onload_amd/shards.py), rank 0 builds the filter tables and broadcasts the
table image over RCCL, no collective touches the timed data path; the timed
region is bracketed by a barrier + device sync, the max over ranks is taken,
and rank 0 prints one JSON line (the records are then gathered to rank 0 and
counted, outside the timed region).

Extra objects on that line:
  roofline      algorithmic HBM bytes of one launch / its average duration
                (HIP events on the launch stream) against the 8 TB/s peak;
                traffic = PMC-measured HBM bytes per launch from
                profiles/pmc_config<N>.json when that file exists, else null.
  cpu_baseline  the CPU restatement of the reference path (fixture-pinned
                oracle, a "port") on every host core this process may use,
                over a bounded sample of the same frames (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Kernel arguments in device memory: a setting of this process's HIP runtime,
# read when the runtime starts (here, before any rank touches a GPU; child
# ranks inherit it).  Every wave of a launch reads its KParams at its start;
# from HBM rather than over PCIe the launch ramps ~1 % sooner.
# An explicit value in the environment wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5))
    ap.add_argument("--n", type=int, default=0, help="packets per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--align", type=int, default=64,
                    help="frame alignment in the packed buffer (diagnostics: 64 is the workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--steady", type=int, default=200,
                    help="side measurement after the timed region: this many more launches, "
                         "event-timed (0: skip); reported as 'steady', never as value")
    ap.add_argument("--scatter", action="store_true",
                    help="N>1: also time an RCCL scatter of every shard from rank 0's GPU")
    ap.add_argument("--tx", action="store_true",
                    help="also time the TX checksum fill (oo_gpu_tx_fill_dev) on the same frames")
    ap.add_argument("--xdp", action="store_true",
                    help="also time the AF_XDP ring path (oo_gpu_rx_xdp_dev): the same frames in "
                         "a UMEM of 2048-B buffers at 256 B headroom, struct xdp_desc ring entries")
    ap.add_argument("--xdp-host", action="store_true",
                    help="also time zero-copy AF_XDP ingest: UMEM and ring in registered host "
                         "memory read by the kernel over PCIe")
    ap.add_argument("--pipelined", action="store_true",
                    help="also time consecutive batches alternating over two streams (a side "
                         "measurement: never value)")
    ap.add_argument("--table-ops", action="store_true",
                    help="also time device-side table maintenance: the world load's flush, "
                         "and a 100-op filter churn batch in front of one batch")
    ap.add_argument("--group", action="store_true",
                    help="N=1: run the rank through the library's joined group anyway (a group "
                         "of one rank: its table image, record gather and counter sum go "
                         "through librccl); N>1 always does")
    ap.add_argument("--host-path", action="store_true",
                    help="also time the host-memory path: oo_gpu_rx_submit/_wait, pinned "
                         "double-buffered H2D + transform + D2H")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv: list[str], script: str | None = None,
                 poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Start n ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, one GPU each) as child processes -- this process never
    touches a GPU -- and return the worst exit status.

    Watchdog: the children are polled together; the first one to exit
    non-zero gets the others terminated (SIGTERM, then SIGKILL after
    grace_s) -- they would otherwise block in a barrier or an RCCL
    collective until an outer timeout -- and its status is returned, with
    the rank named on stderr."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv,
                                      env=env))
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0:
                log(f"bench.py: rank {r} exited with status {c}; stopping ranks {sorted(live)}")
                for k in live:
                    procs[k].terminate()
                deadline = time.time() + grace_s
                for k in live:
                    try:
                        procs[k].wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        procs[k].kill()
                        procs[k].wait()
                return c
        if live:
            time.sleep(poll_s)
    return 0


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus > 1:
            return launch_ranks(args.gpus, argv)
    elif int(world_env) != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
        return 2
    if os.environ.get("OO_BENCH_PROBE"):  # launcher test: report and stop before any GPU use
        import torch
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")),
                          "world": int(os.environ.get("WORLD_SIZE", "1")),
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "cuda_initialized": bool(torch.cuda.is_initialized())}), flush=True)
        return 0
    _json_only_stdout()
    run_rank(args)
    return 0


def _json_only_stdout() -> None:
    """This rank's file descriptor 1 goes to stderr, so libraries that print
    to it (librccl writes its version banner there at communicator init) do
    not mix with the one JSON line, which goes to the original stdout."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(real, "w", buffering=1)


def run_rank(args) -> None:
    import torch
    import torch.distributed as dist

    from onload_amd import pktgen, shards
    from onload_amd.rx import GpuRxStack

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N>1 path on a box with fewer GPUs than ranks (never
    # for a measurement): OO_BENCH_SHARE_GPU=1 puts rank r on GPU r mod the
    # GPUs present, OO_BENCH_BACKEND=gloo replaces RCCL (which takes one rank
    # per GPU).
    if os.environ.get("OO_BENCH_SHARE_GPU") == "1":
        local %= max(1, torch.cuda.device_count())
    backend = os.environ.get("OO_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    cfg = args.config
    n_per = args.n or DEFAULT_N[cfg]
    seed = pktgen.default_seed(cfg)
    n_total = n_per * world  # weak scaling
    first, n = shards.shard_for(cfg, seed, n_total, rank, world)
    t0 = time.time()
    filters, socks = pktgen.world(cfg)
    buf, desc = pktgen.generate(cfg, n, seed=seed, first=first, align=args.align)
    log(f"[rank {rank}] packets [{first}, {first + n}) ({buf.nbytes / 1e9:.2f} GB) "
        f"generated in {time.time() - t0:.1f}s")

    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    table_bcast = None
    group = None
    group_path = None
    if world > 1 or args.group:
        # The library's multi-GPU group across processes (include/oo_gpu_rx.h
        # "Multi-GPU group"): rank 0 makes the RCCL id, torch.distributed's
        # control plane hands it out, every rank joins with one member on its
        # GPU; rank 0 owns the socket world and the group broadcasts its
        # table image over RCCL.  Where the join is refused (RCCL takes one
        # rank per GPU: the shared-GPU rehearsal) the Python path over
        # torch.distributed does the same, and the line says which ran.
        # --group at N=1: a group of one rank, the same librccl calls.
        from onload_amd.group import GpuRxGroup
        gid = [GpuRxGroup.rccl_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(gid, src=0)
        try:
            group = GpuRxGroup.join(local, rank, world, gid[0])
            log(f"[rank {rank}] joined the library's group ({world} rank(s), librccl)")
        except OSError as e:
            if world == 1:
                raise
            log(f"[rank {rank}] group join refused ({e}); torch.distributed path")
        if world > 1:
            ok = torch.tensor([1 if group is not None else 0], device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and group is not None:
                group.close()
                group = None
        group_path = "c_group_rccl" if group is not None else "torch_distributed"
        stack = group.members[0] if group is not None else GpuRxStack(device=local)
        if rank == 0:
            (group or stack).load_world(filters, socks)
        if world > 1:
            dist.barrier()
        tb = time.perf_counter()
        if group is not None:
            group.share_tables(sh)
            nbytes = stack.image_bytes()
        else:
            nbytes = shards.broadcast_tables(stack, torch, dist, dev, 0, sh)
        torch.cuda.synchronize(dev)
        table_bcast = {"bytes": nbytes, "ms": round((time.perf_counter() - tb) * 1e3, 3),
                       "path": group_path}
    else:
        stack = GpuRxStack(device=local)
        stack.load_world(filters, socks)
    frames = torch.from_numpy(buf).to(dev)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    out = torch.empty(max(n, 1) * RESULT_B, dtype=torch.uint8, device=dev)
    ctr = torch.zeros(32, dtype=torch.int32, device=dev)
    stack.sync(sh)

    def step():
        stack.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                                  out.data_ptr(), 0, sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # One HIP event pair on the launch stream around the K back-to-back
    # launches: kernel time = region / K (an event pair around every launch
    # would add the event and dispatch gap to each one: ~7 us on a 265-us
    # kernel, against the rocprofv3 duration).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_end = time.perf_counter()
    local_ms = (t_end - t_start) * 1e3 / args.steps
    kern_ms = float(ev0.elapsed_time(ev1)) / args.steps
    if world > 1:
        t = torch.tensor([local_ms, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms_step, kern_ms_max = float(t[0]), float(t[1])
    else:
        ms_step, kern_ms_max = local_ms, kern_ms

    # Side measurement, after the timed region: the same launch repeated
    # --steady times.  The GPU's clock settles several milliseconds after it
    # becomes busy (2.0-2.1 GHz around launches 7-19,
    # 2.35-2.47 GHz from about the 30th), so K = 20 launches after W = 5 sit
    # in that dip; this shows the settled per-launch time next to it.  It is
    # never `value` or `roofline`.
    steady = None
    if args.steady > 0:
        es0, es1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        es0.record(stream)
        for _ in range(args.steady):
            step()
        es1.record(stream)
        torch.cuda.synchronize(dev)
        st_ms = float(es0.elapsed_time(es1)) / args.steady
        st_mean = float(desc["len"].astype(np.float64).mean()) if n else 0.0
        steady = {"launches": args.steady, "after_launches": args.warmup + args.steps,
                  "kernel_ms": round(st_ms, 5),
                  "frac": round((st_mean + DESC_B + RESULT_B) * n / (st_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}

    # What was timed is checked: one more pass with counters; N>1 gathers
    # every rank's records to rank 0 (outside the timed region).
    stack.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                              out.data_ptr(), ctr.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    gather = None
    if group is not None or world > 1:
        tg = time.perf_counter()
        if group is not None:
            group.sum_counters(ctr.data_ptr(), sh)
            if world > 1:
                cnts = torch.tensor([n], dtype=torch.int64, device=dev)
                allc = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
                dist.all_gather(allc, cnts)
                counts_r = [int(c.item()) for c in allc]
            else:
                counts_r = [n]
            recs = (torch.empty(sum(counts_r) * RESULT_B, dtype=torch.uint8, device=dev)
                    if rank == 0 else None)
            group.gather_rccl(out.data_ptr(), n, recs.data_ptr() if rank == 0 else 0,
                              counts_r if rank == 0 else None, sh)
        else:
            dist.all_reduce(ctr)
            recs = shards.gather_records(out, n, torch, dist, 0)
        torch.cuda.synchronize(dev)
        if rank == 0:
            r = recs.view(-1, RESULT_B)[:, 0].cpu().numpy()
            ok = bool((np.bincount(r, minlength=32) == ctr.cpu().numpy()).all())
            gather = {"records": int(len(r)), "ms": round((time.perf_counter() - tg) * 1e3, 3),
                      "counts_match": ok, "path": group_path}
            if world == 1:  # a group of one: the records came back through librccl
                gather["records_equal"] = bool(torch.equal(recs, out[: n * RESULT_B]))
    counts = ctr.cpu().numpy()
    assert counts.sum() == n_total, counts
    path = stack.last_path()  # which kernels the timed launches ran

    bytes_all = torch.tensor([float(buf.nbytes), float(desc["len"].astype(np.float64).sum())],
                             dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(bytes_all)
    mean_len = float(bytes_all[1]) / n_total
    alg_bytes_pkt = mean_len + DESC_B + RESULT_B
    my_mean = float(desc["len"].astype(np.float64).mean()) if n else 0.0
    achieved = (my_mean + DESC_B + RESULT_B) * n / (kern_ms * 1e-3) / 1e9  # this rank's kernel
    mpps = n_total / (ms_step * 1e-3) / 1e6
    gbs = n_total * alg_bytes_pkt / (ms_step * 1e-3) / 1e9

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_config{cfg}.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if int(pm.get("packets_per_launch", -1)) == n:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    extras = {}
    if steady is not None:
        extras["steady"] = steady
    if table_bcast is not None:
        extras["table_broadcast"] = table_bcast
    if gather is not None:
        extras["record_gather"] = gather
    if args.scatter and world > 1:
        extras["rccl_scatter"] = time_scatter(torch, dist, shards, cfg, seed, n_total, rank,
                                              world, dev, buf)
    if args.pipelined:
        extras["pipelined_2stream"] = time_pipelined(torch, stack, frames, d_desc, n, my_mean, out,
                                                     dev, stream, args.steps, args.warmup)
        log(f"[rank {rank}] pipelined: {json.dumps(extras['pipelined_2stream'])}")
    if args.table_ops:
        extras["table_ops"] = time_table_ops(torch, filters, socks, frames, d_desc, n, out, local)
        log(f"[rank {rank}] table ops: {json.dumps(extras['table_ops'])}")
    if args.host_path:
        extras["host_path"] = time_host_path(torch, filters, socks, buf, desc, local)
        log(f"[rank {rank}] host path: {json.dumps(extras['host_path'])}")
    if args.tx:
        extras["tx_fill"] = time_tx_fill(torch, stack, frames, d_desc, n, my_mean, sh,
                                         args.steps, args.warmup)
        log(f"[rank {rank}] tx fill: {json.dumps(extras['tx_fill'])}")
    if args.xdp:
        extras["xdp_ring"] = time_xdp(torch, stack, buf, desc, out, dev, sh, args.steps,
                                      args.warmup)
        log(f"[rank {rank}] xdp ring: {json.dumps(extras['xdp_ring'])}")
    if args.xdp_host:
        extras["xdp_host"] = time_xdp_host(torch, stack, buf, desc, out, dev, sh)
        log(f"[rank {rank}] xdp host: {json.dumps(extras['xdp_host'])}")

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
            "config": {"workload": WORKLOAD[cfg], "packets_per_gpu": n_per,
                       "packets_total": n_total, "mean_frame_bytes": round(mean_len, 1),
                       "sockets": len(socks), "filters": len(filters),
                       "parallelism": f"shard{world}",
                       "sharding": "bytes" if (world > 1 and cfg in shards.MIXED_CONFIGS)
                       else "count"},
            "gbps": round(gbs, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "kernels": PATH_KERNELS.get(path, []),
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel_ms": round(kern_ms, 5),
                         "kernel_ms_max_rank": round(kern_ms_max, 5),
                         "bytes_per_pkt": round(my_mean + DESC_B + RESULT_B, 1)},
            "cpu_baseline": cpu,
            "hip_env": {"HIP_FORCE_DEV_KERNARG": os.environ.get("HIP_FORCE_DEV_KERNARG")},
            "outcomes": {k: int(v) for k, v in enumerate(counts) if v},
            "path": group_path or "stack",
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
    if group is not None:
        group.close()
    if world > 1:
        dist.destroy_process_group()


# oo_gpu_rx_last_path -> the kernels one timed launch runs (their summed
# duration is the launch's; rocprofv3 lists them separately).
PATH_KERNELS = {1: ["oo_rx::rx_kernel"], 2: ["oo_rx_short::rx_kernel"],
                3: ["oo_rx::win_kernel", "oo_rx::body_kernel"],
                4: ["oo_rx::win_kernel", "oo_rx_short::body_kernel"],
                5: ["oo_rx_poll::rx_kernel"]}


def time_scatter(torch, dist, shards, cfg, seed, n_total, rank, world, dev, my_buf,
                 reps: int = 3):
    """Frames of all shards start on rank 0's GPU and are scattered over
    RCCL/xGMI (one padded slab per rank); timed on its own, outside the
    device-resident metric.  Each rank checks it received its own shard."""
    from onload_amd import pktgen
    size = torch.tensor([my_buf.nbytes], dtype=torch.int64, device=dev)
    dist.all_reduce(size, op=dist.ReduceOp.MAX)
    slab = int(size.item() + 15) // 16 * 16
    src = None
    if rank == 0:
        src = []
        for r in range(world):
            f, c = shards.shard_for(cfg, seed, n_total, r, world)
            b, _ = pktgen.generate(cfg, c, seed=seed, first=f)
            src.append(torch.from_numpy(b).to(dev))
    times = []
    recv = None
    for r in range(reps + 1):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        recv = shards.scatter_frames(src, slab, torch, dist, dev, 0)
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
    ms = _timed(torch, lambda: stack.tx_fill_dev(frames.data_ptr(), frames.numel(),
                                                 d_desc.data_ptr(), n, sh), steps, warmup)
    bpp = mean_len + DESC_B + 4
    gbs = n * bpp / (ms * 1e-3) / 1e9
    return {"kernel_ms": round(ms, 5), "mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "achieved_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "bytes_per_pkt": round(bpp, 1)}


def _umem_layout(buf, desc, headroom, out=None):
    """The frames as AF_XDP delivers them: each in its own 2048-B buffer at
    `headroom` (a longer frame running on into the next buffers).  Returns
    (umem, entry addresses, lengths)."""
    lens = desc["len"].astype(np.int64)
    nch = (headroom + lens + 2047) // 2048
    addr = (np.concatenate(([0], np.cumsum(nch)[:-1])) * 2048 + headroom).astype(np.uint64)
    size = int(nch.sum()) * 2048
    umem = out[:size] if out is not None else np.zeros(size, dtype=np.uint8)
    offs = desc["frame_off"].astype(np.int64)
    for L in np.unique(lens):  # vectorised per frame length, in bounded pieces
        idx = np.nonzero(lens == L)[0]
        step = max(1, (1 << 24) // max(int(L), 1))
        col = np.arange(int(L), dtype=np.int64)
        for i in range(0, len(idx), step):
            j = idx[i:i + step]
            umem[addr[j].astype(np.int64)[:, None] + col] = buf[offs[j][:, None] + col]
    return umem, addr, lens


def _ring(addr, lens, cons):
    from onload_amd import _abi
    n = len(addr)
    log2 = max(1, (n - 1).bit_length())
    ring = np.zeros(1 << log2, dtype=_abi.XDP_DESC_DTYPE)
    at = (cons + np.arange(n, dtype=np.uint64)) & np.uint64((1 << log2) - 1)
    ring["addr"][at] = addr
    ring["len"][at] = lens.astype(np.uint32)
    return ring, (1 << log2) - 1


def _timed(torch, run, steps, warmup):
    for _ in range(warmup):
        run()
    # one event pair around the back-to-back launches (as the main timing)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    ev0.record(stream)
    for _ in range(steps):
        run()
    ev1.record(stream)
    torch.cuda.synchronize()
    return float(ev0.elapsed_time(ev1)) / steps


def time_xdp(torch, stack, buf, desc, ref_out, dev, sh, steps, warmup, headroom=256):
    """The transform straight off an AF_XDP RX ring in HBM: the same frames
    in a UMEM of 2048-B buffers, the ring holding the entries from a consumer
    index just below 2^32 so the ring and the u32 index both wrap.  Records
    must equal the descriptor path's (ref_out).  Algorithmic bytes as the
    main line's: frame + 16-B entry + 32-B record."""
    n = len(desc)
    umem, addr, lens = _umem_layout(buf, desc, headroom)
    cons = (1 << 32) - n // 2
    ring, mask = _ring(addr, lens, cons)
    d_umem = torch.from_numpy(umem).to(dev)
    d_ring = torch.from_numpy(ring.view(np.uint8)).to(dev)
    del umem
    out = torch.empty_like(ref_out)
    intf = int(desc["intf_i"][0]) if n else 0

    def run():
        stack.xdp_dev(d_umem.data_ptr(), d_umem.numel(), d_ring.data_ptr(), mask, cons, n, intf,
                      out.data_ptr(), 0, sh)
    # The UMEM's bytes per packet say nothing of the frames: the caller's
    # mean-length hint picks the kernel instance (oo_gpu_rx_set_len_hint);
    # timed without it too.
    ms_nohint = _timed(torch, run, steps, warmup)
    stack.set_len_hint(int(round(float(lens.mean()))))
    ms = _timed(torch, run, steps, warmup)
    stack.set_len_hint(0)
    same = bool(torch.equal(out, ref_out)) and bool((desc["intf_i"] == intf).all())
    bpp = float(lens.mean()) + DESC_B + RESULT_B
    gbs = n * bpp / (ms * 1e-3) / 1e9
    return {"kernel_ms": round(ms, 5), "kernel_ms_without_len_hint": round(ms_nohint, 5),
            "mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "achieved_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "umem_bytes": int(d_umem.numel()), "headroom": headroom,
            "records_equal_descriptor_path": same}


def _pinned_aligned(nbytes):
    """nbytes of host memory on whole pages of its own (an anonymous mmap,
    unmapped when the array goes): what oo_gpu_rx_host_register takes."""
    m = mmap.mmap(-1, max(1, -(-nbytes // mmap.PAGESIZE)) * mmap.PAGESIZE)
    return np.frombuffer(m, dtype=np.uint8, count=nbytes)


def time_xdp_host(torch, stack, buf, desc, ref_out, dev, sh, reps=5, headroom=192):
    """Zero-copy AF_XDP ingest: UMEM (chunk 2048,
    headroom 192: tcp_helper_resource.c:137, 2205-2208) and ring in
    registered host memory, read by the kernel in place over PCIe; records
    must equal the descriptor path's.  Rate = frames per kernel time;
    PCIe-bound (never `value`)."""
    n = len(desc)
    lens = desc["len"].astype(np.int64)
    size = int(((headroom + lens + 2047) // 2048).sum()) * 2048
    umem, addr, lens = _umem_layout(buf, desc, headroom, out=_pinned_aligned(size))
    cons = (1 << 32) - 77
    ring0, mask = _ring(addr, lens, cons)
    ring = _pinned_aligned(ring0.nbytes).view(ring0.dtype)
    ring[:] = ring0
    d_umem = stack.host_register(umem)
    d_ring = stack.host_register(ring)
    out = torch.empty_like(ref_out)
    intf = int(desc["intf_i"][0]) if n else 0

    def run():
        stack.xdp_dev(d_umem, umem.nbytes, d_ring, mask, cons, n, intf, out.data_ptr(), 0, sh)
    ms = _timed(torch, run, reps, 1)
    same = bool(torch.equal(out, ref_out))
    stack.host_unregister(ring)
    stack.host_unregister(umem)
    frame_bytes = float(lens.sum())
    return {"kernel_ms": round(ms, 3), "mpps": round(n / (ms * 1e-3) / 1e6, 2),
            "pcie_GBps": round((frame_bytes + 16 * n) / (ms * 1e-3) / 1e9, 2),
            "umem_bytes": int(umem.nbytes), "headroom": headroom,
            "records_equal_descriptor_path": same}


def time_pipelined(torch, stack, frames, d_desc, n, mean_len, out, dev, stream, steps, warmup):
    """Consecutive batches alternating over two streams (each its own result
    buffer): a batch's launch no longer waits for the previous one to drain,
    so the next batch's blocks take the CUs as the previous batch's last
    waves finish, and the launch gap overlaps. Region / K over both streams;
    a side measurement (a kernel's own duration is no longer region / K)."""
    s2 = torch.cuda.Stream(dev)
    out2 = torch.empty_like(out)
    streams = (stream, s2)
    bufs = (out, out2)

    def run(k):
        for i in range(k):
            st = streams[i & 1]
            stack.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                                      bufs[i & 1].data_ptr(), 0, st.cuda_stream)

    run(warmup)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    s2.wait_event(ev0)
    run(steps)
    join = torch.cuda.Event()
    join.record(s2)
    stream.wait_event(join)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    ms = float(ev0.elapsed_time(ev1)) / steps
    gbs = (mean_len + DESC_B + RESULT_B) * n / (ms * 1e-3) / 1e9
    stack.stream_done(s2.cuda_stream)  # the context stops tracking s2 before it goes
    return {"ms_per_batch": round(ms, 5), "mpps": round(n / (ms * 1e-3) / 1e6, 2),
            "achieved_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "streams": 2}


def time_table_ops(torch, filters, socks, frames, d_desc, n, out, device, reps=5):
    """Device-side table maintenance: the flush of a
    whole world load (every socket record and filter insert: the ops the
    stack's start-up queues), and a churn batch of 100 ops (50 filters
    removed and re-inserted) flushed in front of one batch, against the
    batch alone.  Event-timed on the stream; a side measurement."""
    from onload_amd.rx import GpuRxStack
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return float(e0.elapsed_time(e1))

    loads = []
    for _ in range(reps):
        g = GpuRxStack(device=device)
        g.load_world(filters, socks)  # queued on the host
        loads.append(timed(lambda: g.sync(sh)))
        g.close()
    g = GpuRxStack(device=device)
    g.load_world(filters, socks)
    g.sync(sh)

    def batch():
        g.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                              out.data_ptr(), 0, sh)

    def churn():
        for f in churn_f:
            ra = None if f.raddr_any else bytes(f.raddr)[:4]
            g.filter_remove_raw(f.sock, 4, bytes(f.laddr)[:4], f.lport_be, ra, f.rport_be, f.proto)
        for f in churn_f:
            ra = None if f.raddr_any else bytes(f.raddr)[:4]
            g.filter_insert_raw(f.sock, 4, bytes(f.laddr)[:4], f.lport_be, ra, f.rport_be, f.proto)

    def churn_and_batch():
        churn()
        batch()
    churn_f = [f for f in filters if f.af == 4][:50]
    for _ in range(3):
        batch()
    alone = sorted(timed(batch) for _ in range(reps))
    # (a) as rounds 3-4 measured it: the host calls between the events (the
    # stream idles while the caller makes them)
    with_churn = sorted(timed(churn_and_batch) for _ in range(reps))
    # (b) the device's share: the 100 ops queued first (host time reported
    # apart), then the events around the batch that flushes them
    dev, host_us = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        churn()
        host_us.append((time.perf_counter() - t) * 1e6 / (2 * len(churn_f)))
        dev.append(timed(batch))
    st = g.table_stats()
    g.close()
    return {"world_ops": len(filters) + len(socks), "world_flush_ms": round(sorted(loads)[reps // 2], 4),
            "churn_ops": 2 * len(churn_f), "batch_ms": round(alone[reps // 2], 4),
            "churn_plus_batch_ms": round(with_churn[reps // 2], 4),
            "queued_churn_flush_plus_batch_ms": round(sorted(dev)[reps // 2], 4),
            "host_us_per_op": round(sorted(host_us)[reps // 2], 2),
            "index_updates": st["index_updates"], "index_rebuilds": st["index_rebuilds"]}


def time_host_path(torch, filters, socks, buf, desc, device, batch=1 << 16, reps=3):
    """The path from host memory (NIC ring -> socket): frames and
    descriptors in registered host memory, oo_gpu_rx_submit / _wait over
    batches of `batch` packets, two in flight (H2D of one beside the
    transform of the other), records landing in registered host memory.
    Rate over the whole stream, PCIe-inclusive (never `value`)."""
    from onload_amd import _abi
    from onload_amd.rx import GpuRxStack
    n = len(desc)
    batch = min(batch, n)
    starts = list(range(0, n, batch))
    ends = [min(s + batch, n) for s in starts]
    spans = [(int(desc["frame_off"][s]),
              int(desc["frame_off"][e - 1]) + int(desc["len"][e - 1])) for s, e in zip(starts, ends)]
    cap = max(b - a for a, b in spans)
    hb = _pinned_aligned(buf.nbytes)
    hb[:] = buf
    hd = _pinned_aligned(desc.nbytes).view(_abi.DESC_DTYPE)
    hd[:] = desc
    for (s, e), (a, _) in zip(zip(starts, ends), spans):
        hd["frame_off"][s:e] -= a  # each batch's offsets relative to its first frame
    ho = _pinned_aligned(n * RESULT_B).view(_abi.RESULT_DTYPE)
    g = GpuRxStack(device=device, host_stage_bytes=cap, host_stage_pkts=batch)
    g.load_world(filters, socks)
    for arr in (hb, hd, ho):
        g.host_register(arr)
    times = []
    for r in range(reps + 1):
        t = time.perf_counter()
        pending = []
        for (s, e), (a, b) in zip(zip(starts, ends), spans):
            if len(pending) == 2:
                g.wait(pending.pop(0))
            pending.append(g.submit(hb[a:b], hd[s:e], ho[s:e]))
        for tk in pending:
            g.wait(tk)
        if r:
            times.append(time.perf_counter() - t)
    s = float(np.median(times))
    byt = buf.nbytes + desc.nbytes + n * RESULT_B
    res = {"mpps": round(n / s / 1e6, 2), "gbs_pcie": round(byt / s / 1e9, 2),
           "ms": round(s * 1e3, 3), "batch_pkts": batch, "in_flight": 2,
           "registered": True}
    for arr in (hb, hd, ho):
        g.host_unregister(arr)
    g.close()
    return res


def cpu_baseline(filters, socks, buf, desc, seconds):
    """The CPU restatement of the reference path (oracle/rx_oracle.c, pinned
    by tests/golden) on every host core this process may use, one thread per
    core over contiguous shards of a bounded sample of the same frames."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from onload_amd.shards import host_cores
    from oracle_lib import OracleStack
    threads = host_cores()
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
            "label": f"Onload CPU-path semantics (restated, fixture-verified), {threads} cores",
            "sample": f"first {sample} frames of the same workload, repeated for {el:.1f}s "
                      f"({threads} threads, contiguous shards)"}


if __name__ == "__main__":
    sys.exit(main())
