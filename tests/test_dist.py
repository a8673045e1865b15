# SPDX-License-Identifier: BSD-2-Clause
"""The N>1 path of bench.py on CPU (gloo, world_size 2), through the same
helpers the GPU run uses (onload_amd/shards.py):

* shards: contiguous ranges covering the stream exactly, byte-balanced for
  the mixed-size configurations;
* the table image broadcast from rank 0 replicates its tables on rank 1,
  and incremental op batches from rank 0 keep them identical;
* per-rank records gathered to rank 0 equal one unsharded run, bit for bit;
* the frame scatter delivers each rank its own shard;
* bench.py --gpus N starts N ranks itself (WORLD_SIZE=N, before anything
  initialises a GPU) and refuses a --gpus that disagrees with WORLD_SIZE."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from onload_amd import pktgen, shards

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, config, n_total, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from onload_amd.rx import GpuRxStack
    from oracle_lib import OracleStack, counters_of
    seed = pktgen.default_seed(config)
    first, n = shards.shard_for(config, seed, n_total, rank, world)
    filters, socks = pktgen.world(config)
    # tables: built on rank 0 only, replicated by the image broadcast
    st = GpuRxStack(device=-1)
    if rank == 0:
        st.load_world(filters, socks)
    shards.broadcast_tables(st, torch, dist, "cpu", 0)
    img = torch.from_numpy(st.image_host())
    ref = img.clone()
    dist.broadcast(ref, src=0)
    same_tables = bool(torch.equal(img, ref))
    # records of this rank's shard, gathered to rank 0
    o = OracleStack()
    o.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n, first=first, nthreads=2)
    res = o.handle_rx_batch(buf, desc)
    ctr = torch.from_numpy(counters_of(res).astype(np.int64))
    dist.all_reduce(ctr)
    recs = shards.gather_records(torch.from_numpy(res.view(np.uint8).copy()), n, torch, dist, 0)
    # frames scattered from rank 0
    slab = torch.tensor([buf.nbytes], dtype=torch.int64)
    dist.all_reduce(slab, op=dist.ReduceOp.MAX)
    src = None
    if rank == 0:
        src = []
        for r in range(world):
            f, c = shards.shard_for(config, seed, n_total, r, world)
            src.append(torch.from_numpy(pktgen.generate(config, c, first=f, nthreads=2)[0]))
    got = shards.scatter_frames(src, int(slab.item()), torch, dist, "cpu", 0)
    scatter_ok = torch.tensor([int(np.array_equal(got[: buf.nbytes].numpy(), buf))])
    dist.all_reduce(scatter_ok, op=dist.ReduceOp.MIN)
    tables_ok = torch.tensor([int(same_tables)])
    dist.all_reduce(tables_ok, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put((ctr.numpy(), recs.numpy().tobytes(), int(scatter_ok.item()),
               int(tables_ok.item()), img.numpy().tobytes()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config", [2, 5])
def test_two_rank_shards_equal_one_run(config):
    n_total = 3001  # uneven split on purpose
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, config, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    ctr, recs, scatter_ok, tables_ok, img = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert scatter_ok == 1 and tables_ok == 1
    from onload_amd.rx import GpuRxStack
    from oracle_lib import OracleStack, counters_of
    filters, socks = pktgen.world(config)
    st = GpuRxStack(device=-1)
    st.load_world(filters, socks)
    assert img == st.image_host().tobytes()  # rank 1's replica is rank 0's tables
    o = OracleStack()
    o.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n_total, nthreads=2)
    want = o.handle_rx_batch(buf, desc)
    assert recs == want.tobytes()
    np.testing.assert_array_equal(ctr, counters_of(want))


def _ops_worker(rank, world, port, q):
    """Image broadcast after the first part of a table script, then the rest
    of it as incremental op batches from rank 0 (shards.broadcast_ops)."""
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import table_scripts as ts
    from onload_amd.rx import GpuRxStack
    cfg, socks, ops = ts.build("mixed")
    ops = [o for o in ops if o[0] in "AR"]
    kind = {"A": "insert", "R": "remove"}
    st = GpuRxStack(device=-1, max_socks=1024, ip4_log2=cfg["log4"], ip6_log2=cfg["log6"],
                    intf_hwport=cfg["hwports"])
    half = len(ops) // 2
    rcs0 = []
    if rank == 0:  # rank 0 owns the sockets and the first half of the ops
        rcs0 = ts.replay(st, socks, ops, upto=half)
    shards.broadcast_tables(st, torch, dist, "cpu", 0)
    rcs = []
    for at in range(half, len(ops), 500):  # the rest in batches, socket churn between
        batch = [(kind[o[0]], o[2], o[1], o[3], o[4], o[5], o[6], o[7]) for o in ops[at:at + 500]]
        s = socks[(at // 500) % len(socks)]
        s.hwports ^= 1
        batch.append(("sock", s.id, ts.sock_struct(s)))
        rcs += shards.broadcast_ops(st, batch if rank == 0 else None, torch, dist, "cpu", 0)
    img = torch.from_numpy(st.image_host())
    ref = img.clone()
    dist.broadcast(ref, src=0)
    got_rcs = torch.tensor(rcs, dtype=torch.int64)
    ref_rcs = got_rcs.clone()
    dist.broadcast(ref_rcs, src=0)
    same = torch.tensor([int(torch.equal(img, ref) and torch.equal(got_rcs, ref_rcs))])
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put((int(same.item()), rcs0 + rcs, img.numpy().tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_incremental_table_ops_keep_ranks_identical():
    """the replicated tables are kept current with incremental
    updates -- after the image broadcast, op batches from rank 0 leave both
    ranks' tables byte-identical, and equal to one stack that applied the
    whole script itself (return codes included)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ops_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    same, rcs, img = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same == 1
    import table_scripts as ts
    from onload_amd.rx import GpuRxStack
    cfg, socks, ops = ts.build("mixed")
    ops = [o for o in ops if o[0] in "AR"]
    st = GpuRxStack(device=-1, max_socks=1024, ip4_log2=cfg["log4"], ip6_log2=cfg["log6"],
                    intf_hwport=cfg["hwports"])
    half = len(ops) // 2
    want = ts.replay(st, socks, ops, upto=half)
    for at in range(half, len(ops), 500):
        want += ts.replay(st, [], ops[at:at + 500])
        s = socks[(at // 500) % len(socks)]
        s.hwports ^= 1
        want.append(st.sock_set(s.id, ts.sock_struct(s)))
    assert rcs == want
    assert img == st.image_host().tobytes()
    assert any(rc != 0 for rc in want)  # the script reaches -ENOBUFS / -ENOENT paths


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 1 << 20, 12345):
        for w in (1, 2, 3, 8):
            spans = [shards.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0
            assert sum(s[1] for s in spans) == n
            for a, b in zip(spans, spans[1:]):
                assert a[0] + a[1] == b[0]


@pytest.mark.parametrize("config,n_total,world", [(5, 200000, 8), (4, 50000, 3), (5, 17, 4)])
def test_byte_balanced_shards(config, n_total, world):
    """Mixed-size traffic: contiguous ranges, equal packed bytes within one
    frame's worth."""
    seed = pktgen.default_seed(config)
    spans = shards.split_bytes(config, seed, n_total, world)
    assert spans[0][0] == 0 and sum(c for _, c in spans) == n_total
    for a, b in zip(spans, spans[1:]):
        assert a[0] + a[1] == b[0]
    per = [pktgen.nbytes(config, seed, f, c) for f, c in spans]
    total = pktgen.nbytes(config, seed, 0, n_total)
    assert sum(per) == total
    if n_total > 1000:
        assert max(per) - min(per) <= 2 * 9088, per  # within about one jumbo frame
        # count-split would be far less even for config 4 / 5
        counts = [pktgen.nbytes(config, seed, *shards.shard_range(n_total, r, world))
                  for r in range(world)]
        assert max(per) - min(per) <= max(counts) - min(counts)


def _bench(args, env):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, env=env, timeout=300)


def test_bench_launches_ranks_before_gpu_use():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OO_BENCH_PROBE"] = "1"
    r = _bench(["--gpus", "3", "--steps", "1"], env)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2]
    assert all(x["world"] == 3 and x["local_rank"] == x["rank"] for x in lines)
    assert not any(x["cuda_initialized"] for x in lines)


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", OO_BENCH_PROBE="1")
    r = _bench(["--gpus", "4"], env)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_launcher_stops_all_ranks_when_one_dies(tmp_path):
    """The rank launcher's watchdog: rank 1 of 3 dies while the other two
    block (as they would in a barrier or an RCCL collective); the launcher
    terminates them and returns rank 1's status within a bound, instead of
    hanging until an outer timeout."""
    import time
    import bench
    script = tmp_path / "rank.py"
    pids = tmp_path / "pids"
    pids.mkdir()
    script.write_text(
        "import os, sys, time\n"
        f"open(os.path.join({str(pids)!r}, os.environ['RANK']), 'w').write(str(os.getpid()))\n"
        "if os.environ['RANK'] == '1':\n"
        "    time.sleep(0.5)\n"
        "    sys.exit(7)\n"
        "time.sleep(120)\n")
    t = time.time()
    rc = bench.launch_ranks(3, [], script=str(script), grace_s=5.0)
    assert rc == 7
    assert time.time() - t < 30
    for r in ("0", "2"):  # the blocked ranks are gone
        pid = int((pids / r).read_text())
        try:
            os.kill(pid, 0)
            alive = os.path.exists(f"/proc/{pid}") and "Z" not in open(f"/proc/{pid}/stat").read().split()[2]
        except ProcessLookupError:
            alive = False
        assert not alive, f"rank {r} still running"
