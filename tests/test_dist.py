# SPDX-License-Identifier: BSD-2-Clause
"""The N>1 path of bench.py on CPU (gloo, world_size 2): each rank owns an
independent packet range (no data-path collective), outcomes aggregate by
all_reduce, and the union of the shards equals one unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from onload_amd import pktgen
from shard import shard_range


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
    from oracle_lib import OracleStack, counters_of
    first, n = shard_range(n_total, rank, world)
    filters, socks = pktgen.world(config)
    o = OracleStack()
    o.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n, first=first, nthreads=2)
    res = o.handle_rx_batch(buf, desc)
    ctr = torch.from_numpy(counters_of(res).astype(np.int64))
    dist.all_reduce(ctr)
    gathered = [None] * world
    dist.all_gather_object(gathered, res.tobytes())
    if rank == 0:
        q.put((ctr.numpy(), b"".join(gathered)))
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
    ctr, recs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle_lib import OracleStack, counters_of
    filters, socks = pktgen.world(config)
    o = OracleStack()
    o.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n_total, nthreads=2)
    want = o.handle_rx_batch(buf, desc)
    assert recs == want.tobytes()
    np.testing.assert_array_equal(ctr, counters_of(want))


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 1 << 20, 12345):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0
            assert sum(s[1] for s in spans) == n
            for a, b in zip(spans, spans[1:]):
                assert a[0] + a[1] == b[0]
