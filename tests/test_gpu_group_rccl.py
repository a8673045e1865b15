# SPDX-License-Identifier: BSD-2-Clause
"""The across-processes group (oo_gpu_rx_group_join) run for real on one
GPU: a group of one rank whose every collective goes through librccl -- the
op broadcast in chunks (config 5's world is 11,936 queued changes: more than
one chunk), the table-image broadcast, the records gathered by a send/receive
pair to itself, the counters summed by an all-reduce -- bit-exact with the
oracle.  The same calls a rank of an 8-GPU job makes (bench.py --gpus N);
only the peers are missing."""
import numpy as np
import pytest

from onload_amd import _abi, pktgen
from onload_amd.group import GpuRxGroup
from oracle_lib import OracleStack, counters_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def test_one_rank_group_runs_every_rccl_leg(cuda):
    torch = cuda
    config, n = 5, 40000
    filters, socks = pktgen.world(config)
    g = GpuRxGroup.join(0, 0, 1, GpuRxGroup.rccl_id())
    assert g.uses_rccl and g.rank == 0
    g.load_world(filters, socks)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    queued = len(filters) + len(socks)
    assert queued > 8192  # more than one broadcast chunk
    assert g.share_ops(sh) == queued
    assert g.share_ops(sh) == 0  # the queue was emptied
    g.share_tables(sh)
    m = g.members[0]
    buf, desc = pktgen.generate(config, n)
    frames = torch.from_numpy(buf).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(32, dtype=torch.int32, device="cuda")
    m.sync(sh)
    m.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                          out.data_ptr(), ctr.data_ptr(), sh)
    g.sum_counters(ctr.data_ptr(), sh)
    dst = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    g.gather_rccl(out.data_ptr(), n, dst.data_ptr(), [n], sh)
    torch.cuda.synchronize()
    o = OracleStack()
    o.load_world(filters, socks)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    got = dst.cpu().numpy().view(_abi.RESULT_DTYPE)
    assert got.tobytes() == want.tobytes()
    assert (ctr.cpu().numpy().view(np.uint32)[:len(counters_of(want))] == counters_of(want)).all()
    # a change after the image: queued, shared, the batch sees it
    f = filters[0]
    ra = None if f.raddr_any else bytes(f.raddr)[: 4 if f.af == 4 else 16]
    la = bytes(f.laddr)[: 4 if f.af == 4 else 16]
    assert g.filter_remove_raw(f.sock, f.af, la, f.lport_be, ra, f.rport_be, f.proto) == 0
    assert g.share_ops(sh) == 1
    g.close()


def test_one_rank_group_rejects_a_bad_count(cuda):
    torch = cuda
    g = GpuRxGroup.join(0, 0, 1, GpuRxGroup.rccl_id())
    out = torch.zeros(64 * 32, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(64 * 32, dtype=torch.uint8, device="cuda")
    with pytest.raises(OSError):
        g.gather_rccl(out.data_ptr(), 64, dst.data_ptr(), [63], 0)
    g.close()
