# SPDX-License-Identifier: BSD-2-Clause
"""The multi-GPU group on one GPU, as a rehearsal: three members on device 0
(a device may repeat), the tables built through the group, a configuration
batch split by bytes, each member transforming its share on its own stream
(oo_gpu_rx_group_process), the records gathered in member order
(oo_gpu_rx_group_gather) -- bit-exact with the unsharded oracle, counters
summed."""
import numpy as np
import pytest

from onload_amd import _abi, pktgen
from onload_amd.group import GpuRxGroup, Shard
from oracle_lib import OracleStack, counters_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.mark.parametrize("config,n", [(5, 40000), (2, 20000), (4, 12000)])
def test_group_of_three_on_one_gpu_matches_unsharded_oracle(cuda, config, n):
    torch = cuda
    filters, socks = pktgen.world(config)
    g = GpuRxGroup(devices=[0, 0, 0])
    g.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n)
    shares = g.split(desc)
    frames = torch.from_numpy(buf).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    outs, ctrs, streams, shards = [], [], [], []
    for (f, c) in shares:
        outs.append(torch.zeros(max(c, 1) * 32, dtype=torch.uint8, device="cuda"))
        ctrs.append(torch.zeros(32, dtype=torch.int32, device="cuda"))
        streams.append(torch.cuda.Stream())
        shards.append(Shard(frames.data_ptr(), frames.numel(), d_desc.data_ptr() + 16 * f, c, 0,
                            outs[-1].data_ptr(), ctrs[-1].data_ptr(),
                            streams[-1].cuda_stream))
    dst = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    # the buffers were filled on torch's stream; the shards' streams are not
    # ordered after it (as with any caller's streams)
    torch.cuda.synchronize()
    g.process(shards)
    counters = np.zeros(32, dtype=np.uint32)
    g.gather(shards, dst.data_ptr(), counters)
    got = dst.cpu().numpy().view(_abi.RESULT_DTYPE)
    o = OracleStack()
    o.load_world(filters, socks)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    assert got.tobytes() == want.tobytes()
    assert (counters == counters_of(want)).all()
    for m, s in zip(g.members, streams):
        m.stream_done(s.cuda_stream)
    g.close()
