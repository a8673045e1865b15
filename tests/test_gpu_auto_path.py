# SPDX-License-Identifier: BSD-2-Clause
"""The launch choice without a caller hint (oo_gpu_rx.cpp launch()): after a
batch's descriptors have been seen once, their sampled length profile picks
the kernels -- config 4's mixed IPv4/TCP sizes the split transform with the
sequences body engine (last_path 4), config 2's uniform 1514-B frames and
config 5's IMIX the one-kernel instances (1 and 2).  Records are bit-exact
with the oracle on both launches."""
import numpy as np
import pytest

from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack, counters_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.mark.parametrize("config,n,first_path,then_path", [(4, 1 << 16, 1, 4), (2, 1 << 16, 1, 1),
                                                           (5, 1 << 16, 2, 2)])
def test_sampled_profile_picks_the_kernels(cuda, config, n, first_path, then_path):
    torch = cuda
    filters, socks = pktgen.world(config)
    g = GpuRxStack(device=0)
    g.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n, first=99)
    frames = torch.from_numpy(buf).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8)).cuda()
    o = OracleStack()
    o.load_world(filters, socks)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    sh = torch.cuda.current_stream().cuda_stream
    paths = []
    for _ in range(2):
        out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        ctr = torch.zeros(32, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        g.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                              out.data_ptr(), ctr.data_ptr(), sh)
        torch.cuda.synchronize()  # (the sample lands with the batch)
        paths.append(g.last_path())
        got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
        assert got.tobytes() == want.tobytes()
        assert (ctr.cpu().numpy().view(np.uint32)[:_abi.R_COUNT] == counters_of(want)).all()
    assert paths == [first_path, then_path]
    # a caller's hint wins over the profile: the one-kernel instance
    g.set_len_hint(1809)
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    g.handle_rx_batch_dev(frames.data_ptr(), frames.numel(), d_desc.data_ptr(), n,
                          out.data_ptr(), 0, sh)
    torch.cuda.synchronize()
    assert g.last_path() == 1
    g.close()
