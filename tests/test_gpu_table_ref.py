# SPDX-License-Identifier: BSD-2-Clause
"""The device side of the filter tables pinned against the reference's own
netif_table.c / netif_table_ip6.c (fixtures of tests/golden/
make_table_golden.py): the table scripts are applied by the device table
kernels (oo_table_kernel.hip, queued ops on the batch stream), the device
tables exported at each checkpoint must equal the reference's table row for
row (or by digest), and the rx kernel's demux of a frame per packet-shaped
query must give the reference walks' deciding stage, first socket, match
count and hash3 (netif_table.c:234-319, netif_table_ip6.c:110-189)."""
import numpy as np
import pytest

import table_scripts as ts
from frames import pack
from gpu_util import run_dev
from onload_amd.rx import GpuRxStack
from test_table_ref import GOLDEN, _stack_kw

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _device_rows(torch, g):
    img = torch.zeros(g.image_bytes(), dtype=torch.uint8, device="cuda")
    g.table_export(img.data_ptr(), img.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return ts.image_rows(img.cpu().numpy())


@pytest.mark.parametrize("name", list(ts.SCRIPTS))
def test_device_tables_match_reference(cuda, name):
    golden = np.load(GOLDEN)
    cfg, socks, ops = ts.build(name)
    g = GpuRxStack(device=0, **_stack_kw(name))

    def at(k, i):
        ts.check_dump(_device_rows(cuda, g), golden, name, k)
        _, matches = ts.queries(name, socks, ts.live_at(ops, i), k)
        buf, desc = pack([(ts.frame_for(q), q[6]) for q in matches])
        rec, _ = run_dev(g, buf, desc)
        want = ts.expected_records(matches, golden[f"{name}/match{k}"])
        for j, (r, w) in enumerate(zip(rec, want)):
            got = (int(r["stage"]), int(r["sock"]), int(r["nmatch"]), int(r["hash3"]))
            assert got == w, (j, matches[j], got, w)

    rcs = ts.replay(g, socks, ops, at)
    np.testing.assert_array_equal(np.array(rcs, np.int32), golden[f"{name}/rc"])
    g.close()
