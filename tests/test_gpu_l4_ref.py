# SPDX-License-Identifier: BSD-2-Clause
"""The gfx950 records against the reference's own receive path
(tests/l4_ref.py, tests/golden/ref_l4_golden.npz): gates, L4 entry, lookup
stages, sockets, pass-to-kernel decisions and the UDP / TCP future sockets
the reference's handle_rx_csum_bad / handle_rx_pkt / ci_{udp,tcp}_handle_rx /
pre-future helpers computed for the same frames -- directly, not through the
oracle."""
import numpy as np
import pytest

import l4_ref
from frames import pack
from gpu_util import run_dev
from onload_amd.rx import GpuRxStack
from test_oracle_l4_ref import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.mark.parametrize("name", l4_ref.CORPORA)
@pytest.mark.parametrize("kernel", (0, 1, 2, 3))
def test_gpu_matches_reference_run(cuda, monkeypatch, name, kernel):
    # 0: auto, 1 / 2: the single-kernel
    # instances, 3: the split transform (win_kernel + body_kernel)
    monkeypatch.setenv("OO_RX_KERNEL", str(kernel))
    out, sha = l4_ref.load(np.load(GOLDEN), name)
    socks, filters, hwports, frames = l4_ref.corpus(name)
    assert l4_ref.frames_sha(frames) == sha
    g = GpuRxStack(device=0, intf_hwport=hwports)
    for i, s in socks.items():
        assert g.sock_set(i, s) == 0
    for (i, af, la, lp, ra, rp, proto) in filters:
        assert g.filter_insert_raw(i, af, la, lp, ra, rp, proto) == 0
    buf, desc = pack(frames)
    recs, _ = run_dev(g, buf, desc)
    g.close()
    bad = l4_ref.mismatches(recs, out)
    assert not bad, "\n".join(bad)
    obs, stats = l4_ref.load_stats(np.load(GOLDEN), name)
    bad = l4_ref.stats_mismatches(recs, obs, stats)
    assert not bad, "\n".join(bad)
