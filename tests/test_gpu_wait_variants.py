# SPDX-License-Identifier: BSD-2-Clause
"""The kernel's static vmcnt waits under other pipeline constants.

rx_kernel / tx_kernel wait for their LDS-DMA rounds with counted
`s_waitcnt vmcnt(N)`, N written in terms of the ring size R, the extra
header-row rounds E, the staging operations per tile and the stores per tile
(oo_rx_kernel.hip).  `make` also builds the same sources with other values
(build/check/, Makefile CHECK_VARIANTS: R 6 / E 4, R 8 / E 2, one wave per
block with E 0); each build is loaded beside the product (its own soname) and
must stay bit-exact with the oracle -- a count that does not follow its
constants shows up here as wrong sums, not only when the product's values
change.  The split transform's body ring (RB, oo_rx_kernel.hip body_loop)
has its own builds (rb6, rb12 -- the latter with win_kernel at three waves
per SIMD), run through the split path (OO_RX_KERNEL 3)."""
import os

import numpy as np
import pytest

from frames import edge_frames, edge_world, install, pack
from gpu_util import diff_report, run_dev
from oracle_lib import OracleStack, counters_of, oracle_tx_fill
from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = ("r6e4", "r8e2", "w1e0")
SPLIT_VARIANTS = ("rb6", "rb12")
HWPORTS = (0, 1, 3, 2, 5)
_libs: dict = {}


def _lib(name):
    if name not in _libs:
        path = os.path.join(ROOT, "build", "check", f"liboo_gpu_rx_{name}.so")
        assert os.path.exists(path), f"{path} missing: run make (the check builds are part of all)"
        _libs[name] = _abi.bind_library(path)
    return _libs[name]


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _check(g, o, buf, desc):
    got, ctr = run_dev(g, buf, desc)
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    assert got.tobytes() == want.tobytes(), diff_report(got, want, desc)
    np.testing.assert_array_equal(ctr, counters_of(want))


@pytest.mark.parametrize("variant", VARIANTS + SPLIT_VARIANTS)
def test_variant_edge_corpus(cuda, variant, monkeypatch):
    if variant in SPLIT_VARIANTS:
        monkeypatch.setenv("OO_RX_KERNEL", "3")
    g = GpuRxStack(device=0, intf_hwport=HWPORTS, lib=_lib(variant))
    o = OracleStack(intf_hwport=HWPORTS)
    install(g, edge_world())
    install(o, edge_world())
    for shift in (0, 3):
        buf, desc = pack(edge_frames(), align=64 if shift % 2 == 0 else 16, shift=shift)
        _check(g, o, buf, desc)


@pytest.mark.parametrize("variant", VARIANTS + SPLIT_VARIANTS)
@pytest.mark.parametrize("config,n", [(2, 1 << 14), (3, 1 << 16), (4, 1 << 13), (5, 1 << 15)])
def test_variant_config_samples(cuda, variant, config, n, monkeypatch):
    if variant in SPLIT_VARIANTS:
        monkeypatch.setenv("OO_RX_KERNEL", "3")
    filters, socks = pktgen.world(config)
    g = GpuRxStack(device=0, lib=_lib(variant))
    o = OracleStack()
    g.load_world(filters, socks)
    o.load_world(filters, socks)
    buf, desc = pktgen.generate(config, n, first=777 * config)
    _check(g, o, buf, desc)


@pytest.mark.parametrize("variant", VARIANTS)
def test_variant_tx_fill(cuda, variant):
    torch = cuda
    g = GpuRxStack(device=0, lib=_lib(variant))
    buf, desc = pktgen.generate(4, 1 << 12, first=99)
    want = oracle_tx_fill(buf, desc)
    fr = torch.from_numpy(np.ascontiguousarray(buf)).to("cuda")
    de = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8)).to("cuda")
    g.tx_fill_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), len(desc),
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = fr.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
