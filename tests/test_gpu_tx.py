# SPDX-License-Identifier: BSD-2-Clause
"""TX checksum fill on the GPU (oo_gpu_tx_fill_dev) against the reference's
golden frames and the oracle, bit for bit over whole frame buffers."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from frames import edge_frames, pack  # noqa: E402
from oracle_lib import oracle_tx_fill, tx_golden  # noqa: E402

from onload_amd import _abi, pktgen  # noqa: E402
from onload_amd.rx import GpuRxStack  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stack():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return GpuRxStack(device=0)


def gpu_fill(stack, buf: np.ndarray, desc: np.ndarray) -> np.ndarray:
    import torch
    fr = torch.from_numpy(np.ascontiguousarray(buf)).to("cuda")
    de = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8)).to("cuda")
    stack.tx_fill_dev(fr.data_ptr(), fr.numel(), de.data_ptr(), len(desc),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return fr.cpu().numpy()


def _same(got, want):
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"


def test_tx_golden_on_gpu(stack):
    fin, fout, desc = tx_golden()
    _same(gpu_fill(stack, fin, desc), fout)


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 8, 15])
def test_tx_edge_corpus(stack, shift):
    """Every RX edge frame (VLAN, options, IPv6, bad lengths, fragments, odd
    sizes) filled at every alignment; odd offsets exercise the byte swap."""
    buf, desc = pack(edge_frames(), align=64 if shift % 2 == 0 else 16, shift=shift)
    _same(gpu_fill(stack, buf, desc), oracle_tx_fill(buf, desc))


@pytest.mark.parametrize("config,n", [(2, 1 << 15), (4, 1 << 13), (5, 1 << 15), (3, 1 << 16)])
def test_tx_config_samples(stack, config, n):
    buf, desc = pktgen.generate(config, n, first=999)
    _same(gpu_fill(stack, buf, desc), oracle_tx_fill(buf, desc))


def test_tx_full_size_config2_then_rx(stack):
    """2^20 frames filled on the GPU equal the oracle's fill, and the RX
    transform then finds no checksum failures."""
    import torch

    from gpu_util import run_dev
    n = 1 << 20
    filters, socks = pktgen.world(2)
    buf, desc = pktgen.generate(2, n)
    got = gpu_fill(stack, buf, desc)
    _same(got, oracle_tx_fill(buf, desc))
    g = GpuRxStack(device=0)
    g.load_world(filters, socks)
    res, ctr = run_dev(g, got, desc)
    for r in (_abi.R_IP4_CSUM, _abi.R_UDP_CSUM, _abi.R_TCP_CSUM):
        assert ctr[r] == 0
    torch.cuda.synchronize()


def test_tx_wrapping_descriptors_write_nothing_outside(stack):
    """Descriptors with offsets near 2^64 (offset + length wraps) and ones
    running past the buffer are left alone: no byte outside the frame buffer
    and no other frame changes."""
    import torch
    buf, desc = pack(edge_frames()[:64], align=64)
    n = len(buf)
    desc[2]["frame_off"] = (1 << 64) - 64
    desc[2]["len"] = 64
    desc[3]["frame_off"] = (1 << 64) - 16
    desc[4]["frame_off"] = n - 8
    guard = 1 << 16
    big = np.full(n + 2 * guard, 0x5A, dtype=np.uint8)
    big[guard:guard + n] = buf
    d = torch.from_numpy(big).to("cuda")
    de = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8)).to("cuda")
    stack.tx_fill_dev(d.data_ptr() + guard, n, de.data_ptr(), len(desc),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    assert (got[:guard] == 0x5A).all() and (got[guard + n:] == 0x5A).all()
    _same(got[guard:guard + n], oracle_tx_fill(buf, desc))
