# SPDX-License-Identifier: BSD-2-Clause
"""The transform straight off an AF_XDP RX ring (oo_gpu_rx_xdp_dev /
oo_gpu_rx_xdp_poll; efxdp_ef_eventq_poll, efxdp_vi.c:309-358) against the
oracle's ring batch: bit-exact records, ring and u32 index wrap-around,
varying headroom, the 16-bit length, entries outside the UMEM."""
import numpy as np
import pytest

from frames import edge_frames, edge_world, install
from gpu_util import diff_report, to_dev
from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack, counters_of
from xdp_util import frames_of, ring_of, to_umem

pytestmark = pytest.mark.gpu

HWPORTS = (0, 1, 3, 2, 5)


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _pair(installer, **kw):
    g = GpuRxStack(device=0, **kw)
    o = OracleStack(**kw)
    installer(g)
    installer(o)
    return g, o


def _run(torch, g, umem, ring, mask, cons, n, intf):
    du, dr = to_dev(umem), to_dev(ring)
    out = torch.full((max(n, 1) * 32,), 0xAB, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(_abi.R_COUNT, dtype=torch.int32, device="cuda")
    g.xdp_dev(du.data_ptr(), du.numel(), dr.data_ptr(), mask, cons, n, intf, out.data_ptr(),
              ctr.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return (out.cpu().numpy()[: n * 32].view(_abi.RESULT_DTYPE),
            ctr.cpu().numpy().astype(np.uint32))


def _check(torch, g, o, umem, ring, mask, cons, n, intf):
    got, ctr = _run(torch, g, umem, ring, mask, cons, n, intf)
    want = o.handle_xdp_batch(umem, ring, mask, cons, n, intf)
    assert got.tobytes() == want.tobytes(), diff_report(got, want)
    np.testing.assert_array_equal(ctr, counters_of(want))
    return got


@pytest.mark.parametrize("log2,cons", [(12, 0), (12, 4090), (13, (1 << 32) - 100)])
@pytest.mark.parametrize("intf", [0, 2])
def test_edge_corpus_off_ring(cuda, log2, cons, intf):
    g, o = _pair(lambda s: install(s, edge_world()), intf_hwport=HWPORTS)
    frames = [f for f, _ in edge_frames()]
    umem, ents = to_umem(frames, seed=log2 + intf)
    ring, mask = ring_of(ents, log2, cons, seed=cons & 0xffff)
    got = _check(cuda, g, o, umem, ring, mask, cons, len(ents), intf)
    assert len(set(got["reason"].tolist())) >= 15


def test_length_bits_and_outside_entries(cuda):
    g, o = _pair(lambda s: install(s, edge_world()), intf_hwport=HWPORTS)
    frames = [f for f, _ in edge_frames(seed=7)][:200]
    umem, ents = to_umem(frames, seed=11, headroom=(0, 2048 - 64))
    ents["len"][::3] += np.uint32(1 << 16)
    ents["addr"][5] = umem.nbytes - 7
    ents["addr"][6] = (1 << 63) + 3
    ents["len"][7] = 0
    ents["addr"][8] = (1 << 64) - 64  # addr + len wraps u64
    ents["len"][8] = 64
    ents["addr"][9] = (1 << 64) - 2048 + 16
    ring, mask = ring_of(ents, 8, 77)
    _check(cuda, g, o, umem, ring, mask, 77, len(ents), 0)


@pytest.mark.parametrize("config,n", [(2, 1 << 14), (4, 1 << 12), (5, 1 << 14)])
def test_config_samples_off_ring(cuda, config, n):
    filters, socks = pktgen.world(config)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    buf, desc = pktgen.generate(config, n, first=999 * config)
    umem, ents = to_umem(frames_of(buf, desc), seed=config)
    cons = (1 << 32) - n // 3
    ring, mask = ring_of(ents, (n - 1).bit_length(), cons)
    got = _check(cuda, g, o, umem, ring, mask, cons, n, 0)
    assert (got["reason"] == _abi.R_DELIVER).mean() > 0.8


def test_poll_consumes_in_batches(cuda):
    """oo_gpu_rx_xdp_poll: min(producer - consumer, max_n) entries per call,
    the consumer published after each, records equal to one big batch."""
    torch = cuda
    filters, socks = pktgen.world(5)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    n = 3000
    buf, desc = pktgen.generate(5, n, first=31)
    umem, ents = to_umem(frames_of(buf, desc), seed=9)
    cons0 = (1 << 32) - 1000
    ring, mask = ring_of(ents, 12, cons0)
    want = o.handle_xdp_batch(umem, ring, mask, cons0, n, 1)
    du, dr = to_dev(umem), to_dev(ring)
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    consumer = np.array([cons0], dtype=np.uint32)
    producer = np.array([(cons0 + n) & 0xffffffff], dtype=np.uint32)
    stream = torch.cuda.current_stream().cuda_stream
    done, calls = 0, 0
    while True:
        got_n = g.xdp_poll(du.data_ptr(), du.numel(), dr.data_ptr(), mask, consumer, producer,
                           1024, 1, out.data_ptr() + 32 * done, 0, stream)
        if got_n == 0:
            break
        assert got_n == min(1024, n - done)
        done += got_n
        calls += 1
        assert int(consumer[0]) == (cons0 + done) & 0xffffffff
    assert done == n and calls == 3
    got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
    assert got.tobytes() == want.tobytes(), diff_report(got, want)


def test_ring_argument_errors(cuda):
    """-EINVAL for a mask that is not 2^k - 1 or more entries than the ring
    holds; n = 0 is a no-op; a poll with nothing produced consumes nothing."""
    import errno
    torch = cuda
    g = GpuRxStack(device=0)
    umem = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    ring = torch.zeros(16 * 8, dtype=torch.uint8, device="cuda")
    out = torch.zeros(32 * 8, dtype=torch.uint8, device="cuda")
    for mask, n in ((6, 1), (7, 9), (0xffffffff, 1)):
        with pytest.raises(OSError) as e:
            g.xdp_dev(umem.data_ptr(), umem.numel(), ring.data_ptr(), mask, 0, n, 0,
                      out.data_ptr())
        assert e.value.errno == errno.EINVAL
    g.xdp_dev(umem.data_ptr(), umem.numel(), ring.data_ptr(), 7, 5, 0, 0, out.data_ptr())
    cons = np.array([123], dtype=np.uint32)
    prod = np.array([123], dtype=np.uint32)
    assert g.xdp_poll(umem.data_ptr(), umem.numel(), ring.data_ptr(), 7, cons, prod, 8, 0,
                      out.data_ptr()) == 0
    assert int(cons[0]) == 123
    prod[0] = 125
    assert g.xdp_poll(umem.data_ptr(), umem.numel(), ring.data_ptr(), 7, cons, prod, 0, 0,
                      out.data_ptr()) == 0
    assert int(cons[0]) == 123
