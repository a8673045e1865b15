# SPDX-License-Identifier: BSD-2-Clause
"""The host-memory boundary:

* oo_gpu_rx_submit / oo_gpu_rx_wait -- asynchronous batches from host
  memory through two pinned staging slots on two streams -- give the records
  and counters of the device-resident path, from pageable and from
  registered (hipHostRegister) buffers, with the ticket rules of the header;
* zero-copy AF_XDP ingest: a UMEM and RX ring in registered host memory read
  by the kernel directly (no copy), as efhw/af_xdp.c:463-500 registers the
  same UMEM with the kernel, chunk 2048 / headroom 192
  (tcp_helper_resource.c:137, 2205-2208); records equal the oracle's ring
  batch (efxdp_vi.c:309-358)."""
import errno

import numpy as np
import pytest

from gpu_util import diff_report, run_dev
from hostmem import page_buffer
from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack, counters_of
from xdp_util import frames_of, ring_of, to_umem

pytestmark = pytest.mark.gpu

PAGE = 4096


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def aligned(nbytes: int, dtype=np.uint8) -> np.ndarray:
    """A host array on pages of its own (hostmem.page_buffer: hipHostRegister
    works on whole pages)."""
    return page_buffer(nbytes, dtype)


def test_submit_wait_pageable_matches_device_path(cuda):
    filters, socks = pktgen.world(5)
    n = 8192
    batches = [pktgen.generate(5, n, first=n * k) for k in range(3)]
    cap = max(b.nbytes for b, _ in batches)
    g = GpuRxStack(device=0, host_stage_bytes=cap, host_stage_pkts=n)
    g.load_world(filters, socks)
    outs = [np.zeros(n, dtype=_abi.RESULT_DTYPE) for _ in batches]
    deltas = [np.zeros(_abi.R_COUNT, dtype=np.uint32) for _ in batches]
    # two in flight, waited out of order
    t0 = g.submit(batches[0][0], batches[0][1], outs[0], deltas[0])
    t1 = g.submit(batches[1][0], batches[1][1], outs[1], deltas[1])
    assert g.wait(t1) == n and g.wait(t0) == n
    # a third submit onto a slot whose batch was never waited for completes it
    t2 = g.submit(batches[2][0], batches[2][1], outs[2], deltas[2])
    spare = [np.zeros(n, _abi.RESULT_DTYPE) for _ in range(2)]  # alive until waited
    t3 = g.submit(batches[0][0], batches[0][1], spare[0])
    t4 = g.submit(batches[1][0], batches[1][1], spare[1])  # the slot of t2
    with pytest.raises(OSError) as e:
        g.wait(t2)
    assert e.value.errno == errno.ENOENT
    with pytest.raises(OSError) as e:
        g.wait(t0)  # already waited
    assert e.value.errno == errno.ENOENT
    g.wait(t3)
    g.wait(t4)
    assert spare[0].tobytes() == outs[0].tobytes() and spare[1].tobytes() == outs[1].tobytes()
    for (buf, desc), out, delta in zip(batches, outs, deltas):
        want, ctr = run_dev(g, buf, desc)
        assert out.tobytes() == want.tobytes(), diff_report(out, want, desc)
        np.testing.assert_array_equal(delta, ctr)


def test_submit_registered_buffers(cuda):
    """Registered frames, descriptors and results: no staging copies; the
    records land in the caller's registered array."""
    filters, socks = pktgen.world(4)
    n = 4096
    buf0, desc0 = pktgen.generate(4, n, first=31337)
    buf = aligned(buf0.nbytes)
    buf[:] = buf0
    desc = aligned(n, _abi.DESC_DTYPE)
    desc[:] = desc0
    out = aligned(n, _abi.RESULT_DTYPE)
    g = GpuRxStack(device=0, host_stage_bytes=buf.nbytes, host_stage_pkts=n)
    g.load_world(filters, socks)
    o = OracleStack()
    o.load_world(filters, socks)
    for arr in (buf, desc, out):
        assert g.host_register(arr) != 0
    delta = np.zeros(_abi.R_COUNT, dtype=np.uint32)
    assert g.wait(g.submit(buf, desc, out, delta)) == n
    want = o.handle_rx_batch(buf, desc, nthreads=8)
    assert out.tobytes() == want.tobytes(), diff_report(out, want, desc)
    np.testing.assert_array_equal(delta, counters_of(want))
    for arr in (buf, desc, out):
        g.host_unregister(arr)
    with pytest.raises(OSError) as e:
        g.host_unregister(out)
    assert e.value.errno == errno.ENOENT


def test_submit_limits(cuda):
    g = GpuRxStack(device=0, host_stage_bytes=1 << 16, host_stage_pkts=64)
    buf = np.zeros(1 << 17, np.uint8)
    desc = np.zeros(65, _abi.DESC_DTYPE)
    out = np.zeros(65, _abi.RESULT_DTYPE)
    for b, d in ((buf, desc[:8]), (buf[: 1 << 16], desc)):
        with pytest.raises(OSError) as e:
            g.submit(b, d, out)
        assert e.value.errno == errno.EINVAL
    nostage = GpuRxStack(device=0)
    with pytest.raises(OSError) as e:
        nostage.submit(buf[:64], desc[:1], out)
    assert e.value.errno == errno.EINVAL


def test_zero_copy_umem_ring_poll(cuda):
    """UMEM and ring in registered host memory, read by the kernel in place:
    oo_gpu_rx_xdp_poll over them (ring and u32 index wrap) equals the
    oracle's ring batch; consumer published per batch."""
    torch = cuda
    filters, socks = pktgen.world(5)
    g = GpuRxStack(device=0)
    o = OracleStack()
    for st in (g, o):
        st.load_world(filters, socks)
    n = 6000
    buf, desc = pktgen.generate(5, n, first=4040)
    umem0, ents = to_umem(frames_of(buf, desc), seed=5, headroom=(192, 193))
    cons0 = (1 << 32) - 2500
    ring0, mask = ring_of(ents, 13, cons0)
    umem = aligned(umem0.nbytes)
    umem[:] = umem0
    ring = aligned(len(ring0), _abi.XDP_DESC_DTYPE)
    ring[:] = ring0
    d_umem = g.host_register(umem)
    d_ring = g.host_register(ring)
    want = o.handle_xdp_batch(umem, ring, mask, cons0, n, 1)
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(_abi.R_COUNT, dtype=torch.int32, device="cuda")
    consumer = np.array([cons0], dtype=np.uint32)
    producer = np.array([(cons0 + n) & 0xFFFFFFFF], dtype=np.uint32)
    stream = torch.cuda.current_stream().cuda_stream
    done = 0
    while done < n:
        k = g.xdp_poll(d_umem, umem.nbytes, d_ring, mask, consumer, producer, 2048, 1,
                       out.data_ptr() + 32 * done, ctr.data_ptr(), stream)
        assert k == min(2048, n - done)
        done += k
        assert int(consumer[0]) == (cons0 + done) & 0xFFFFFFFF
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
    assert got.tobytes() == want.tobytes(), diff_report(got, want)
    np.testing.assert_array_equal(ctr.cpu().numpy().astype(np.uint32), counters_of(want))
    g.host_unregister(ring)
    g.host_unregister(umem)


@pytest.mark.parametrize("kernel", ["0", "1", "2", "3"])
def test_frames_flush_with_registered_page_ends(cuda, kernel, monkeypatch):
    """Frames read in place from registered host memory, each page holding
    one frame from its first bytes (odd offset) and one ending at its last
    byte -- the pool's last frame ends at the registration's last byte, and
    the page after it is not mapped for the device.  Every kernel reads only
    the lines that hold its frames' bytes, so no access leaves the
    registered pages (one that did would fault the GPU); records equal the
    oracle's."""
    torch = cuda
    monkeypatch.setenv("OO_RX_KERNEL", kernel)
    filters, socks = pktgen.world(2)
    g = GpuRxStack(device=0)
    o = OracleStack()
    for st in (g, o):
        st.load_world(filters, socks)
    buf0, desc0 = pktgen.generate(2, 8, first=4242)
    frames = [bytes(buf0[int(d["frame_off"]):int(d["frame_off"]) + int(d["len"])]) for d in desc0]
    frames[5] = frames[5][:61]  # a short capture among them
    pages = 4
    pool = page_buffer(pages * PAGE)
    desc = np.zeros(2 * pages, _abi.DESC_DTYPE)
    for p in range(pages):
        for k, f in enumerate(frames[2 * p:2 * p + 2]):
            off = p * PAGE + 3 if k == 0 else (p + 1) * PAGE - len(f)
            pool[off:off + len(f)] = np.frombuffer(f, np.uint8)
            desc[2 * p + k] = (off, len(f), 0, 0)
    d_pool = g.host_register(pool)
    de = torch.from_numpy(desc.view(np.uint8)).to("cuda")
    out = torch.full((len(desc) * 32,), 0xAB, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(_abi.R_COUNT, dtype=torch.int32, device="cuda")
    g.handle_rx_batch_dev(d_pool, pool.nbytes, de.data_ptr(), len(desc), out.data_ptr(),
                          ctr.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
    want = o.handle_rx_batch(pool, desc, nthreads=1)
    assert got.tobytes() == want.tobytes(), diff_report(got, want, desc)
    np.testing.assert_array_equal(ctr.cpu().numpy().astype(np.uint32), counters_of(want))
    g.host_unregister(pool)
    g.close()


def test_xdp_frames_and_ring_flush_with_registered_page_ends(cuda):
    """The AF_XDP form of the page-end test: UMEM frames flush with the first
    and last bytes of registered pages, the RX ring exactly one registered
    page (256 entries, the batch wrapping its end), read in place by
    oo_gpu_rx_xdp_poll; records equal the oracle's ring batch."""
    torch = cuda
    filters, socks = pktgen.world(2)
    g = GpuRxStack(device=0)
    o = OracleStack()
    for st in (g, o):
        st.load_world(filters, socks)
    buf0, desc0 = pktgen.generate(2, 8, first=777)
    frames = [bytes(buf0[int(d["frame_off"]):int(d["frame_off"]) + int(d["len"])]) for d in desc0]
    pages = 4
    umem = page_buffer(pages * PAGE)
    ents = np.zeros(2 * pages, _abi.XDP_DESC_DTYPE)
    for p in range(pages):
        for k, f in enumerate(frames[2 * p:2 * p + 2]):
            off = p * PAGE + 1 if k == 0 else (p + 1) * PAGE - len(f)
            umem[off:off + len(f)] = np.frombuffer(f, np.uint8)
            ents[2 * p + k] = (off, len(f), 0)
    ring = page_buffer(PAGE // 16, _abi.XDP_DESC_DTYPE)
    cons0 = 256 - 3
    ring0, mask = ring_of(ents, 8, cons0)
    ring[:] = ring0
    n = len(ents)
    d_umem = g.host_register(umem)
    d_ring = g.host_register(ring)
    want = o.handle_xdp_batch(umem, ring, mask, cons0, n, 1)
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(_abi.R_COUNT, dtype=torch.int32, device="cuda")
    consumer = np.array([cons0], dtype=np.uint32)
    producer = np.array([cons0 + n], dtype=np.uint32)
    k = g.xdp_poll(d_umem, umem.nbytes, d_ring, mask, consumer, producer, 64, 1,
                   out.data_ptr(), ctr.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert k == n and int(consumer[0]) == cons0 + n
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
    assert got.tobytes() == want.tobytes(), diff_report(got, want)
    np.testing.assert_array_equal(ctr.cpu().numpy().astype(np.uint32), counters_of(want))
    g.host_unregister(ring)
    g.host_unregister(umem)
    g.close()


def _libc():
    import ctypes
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return libc


def test_register_unregister_unmap_then_pageable_copies_at_the_same_address(cuda):
    """The round-5 faults' lifetime, the legal way round (DESIGN.md §5 round
    6): pages registered with a context and read in place by a batch, then
    unregistered, unmapped, and mapped again at the same address as ordinary
    pageable memory; torch's pageable copies to and from that address (the
    copies the faults were reported at) move the new bytes, both a copy
    large enough for the runtime to pin it in place and a small one.  The
    context closes only once nothing is registered."""
    import ctypes
    torch = cuda
    libc = _libc()
    PROT_RW, MAP_PRIV_ANON, MAP_FIXED_NOREPLACE = 0x3, 0x22, 0x100000
    filters, socks = pktgen.world(2)
    n = 4096
    buf0, desc = pktgen.generate(2, n, first=777)
    size = -(-buf0.nbytes // PAGE) * PAGE + (64 << 20)  # the batch's frames, then 64 MiB more
    addr = libc.mmap(None, size, PROT_RW, MAP_PRIV_ANON, -1, 0)
    assert addr not in (None, ctypes.c_void_p(-1).value)
    host = np.frombuffer((ctypes.c_uint8 * size).from_address(addr), np.uint8)
    host[:buf0.nbytes] = buf0
    g = GpuRxStack(device=0, host_stage_bytes=1 << 20, host_stage_pkts=n)
    g.load_world(filters, socks)
    o = OracleStack()
    o.load_world(filters, socks)
    d = g.host_register(host, nbytes=size)
    assert d != 0 and g.host_registered() == 1
    # the frames read in place by the kernel: the mapping is used
    dd = torch.from_numpy(desc.view(np.uint8).copy()).to("cuda")
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    g.handle_rx_batch_dev(d, buf0.nbytes, dd.data_ptr(), n, out.data_ptr(), 0, s.cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(_abi.RESULT_DTYPE)
    want = o.handle_rx_batch(buf0, desc, nthreads=8)
    assert got.tobytes() == want.tobytes(), diff_report(got, want, desc)
    with pytest.raises(OSError) as e:  # still registered: the context stays open
        g.close()
    assert e.value.errno == errno.EBUSY
    g.host_unregister(host)
    del host
    assert libc.munmap(ctypes.c_void_p(addr), size) == 0
    again = libc.mmap(ctypes.c_void_p(addr), size, PROT_RW, MAP_PRIV_ANON | MAP_FIXED_NOREPLACE,
                      -1, 0)
    assert again == addr, "the kernel did not give the same address back"
    fresh = np.frombuffer((ctypes.c_uint8 * size).from_address(addr), np.uint8)
    rng = np.random.default_rng(3)
    for nbytes in (size, 4096 * 3 + 100):
        src = rng.integers(0, 256, nbytes, dtype=np.uint8)
        fresh[:nbytes] = src
        dev = torch.from_numpy(fresh[:nbytes]).to("cuda")  # pageable H2D from those pages
        torch.cuda.synchronize()
        assert torch.equal(dev.cpu(), torch.from_numpy(src))
        dev.add_(1)
        torch.from_numpy(fresh[:nbytes]).copy_(dev)  # pageable D2H into those pages
        torch.cuda.synchronize()
        assert (fresh[:nbytes] == (src + 1).astype(np.uint8)).all()
    del fresh
    assert libc.munmap(ctypes.c_void_p(addr), size) == 0
    g.close()
