# SPDX-License-Identifier: BSD-2-Clause
"""Parity of the gfx950 kernels (through the C ABI) with the oracle:
bit-exact 32-byte records on identical frame buffers, plus counters."""
import os

import numpy as np
import pytest

import cases
from frames import edge_frames, edge_world, install, pack
from gpu_util import diff_report, run_dev
from onload_amd import _abi, pktgen
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack, counters_of

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)
HWPORTS = (0, 1, 3, 2, 5)  # intf 2 -> hwport 3 (edge world's bind2dev socket)


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _pair(world_installer, **kw):
    g = GpuRxStack(device=0, **kw)
    o = OracleStack(**kw)
    world_installer(g)
    world_installer(o)
    return g, o


def _check(g, o, buf, desc, frames_bytes=None):
    got, ctr = run_dev(g, buf, desc, frames_bytes)
    want = o.handle_rx_batch(buf, desc, nthreads=NTHREADS)
    assert got.tobytes() == want.tobytes(), diff_report(got, want, desc)
    np.testing.assert_array_equal(ctr, counters_of(want))
    return got


def test_survey_cases_on_gpu(cuda):
    g, o = _pair(lambda s: install(s, cases.survey_world()))
    frames = [(f, intf) for (_, f, intf, _) in cases.survey_cases()]
    buf, desc = pack(frames)
    got = _check(g, o, buf, desc)
    for r, (name, _, _, want) in zip(got, cases.survey_cases()):
        for k, v in want.items():
            assert r[k] == v, (name, k)


def test_lookup_order_on_gpu(cuda):
    socks, filters = cases.order_world()
    g, o = _pair(lambda s: install(s, (socks, filters)))
    buf, desc = pack([(cases.order_frame(), 0)])
    for stage in (1, 2, 3):
        r = _check(g, o, buf, desc)[0]
        assert r["stage"] == stage
        g.filter_remove(*filters[stage - 1])
        o.filter_remove(*filters[stage - 1])
    assert _check(g, o, buf, desc)[0]["reason"] == _abi.R_NO_MATCH


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 6, 8, 15])
def test_edge_corpus(cuda, shift):
    """Every gate of SURVEY §8(a) on both sides, at every frame alignment
    (odd offsets exercise the RFC 1071 byte-swap path)."""
    g, o = _pair(lambda s: install(s, edge_world()), intf_hwport=HWPORTS)
    buf, desc = pack(edge_frames(), align=64 if shift % 2 == 0 else 16, shift=shift)
    got = _check(g, o, buf, desc)
    assert len(set(got["reason"].tolist())) >= 15


def test_edge_corpus_shuffled_and_unaligned_tail(cuda):
    """Random order, random 1-byte offsets, frames abutting the buffer end."""
    g, o = _pair(lambda s: install(s, edge_world()), intf_hwport=HWPORTS)
    fr = edge_frames(seed=99)
    rng = np.random.default_rng(3)
    chunks, desc, off = [], np.zeros(len(fr), dtype=_abi.DESC_DTYPE), 0
    for i in rng.permutation(len(fr)):
        f, intf = fr[i]
        pad = int(rng.integers(0, 5))
        chunks.append(bytes(pad) + f)
        desc[len(chunks) - 1] = (off + pad, len(f), intf, 0)
        off += pad + len(f)
    buf = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy()
    _check(g, o, buf, desc, frames_bytes=len(buf))


def test_descriptor_outside_buffer_is_empty_frame(cuda):
    """Out-of-buffer descriptors are empty frames, including offsets near
    2^64 whose offset + length wraps (the bounds test must not
    wrap)."""
    g, o = _pair(lambda s: install(s, edge_world()))
    buf, desc = pack(edge_frames()[:40])
    n = len(buf)
    desc[3]["frame_off"] = n + 100
    desc[5]["frame_off"] = (1 << 64) - 16
    desc[6]["frame_off"] = (1 << 64) - 64
    desc[6]["len"] = 64
    desc[7]["frame_off"] = n - 10  # runs 10 bytes past the end
    desc[8]["frame_off"] = n - int(desc[8]["len"])  # abuts the end exactly
    got = _check(g, o, buf, desc)
    for i in (3, 5, 6, 7):
        assert got[i]["reason"] == _abi.R_SHORT_L2, i


@pytest.mark.parametrize("config,n", [(2, 1 << 16), (3, 1 << 18), (4, 1 << 14), (5, 1 << 17)])
def test_config_samples(cuda, config, n):
    filters, socks = pktgen.world(config)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    first = 12345 * config  # an arbitrary shard
    buf, desc = pktgen.generate(config, n, first=first)
    got = _check(g, o, buf, desc)
    r = got["reason"]
    assert (r == _abi.R_DELIVER).mean() > 0.8
    if config in (4, 5):
        assert set(np.unique(got["stage"][r == 0]).tolist()) == {1, 2, 3}


@pytest.mark.parametrize("n", [1, 7, 9, 63, 65, 1000, 20001])
def test_ragged_batch_sizes(cuda, n):
    """Tile partition edges: batches far below one tile per wave, sizes that
    are not multiples of 8 (the last tile takes the rest)."""
    filters, socks = pktgen.world(4)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    buf, desc = pktgen.generate(4, n, first=777)
    _check(g, o, buf, desc)


def test_host_path_matches_device_path(cuda):
    filters, socks = pktgen.world(5)
    buf, desc = pktgen.generate(5, 4096)
    g = GpuRxStack(device=0, host_stage_bytes=len(buf), host_stage_pkts=len(desc))
    g.load_world(filters, socks)
    a, ca = g.handle_rx_batch(buf, desc)
    b, cb = run_dev(g, buf, desc)
    assert a.tobytes() == b.tobytes()
    np.testing.assert_array_equal(ca, cb)


def test_table_updates_reach_device_between_batches(cuda):
    g, o = _pair(lambda s: install(s, cases.survey_world()))
    frames = [(f, i) for (_, f, i, _) in cases.survey_cases()]
    buf, desc = pack(frames)
    _check(g, o, buf, desc)
    for s in (g, o):  # connect a UDP socket to the peer: stage 1 now wins
        s.sock_set(40, cases._sock(17, 6003, cases.PEER, 33000, flags=_abi.SOCK_CONNECTED))
        assert s.filter_insert(40, 4, cases.LA, 6003, cases.PEER, 33000, 17) == 0
    got = _check(g, o, buf, desc)
    assert got[0]["stage"] == 1 and got[0]["sock"] == 40
    for s in (g, o):
        s.filter_remove(3, 4, cases.LA, 6003, None, 0, 17)
    _check(g, o, buf, desc)


def test_full_size_config2_bit_exact(cuda):
    """BASELINE config 2 at full size: 2^20 x 1514 B, every record."""
    filters, socks = pktgen.world(2)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    buf, desc = pktgen.generate(2, 1 << 20)
    got = _check(g, o, buf, desc)
    assert g.last_path() == 1  # long frames: rx_kernel, 4-slot ring
    frac = np.bincount(got["reason"], minlength=32) / len(got)
    assert abs(frac[_abi.R_UDP_CSUM] - 0.01) < 0.002
    assert abs(frac[_abi.R_NO_MATCH] - 0.005) < 0.002
    assert frac[_abi.R_DELIVER] > 0.98


def test_full_size_config3_bit_exact(cuda):
    """BASELINE config 3 at full size: 2^24 x 64 B, every record."""
    filters, socks = pktgen.world(3)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    buf, desc = pktgen.generate(3, 1 << 24, nthreads=NTHREADS)
    got = _check(g, o, buf, desc)
    assert g.last_path() == 4  # window-sized frames, 2^20+: the split transform
    # (short-frame class: the per-group-sequence body engine)
    assert (got["stage"][got["reason"] == 0] == 2).all()


def test_full_size_config4_bit_exact(cuda):
    """BASELINE config 4 at the bench's full single-GPU size: 2^22 mixed
    IPv4/TCP frames of 64-9014 B with IP and TCP options, every record."""
    filters, socks = pktgen.world(4)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    buf, desc = pktgen.generate(4, 1 << 22, nthreads=NTHREADS)
    got = _check(g, o, buf, desc)
    assert set(np.unique(got["stage"][got["reason"] == 0]).tolist()) == {1, 2, 3}


def test_full_size_config5_last_shard_bit_exact(cuda):
    """BASELINE config 5 at full per-GPU size: the 8th of the eight
    byte-balanced shards of 2^27 IMIX TCP/UDP IPv4/IPv6 frames (what rank 7
    processes in `bench.py --gpus 8`), every record."""
    from onload_amd import shards
    filters, socks = pktgen.world(5)
    g, o = _pair(lambda s: s.load_world(filters, socks))
    seed = pktgen.default_seed(5)
    first, n = shards.shard_for(5, seed, 8 << 24, 7, 8)
    buf, desc = pktgen.generate(5, n, seed=seed, first=first, nthreads=NTHREADS)
    got = _check(g, o, buf, desc)
    assert (got["reason"] == _abi.R_DELIVER).mean() > 0.9


@pytest.mark.parametrize("env", [{"OO_RX_STATIC": "1"}, {"OO_RX_TAIL_TILE": "8", "OO_RX_TAIL_PER_WAVE": "3"},
                                 {"OO_RX_TAIL_TILE": "64"}, {"OO_RX_GRID_PCT": "37"},
                                 {"OO_RX_GSHIFT": "4", "OO_RX_GROUPS": "8"}, {"OO_RX_GSHIFT": "4"},
                                 {"OO_RX_GSHIFT": "5", "OO_RX_GROUPS": "16", "OO_RX_GRID_PCT": "37"},
                                 {"OO_RX_GSHIFT": "0", "OO_RX_GROUPS": "64"}, {"OO_RX_KERNEL": "1"},
                                 {"OO_RX_KERNEL": "2", "OO_RX_GRID_PCT": "37"},
                                 {"OO_RX_KERNEL": "3"}, {"OO_RX_KERNEL": "3", "OO_RX_BODY_TAIL": "64"},
                                 {"OO_RX_KERNEL": "3", "OO_RX_GRID_PCT": "37", "OO_RX_BODY_BPC": "2"},
                                 {"OO_RX_KERNEL": "4"}, {"OO_RX_KERNEL": "4", "OO_RX_GRID_PCT": "37"}])
def test_tile_partitions_and_claim_reuse(cuda, env, monkeypatch):
    """Static and dynamic (claimed) tile schedules with several tail shapes
    give the same records; 40 launches in a row reuse every claim-counter
    set (16 per context) and must each see them reset (oo_rx_kernel.hip
    tile_loop, oo_gpu_rx.cpp launch())."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    filters, socks = pktgen.world(5)
    g = GpuRxStack(device=0)
    o = OracleStack()
    g.load_world(filters, socks)
    o.load_world(filters, socks)
    for n in (200003, 4099, 64, 1):
        buf, desc = pktgen.generate(5, n, nthreads=NTHREADS)
        want = o.handle_rx_batch(buf, desc, nthreads=NTHREADS)
        for rep in range(10 if n > 1000 else 5):
            got, ctr = run_dev(g, buf, desc)
            assert got.tobytes() == want.tobytes(), (n, rep, diff_report(got, want, desc))
            np.testing.assert_array_equal(ctr, counters_of(want))
    g.close()


@pytest.mark.parametrize("kernel", ["1", "2", "3", "3:1", "3:2"])
def test_both_rx_kernels_on_every_corpus(cuda, kernel, monkeypatch):
    """The 4-slot-ring rx_kernel (long frames) and the 2-slot one (short
    frames, 12 waves per CU) are chosen per launch by buffer bytes per packet
    (oo_gpu_rx.cpp launch()); forced here (OO_RX_KERNEL 1 / 2, and 3: the
    split transform, win_kernel + body_kernel; 3:1 / 3:2 with its lockstep
    or per-group-sequence body engine forced), each must be
    bit-exact on the edge corpus at odd and even alignments and on samples of
    every configuration, with several launches per context."""
    kernel, _, engine = kernel.partition(":")  # 3:E -- the split with body engine E
    monkeypatch.setenv("OO_RX_KERNEL", kernel)
    if engine:
        monkeypatch.setenv("OO_RX_BODY_ENGINE", engine)
    g, o = _pair(lambda s: install(s, edge_world()), intf_hwport=HWPORTS)
    for shift in (0, 3):
        buf, desc = pack(edge_frames(), align=64 if shift % 2 == 0 else 16, shift=shift)
        _check(g, o, buf, desc)
    g.close()
    for config, n in ((2, 1 << 15), (3, 1 << 17), (4, 1 << 14), (5, 1 << 17)):
        filters, socks = pktgen.world(config)
        g, o = _pair(lambda s: s.load_world(filters, socks))
        buf, desc = pktgen.generate(config, n, first=999 * config, nthreads=NTHREADS)
        for _ in range(3):
            _check(g, o, buf, desc)
        g.close()
