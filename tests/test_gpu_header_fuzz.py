# SPDX-License-Identifier: BSD-2-Clause
"""Seeded random headers through every kernel path, against the oracle:
the general header walk's inputs -- VLAN tags, IHL 0..15 with random option
bytes (NOP runs, EOL, the four accepted kinds with any length byte, other
kinds), IPv6, TCP data offsets with options, wrong total lengths, fragments,
truncated frames -- at odd and even alignments.  win_kernel (OO_RX_KERNEL 3)
takes its fields from word runs and walks the options between non-NOP bytes
(oo_rx_kernel.hip parse_general_runs); rx_kernel (1, 2) walks them byte by
byte; both must give the oracle's records (netif_event.c:135-185, 1024-1127)."""
import os
import random

import pytest

from frames import L4A, L6A, PEER4, PEER6, edge_world, eth, install, ipv4, ipv6, pack, tcp, udp
from gpu_util import diff_report, run_dev
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack, counters_of

import numpy as np

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)
HWPORTS = (0, 1, 3, 2, 5)


@pytest.fixture(scope="module")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _options(rnd: random.Random, n: int) -> bytes:
    out = bytearray()
    while len(out) < n:
        r = rnd.random()
        if r < 0.35:
            out += b"\x01" * rnd.randrange(1, 9)
        elif r < 0.45:
            out += b"\x00" + bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 4)))
        elif r < 0.85:
            ln = rnd.choice([0, 1, 2, 3, 4, 4, 5, 8, 8, 11, 12, rnd.randrange(46), 0x80, 0xFF])
            out += bytes([rnd.choice([7, 68, 130, 136]), ln])
            out += bytes(rnd.randrange(256) for _ in range(max(0, min(ln, 44) - 2)))
        else:
            out += bytes([rnd.choice([2, 3, 9, 131, 137, 148, 0x99, rnd.randrange(256)])])
    return bytes(out[:n])


def fuzz_frames(seed: int, n: int) -> list[tuple[bytes, int]]:
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        six = rnd.random() < 0.15
        vlan = rnd.randrange(4096) if rnd.random() < 0.25 else None
        proto = rnd.choice([6, 6, 17, 17, 17, 1])
        pay = bytes(rnd.randrange(256) for _ in range(rnd.choice([0, 1, 7, 8, 22, 31, 64, 101, 300])))
        dport = rnd.choice([5001, 80, 8080, 9999, rnd.randrange(65536)])
        sport = rnd.choice([1, 40000, 5, rnd.randrange(65536)])
        src, dst = (PEER6, L6A) if six else (PEER4, L4A)
        af = 6 if six else 4
        csum = rnd.choice(["ok"] * 8 + ["bad"])
        if proto == 17:
            l4 = udp(af, src, dst, sport, dport, pay, csum=rnd.choice(["ok"] * 6 + ["bad", "zero"]))
        elif proto == 6:
            doff = rnd.choice([5, 5, 5, 6, 8, 8, 10, 15, rnd.randrange(16)])
            l4 = tcp(af, src, dst, sport, dport, pay, doff=doff,
                     options=bytes(rnd.randrange(256) for _ in range(max(0, doff - 5) * 4)),
                     csum=csum)
        else:
            l4 = pay
        if six:
            f = eth(ipv6(src, dst, proto, l4, plen=rnd.choice([None] * 9 + [rnd.randrange(600)])),
                    0x86DD, vlan=vlan)
        else:
            ihl = rnd.choice([5] * 6 + list(range(16)))
            f = eth(ipv4(src, dst, proto, l4, ihl=ihl, options=_options(rnd, max(0, ihl - 5) * 4),
                         tot_len=rnd.choice([None] * 9 + [rnd.randrange(16, 1600)]),
                         frag=rnd.choice([0x4000] * 8 + [0, 0x2000, 0x0001]), csum=csum),
                    0x0800, vlan=vlan)
        if rnd.random() < 0.1:
            f = f[: rnd.randrange(1, len(f) + 1)]
        out.append((f, rnd.randrange(len(HWPORTS))))
    return out


@pytest.mark.parametrize("kernel", ["3", "2", "1"])
def test_random_headers_every_path(cuda, kernel, monkeypatch):
    monkeypatch.setenv("OO_RX_KERNEL", kernel)
    g = GpuRxStack(device=0, intf_hwport=HWPORTS)
    o = OracleStack(intf_hwport=HWPORTS)
    install(g, edge_world())
    install(o, edge_world())
    frames = fuzz_frames(77 + int(kernel), 6000)
    for shift in (0, 5, 11):
        buf, desc = pack(frames, align=16, shift=shift)
        got, ctr = run_dev(g, buf, desc)
        want = o.handle_rx_batch(buf, desc, nthreads=NTHREADS)
        assert got.tobytes() == want.tobytes(), (shift, diff_report(got, want, desc))
        np.testing.assert_array_equal(ctr, counters_of(want))
    # the corpus reaches the walk's outcomes
    reasons = set(want["reason"].tolist())
    assert len(reasons) >= 10, reasons
    g.close()
