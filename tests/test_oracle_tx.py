# SPDX-License-Identifier: BSD-2-Clause
"""The oracle's TX checksum fill (oo_pkt_calc_checksums restated) against the
reference's own checksum.c: the committed golden frames
(tests/golden/make_tx_golden.py) and, where the compiled reference is
present, fresh random frames."""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle_lib import oracle_tx_fill, REF_PATH, ref_lib, tx_golden  # noqa: E402


def test_tx_fill_golden():
    fin, fout, desc = tx_golden()
    got = oracle_tx_fill(fin, desc)
    bad = np.nonzero(got != fout)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:5]}"
    assert (fin != fout).any()  # the fill changed something


def test_tx_fill_untouched_cases():
    """Frames the fill must not change: non-IP, other protocols, IHL < 5,
    TCP doff < 5, truncated headers."""
    from onload_amd import _abi
    frames = []
    eth4, eth6 = bytes(12) + b"\x08\x00", bytes(12) + b"\x86\xdd"
    ip = bytearray(20)
    ip[0], ip[9] = 0x45, 1  # ICMP
    frames.append(eth4 + bytes(ip) + bytes(30))
    ip[0], ip[9] = 0x44, 17  # IHL 4
    frames.append(eth4 + bytes(ip) + bytes(30))
    frames.append(bytes(12) + b"\x08\x06" + bytes(40))  # ARP
    frames.append(eth6 + bytes(20))  # IPv6 header cut short
    frames.append(bytes(10))
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    desc = np.zeros(len(frames), dtype=_abi.DESC_DTYPE)
    desc["frame_off"] = np.concatenate([[0], np.cumsum([len(f) for f in frames])[:-1]])
    desc["len"] = [len(f) for f in frames]
    assert np.array_equal(oracle_tx_fill(buf, desc), buf)

    # TCP doff < 5 or a TCP header cut short: the IPv4 header checksum is
    # still filled (the reference fills it before looking at L4), L4 is not.
    ip[0], ip[9] = 0x45, 6
    tcp = bytearray(20)
    tcp[12] = 0x40  # doff 4
    for f in (eth4 + bytes(ip) + bytes(tcp) + bytes(10), eth4 + bytes(ip) + bytes(10)):
        b = np.frombuffer(f, np.uint8).copy()
        d = np.zeros(1, dtype=_abi.DESC_DTYPE)
        d["len"] = len(f)
        got = oracle_tx_fill(b, d)
        assert set(np.nonzero(got != b)[0].tolist()) <= {24, 25}
        assert got[24:26].tobytes() != b"\0\0"


@pytest.mark.skipif(not os.path.exists(REF_PATH), reason="compiled reference absent (oracle/_ref)")
def test_tx_fill_live_against_reference():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_tx_golden as g
    ref = ref_lib()
    ref.ef_ip_checksum.argtypes = [ctypes.c_void_p]
    ref.ef_ip_checksum.restype = ctypes.c_uint32
    for name in ("ef_udp_checksum", "ef_udp_checksum_ip6", "ef_tcp_checksum",
                 "ef_tcp_checksum_ip6"):
        getattr(ref, name).argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
        getattr(ref, name).restype = ctypes.c_uint32
    from onload_amd import _abi
    rng = np.random.default_rng(99)
    frames = [g.frame(rng, k) for k in range(300)]
    want = b"".join(g.fill(ref, f) for f in frames)
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    desc = np.zeros(len(frames), dtype=_abi.DESC_DTYPE)
    desc["frame_off"] = np.concatenate([[0], np.cumsum([len(f) for f in frames])[:-1]])
    desc["len"] = [len(f) for f in frames]
    assert oracle_tx_fill(buf, desc).tobytes() == want
