# SPDX-License-Identifier: BSD-2-Clause
"""Generate tests/golden/ref_tx_fill.npz from the REFERENCE's own code.

Run in the build container (where /root/reference exists) after `make`:

    python tests/golden/make_tx_golden.py

Inputs are seeded random frames (untagged / VLAN, IPv4 with and without
options / IPv6, TCP with options / UDP / other protocols, fragments, odd
lengths, random initial check fields).  The expected frames come from the
reference's checksum.c (ef_ip_checksum, ef_udp_checksum{,_ip6},
ef_tcp_checksum{,_ip6}) compiled unmodified into oracle/_ref/libref_rx.so,
driven by the control flow of oo_pkt_calc_checksums
(src/lib/transport/ip/pkt_checksum.c:20-102) as calc_csum_if_needed
(netif_tx.c:24-40) calls it.  The oracle is NOT used here.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle_lib import ref_lib  # noqa: E402

N = 800
_P = ctypes.c_void_p


def frame(rng: np.random.Generator, k: int) -> bytes:
    vlan = k % 5 == 0
    af6 = k % 4 == 3
    proto = [6, 17, 17, 6, 1][k % 5] if k % 23 else 58
    pay = int(rng.integers(0, 1200)) if k % 3 else int(rng.integers(0, 40))
    eth = bytearray(rng.integers(0, 256, 12, dtype=np.uint8).tobytes())
    if vlan:
        eth += b"\x81\x00" + int(rng.integers(0, 65536)).to_bytes(2, "big")
    eth += b"\x86\xdd" if af6 else b"\x08\x00"
    if af6:
        l3 = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
        l3[0] = 0x60 | (l3[0] & 0xF)
        l3[6] = proto
    else:
        ihl = 5 if k % 7 else int(rng.integers(5, 16))
        l3 = bytearray(rng.integers(0, 256, 4 * ihl, dtype=np.uint8).tobytes())
        l3[0] = 0x40 | ihl
        l3[9] = proto
        fr = k % 11
        l3[6:8] = (0x4000 if fr < 6 else 0 if fr < 9 else
                   int(rng.integers(0, 65536))).to_bytes(2, "big")
    if proto == 6:
        doff = 5 if k % 3 else int(rng.integers(5, 16))
        l4 = bytearray(rng.integers(0, 256, 4 * doff, dtype=np.uint8).tobytes())
        l4[12] = (doff << 4) | (l4[12] & 0xF)
    elif proto == 17:
        l4 = bytearray(rng.integers(0, 256, 8, dtype=np.uint8).tobytes())
        l4[4:6] = (8 + pay).to_bytes(2, "big")
    else:
        l4 = bytearray(rng.integers(0, 256, 8, dtype=np.uint8).tobytes())
    if af6:
        l3[4:6] = (len(l4) + pay).to_bytes(2, "big")
    else:
        tl = len(l3) + len(l4) + pay
        if k % 13 == 0:
            tl = int(rng.integers(0, 65536))  # tot_len inconsistent with the frame
        l3[2:4] = tl.to_bytes(2, "big")
    return bytes(eth + l3 + l4) + rng.integers(0, 256, pay, dtype=np.uint8).tobytes()


def fill(ref, fr: bytes) -> bytes:
    """oo_pkt_calc_checksums on one frame, arithmetic by the reference."""
    b = bytearray(fr)
    l3 = 18 if b[12:14] == b"\x81\x00" else 14
    et = b[l3 - 2:l3]
    af6 = et == b"\x86\xdd"
    if not af6 and et != b"\x08\x00":
        return bytes(b)
    buf = ctypes.create_string_buffer(bytes(b), len(b))
    base = ctypes.addressof(buf)
    if af6:
        proto, l4 = b[l3 + 6], l3 + 40
    else:
        proto, l4 = b[l3 + 9], l3 + (b[l3] & 0xF) * 4
    if proto not in (6, 17):
        return bytes(b)
    if not af6:
        v = ref.ef_ip_checksum(base + l3)
        ctypes.memmove(base + l3 + 10, v.to_bytes(4, "little")[:2], 2)
    if proto == 17:
        if not af6 and (int.from_bytes(b[l3 + 6:l3 + 8], "big") & ~0x4000):
            return buf.raw
        iov = (_P * 2)(base + l4 + 8, len(b) - l4 - 8)
        f = ref.ef_udp_checksum_ip6 if af6 else ref.ef_udp_checksum
        v = f(base + l3, base + l4, iov, 1)
        ctypes.memmove(base + l4 + 6, v.to_bytes(4, "little")[:2], 2)
    else:
        hl = (b[l4 + 12] >> 4) * 4
        iov = (_P * 2)(base + l4 + hl, len(b) - l4 - hl)
        f = ref.ef_tcp_checksum_ip6 if af6 else ref.ef_tcp_checksum
        v = f(base + l3, base + l4, iov, 1)
        ctypes.memmove(base + l4 + 16, v.to_bytes(4, "little")[:2], 2)
    return buf.raw


def main():
    ref = ref_lib()
    if ref is None:
        sys.exit("oracle/_ref/libref_rx.so missing: run `make` where /root/reference exists")
    ref.ef_ip_checksum.argtypes = [_P]
    ref.ef_ip_checksum.restype = ctypes.c_uint32
    for name in ("ef_udp_checksum", "ef_udp_checksum_ip6", "ef_tcp_checksum",
                 "ef_tcp_checksum_ip6"):
        getattr(ref, name).argtypes = [_P, _P, _P, ctypes.c_int]
        getattr(ref, name).restype = ctypes.c_uint32
    rng = np.random.default_rng(0x7C5F)
    frames = [frame(rng, k) for k in range(N)]
    out = [fill(ref, f) for f in frames]
    lens = np.array([len(f) for f in frames], np.uint32)
    np.savez_compressed(os.path.join(HERE, "ref_tx_fill.npz"),
                        frames_in=np.frombuffer(b"".join(frames), np.uint8),
                        frames_out=np.frombuffer(b"".join(out), np.uint8), lens=lens)
    changed = sum(a != b for a, b in zip(frames, out))
    print(f"{N} frames, {changed} changed by the fill")


if __name__ == "__main__":
    main()
