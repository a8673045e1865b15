# SPDX-License-Identifier: BSD-2-Clause
"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Run in the build container (where /root/reference exists) after `make`:

    python tests/golden/make_golden.py

Inputs are seeded random headers/payloads; expected outputs come from the
reference's checksum.c / ip_csum_partial.c / hash.h compiled unmodified into
oracle/_ref/libref_rx.so (oracle/Makefile).  The oracle is NOT used here.

Writes:
  ref_csum_vectors.npz   L3/L4 checksum verdicts + ef_*_checksum fill values
  ref_hash_vectors.npz   __onload_hash1/2/3 and onload_addr_xor values
  ref_unit_checksum.json the known answers of src/tests/unit/lib/ciul/checksum.c:13-62
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle_lib import ref_lib  # noqa: E402

N_CSUM = 3000
N_HASH = 2000
MAXPAY = 400


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), max(len(b), 1))


def csum_vectors(ref, rng: np.random.Generator):
    """Random (af, proto) headers + payloads; ~half made valid by the
    reference's own fill function, then some corrupted."""
    recs = []
    for k in range(N_CSUM):
        af = 4 if (k // 8) % 3 else 6
        proto = 17 if k % 2 else 6
        paylen = int(rng.integers(0, MAXPAY)) if k % 5 else int(rng.integers(0, 9))
        pay = rng.integers(0, 256, paylen, dtype=np.uint8).tobytes()
        if af == 4:
            l3 = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
            l3[0] = 0x45
            l3[9] = proto
        else:
            l3 = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
            l3[0] = 0x60
            l3[6] = proto
        if proto == 17:
            l4 = bytearray(rng.integers(0, 256, 8, dtype=np.uint8).tobytes())
            ul = 8 + paylen
            l4[4:6] = ul.to_bytes(2, "big")
            if af == 4:
                l3[2:4] = (20 + ul).to_bytes(2, "big")
            else:
                l3[4:6] = ul.to_bytes(2, "big")
        else:
            doff = int(rng.integers(5, 16))
            l4 = bytearray(rng.integers(0, 256, doff * 4, dtype=np.uint8).tobytes())
            l4[12] = (doff << 4) | (l4[12] & 0xF)
            if af == 4:
                l3[2:4] = (20 + doff * 4 + paylen).to_bytes(2, "big")
            else:
                l3[4:6] = (doff * 4 + paylen).to_bytes(2, "big")
        mode = (k // 2) % 4  # 0: random check, 1: valid, 2: valid then flip, 3: valid & 0/ffff swap
        fill = 0
        if mode and af == 4:
            b3, b4, bp = _buf(l3), _buf(l4), _buf(pay)
            iov = (ctypes.c_void_p * 2)(ctypes.cast(bp, ctypes.c_void_p), paylen)
            if proto == 17:
                fill = ref.ef_udp_checksum(b3, b4, iov, 1)
                l4[6:8] = fill.to_bytes(2, "little")  # ef_udp_checksum returns a network-order value in a host u16
            else:
                fill = ref.ef_tcp_checksum(b3, b4, iov, 1)
                l4[16:18] = fill.to_bytes(2, "little")
        elif mode:
            # IPv6: build the check value here (input construction only); the
            # recorded verdict below is still the reference verifier's.
            off = 6 if proto == 17 else 16
            l4[off:off + 2] = b"\0\0"
            data = bytes(l3[8:40]) + bytes(l4) + pay
            if len(data) & 1:
                data += b"\0"
            s = sum(int.from_bytes(data[i:i + 2], "big") for i in range(0, len(data), 2))
            s += proto + len(l4) + paylen
            while s >> 16:
                s = (s & 0xFFFF) + (s >> 16)
            fill = (~s) & 0xFFFF
            l4[off:off + 2] = fill.to_bytes(2, "big")
        if mode == 2:
            j = int(rng.integers(0, len(l4) + paylen))
            if j < len(l4):
                l4[j] ^= 0x40
            else:
                pay = bytearray(pay)
                pay[j - len(l4)] ^= 0x40
                pay = bytes(pay)
        if mode == 3 and proto == 6:
            off = 16
            c = int.from_bytes(l4[off:off + 2], "big")
            if c in (0, 0xFFFF):
                l4[off:off + 2] = (0xFFFF - c).to_bytes(2, "big")
        ok = (ref.ref_udp_ok if proto == 17 else ref.ref_tcp_ok)(
            af, _buf(l3), _buf(l4), _buf(pay), paylen)
        recs.append((af, proto, bytes(l3), bytes(l4), bytes(pay), int(ok != 0), fill))
    return recs


def main():
    ref = ref_lib()
    if ref is None:
        sys.exit("oracle/_ref/libref_rx.so missing: run `make` where /root/reference exists")
    rng = np.random.default_rng(0x0E1D)
    recs = csum_vectors(ref, rng)
    blob = b"".join(r[2] + r[3] + r[4] for r in recs)
    meta = np.array([(r[0], r[1], len(r[2]), len(r[3]), len(r[4]), r[5], r[6]) for r in recs],
                    dtype=[("af", "u1"), ("proto", "u1"), ("l3len", "<u2"), ("l4len", "<u2"),
                           ("paylen", "<u2"), ("ok", "u1"), ("fill", "<u4")])
    # IPv4 header verdicts (ci_ip_csum_partial + ci_ip_hdr_csum_finish).
    hdrs, hok, hmax = [], [], []
    for k in range(1000):
        ihl = int(rng.integers(0, 16))
        h = bytearray(rng.integers(0, 256, 60, dtype=np.uint8).tobytes())
        h[0] = (4 << 4) | ihl
        h[2:4] = int(rng.integers(0, 200)).to_bytes(2, "big")
        if k % 2 and ihl >= 5:
            h[10:12] = b"\0\0"
            s = sum(int.from_bytes(h[i:i + 2], "big") for i in range(0, ihl * 4, 2))
            while s >> 16:
                s = (s & 0xFFFF) + (s >> 16)
            h[10:12] = ((~s) & 0xFFFF).to_bytes(2, "big")
        mx = int(rng.integers(0, 200))
        hdrs.append(bytes(h))
        hmax.append(mx)
        hok.append(ref.ref_ip_hdr_csum_ok(_buf(h), mx))
    np.savez_compressed(os.path.join(HERE, "ref_csum_vectors.npz"),
                        meta=meta, blob=np.frombuffer(blob, dtype=np.uint8),
                        ip_hdr=np.frombuffer(b"".join(hdrs), dtype=np.uint8).reshape(-1, 60),
                        ip_max=np.array(hmax, dtype=np.int32),
                        ip_ok=np.array(hok, dtype=np.uint8))

    # Hashes.
    t = rng.integers(0, 2**32, size=(N_HASH, 5), dtype=np.uint64)
    t[:, 1] &= 0xFFFF
    t[:, 3] &= 0xFFFF
    t[:, 4] = np.where(t[:, 4] % 2 == 0, 6, 17)
    t[: N_HASH // 4, 2] = 0
    t[: N_HASH // 4, 3] = 0
    masks = np.array([(1 << int(rng.integers(1, 25))) - 1 for _ in range(N_HASH)], np.uint32)
    h1, h2, h3 = [], [], []
    for k in range(N_HASH):
        a = [int(x) for x in t[k]]
        h3.append(ref.ref_hash3(*a))
        h2.append(ref.ref_hash2(*a))
        h1.append(ref.ref_hash1(int(masks[k]), *a))
    a6 = rng.integers(0, 256, size=(N_HASH, 16), dtype=np.uint8)
    ax = [ref.ref_addr_xor(_buf(a6[k].tobytes())) for k in range(N_HASH)]
    np.savez_compressed(os.path.join(HERE, "ref_hash_vectors.npz"),
                        tuples=t.astype(np.uint32), masks=masks,
                        hash1=np.array(h1, np.uint32), hash2=np.array(h2, np.uint32),
                        hash3=np.array(h3, np.uint32), addr6=a6,
                        addr_xor=np.array(ax, np.uint32))

    # The reference unit test's known answers (checksum.c:13-62): data only.
    ipdata = bytes([0x45, 0x00, 0x00, 0x3c, 0x73, 0x63, 0x40, 0x00, 0x40, 0x06, 0x9e, 0x66,
                    0x0a, 0x78, 0x0a, 0x02, 0x0a, 0x78, 0x0a, 0x01])
    tcpdata = bytes([0xa9, 0xf6, 0x52, 0x13, 0x08, 0x15, 0xf7, 0x44, 0x00, 0x00, 0x00, 0x00,
                     0xa0, 0x02, 0xfa, 0xf0, 0xff, 0xff, 0x00, 0x00, 0x02, 0x04, 0x05, 0xb4,
                     0x04, 0x02, 0x08, 0x0a, 0x7f, 0xd1, 0xa8, 0xe7, 0x00, 0x00, 0x00, 0x00,
                     0x01, 0x03, 0x03, 0x07])
    udpdata = bytes([0xD6, 0xBE, 0x00, 0x13, 0x00, 0x15, 0x00, 0x00])
    json.dump({
        "source": "src/tests/unit/lib/ciul/checksum.c:13-62",
        "ip": ipdata.hex(), "tcp": tcpdata.hex(), "udp": udpdata.hex(),
        "expect": {
            "tcp_is_correct_check_ffff": True,
            "tcp_is_correct_check_0": True,
            "tcp_checksum_with_check_0": 0,
            "udp_is_correct_proto17": True,
            "udp_checksum_proto17": 0xFFFF,
        },
    }, open(os.path.join(HERE, "ref_unit_checksum.json"), "w"), indent=1)
    print(f"wrote {len(recs)} csum vectors, {N_HASH} hash vectors")


if __name__ == "__main__":
    main()
