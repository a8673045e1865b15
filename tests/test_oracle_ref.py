# SPDX-License-Identifier: BSD-2-Clause
"""Pin the oracle's arithmetic to the reference's own code.

* tests/golden/ref_*.npz / .json were produced by tests/golden/make_golden.py
  from the reference's checksum.c, ip_csum_partial.c and hash.h compiled
  unmodified (oracle/_ref); they travel with the repo, so these tests need no
  reference at run time.
* When oracle/_ref/libref_rx.so is present, extra random vectors are checked
  against it live.
"""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle_lib import REF_PATH, oracle, ref_lib

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _b(x: bytes):
    return ctypes.create_string_buffer(bytes(x), max(len(x), 1))


def _verify(lib, af, proto, l3, l4, pay):
    fn = {(4, 17): lib.oo_or_udp4_ok, (6, 17): lib.oo_or_udp6_ok,
          (4, 6): lib.oo_or_tcp4_ok, (6, 6): lib.oo_or_tcp6_ok}[(af, proto)]
    return fn(_b(l3), _b(l4), _b(pay), len(pay))


def test_unit_test_known_answers():
    """src/tests/unit/lib/ciul/checksum.c:13-62 (5 checks)."""
    d = json.load(open(os.path.join(GOLD, "ref_unit_checksum.json")))
    ip, tcp, udp = (bytearray(bytes.fromhex(d[k])) for k in ("ip", "tcp", "udp"))
    lib = oracle()
    assert _verify(lib, 4, 6, ip, tcp, b"") == d["expect"]["tcp_is_correct_check_ffff"]
    tcp[16:18] = b"\0\0"
    assert _verify(lib, 4, 6, ip, tcp, b"") == d["expect"]["tcp_is_correct_check_0"]
    ip[9] = 17
    assert _verify(lib, 4, 17, ip, udp, b"") == d["expect"]["udp_is_correct_proto17"]


def test_csum_golden_vectors():
    d = np.load(os.path.join(GOLD, "ref_csum_vectors.npz"))
    meta, blob = d["meta"], d["blob"].tobytes()
    lib = oracle()
    off = 0
    bad = []
    for k, m in enumerate(meta):
        n3, n4, npay = int(m["l3len"]), int(m["l4len"]), int(m["paylen"])
        l3 = blob[off: off + n3]
        l4 = blob[off + n3: off + n3 + n4]
        pay = blob[off + n3 + n4: off + n3 + n4 + npay]
        off += n3 + n4 + npay
        got = _verify(lib, int(m["af"]), int(m["proto"]), l3, l4, pay)
        if int(got != 0) != int(m["ok"]):
            bad.append(k)
    assert off == len(blob)
    assert not bad, f"{len(bad)} vectors disagree with the reference, first {bad[:5]}"
    assert 0.3 < meta["ok"].mean() < 0.7  # both verdicts covered


def test_ip_header_golden_vectors():
    d = np.load(os.path.join(GOLD, "ref_csum_vectors.npz"))
    lib = oracle()
    got = np.array([lib.oo_or_ip4_hdr_ok(_b(h.tobytes()), int(mx))
                    for h, mx in zip(d["ip_hdr"], d["ip_max"])])
    np.testing.assert_array_equal((got != 0).astype(np.uint8), d["ip_ok"])
    assert d["ip_ok"].sum() > 50


def test_hash_golden_vectors():
    d = np.load(os.path.join(GOLD, "ref_hash_vectors.npz"))
    lib = oracle()
    for k in range(len(d["tuples"])):
        t = [int(x) for x in d["tuples"][k]]
        assert lib.oo_or_hash3(*t) == d["hash3"][k]
        assert lib.oo_or_hash2(*t) == d["hash2"][k]
        assert lib.oo_or_hash1(int(d["masks"][k]), *t) == d["hash1"][k]
        assert lib.oo_or_addr_xor(_b(d["addr6"][k].tobytes())) == d["addr_xor"][k]


@pytest.mark.skipif(not os.path.exists(REF_PATH),
                    reason="oracle/_ref not built (no /root/reference)")
def test_live_against_reference_random():
    """Fresh random vectors (odd lengths, check 0/ffff, IPv6) vs the reference."""
    ref, lib = ref_lib(), oracle()
    rng = np.random.default_rng(7)
    for k in range(3000):
        af = 4 if k % 3 else 6
        proto = 6 if k % 2 else 17
        paylen = int(rng.integers(0, 70))
        pay = rng.integers(0, 256, paylen, dtype=np.uint8).tobytes()
        l3 = bytearray(rng.integers(0, 256, 20 if af == 4 else 40, dtype=np.uint8).tobytes())
        l3[0] = 0x45 if af == 4 else 0x60
        if proto == 6:
            doff = int(rng.integers(5, 16))
            l4 = bytearray(rng.integers(0, 256, doff * 4, dtype=np.uint8).tobytes())
            l4[12] = (doff << 4) | (l4[12] & 15)
        else:
            l4 = bytearray(rng.integers(0, 256, 8, dtype=np.uint8).tobytes())
        # Force a near-valid check: set check so the sum is valid with prob ~1/2.
        for trial in range(2):
            fn_ref = ref.ref_tcp_ok if proto == 6 else ref.ref_udp_ok
            want = fn_ref(af, _b(l3), _b(l4), _b(pay), paylen)
            got = _verify(lib, af, proto, l3, l4, pay)
            assert (want != 0) == (got != 0), (k, af, proto, paylen)
            o = 16 if proto == 6 else 6
            l4[o:o + 2] = bytes([0, 0]) if trial == 0 else bytes([0xFF, 0xFF])
    # IPv4 header: every IHL, truncated max lengths
    for k in range(2000):
        h = bytearray(rng.integers(0, 256, 60, dtype=np.uint8).tobytes())
        h[0] = 0x40 | (k % 16)
        mx = int(rng.integers(0, 100))
        assert (ref.ref_ip_hdr_csum_ok(_b(h), mx) != 0) == (lib.oo_or_ip4_hdr_ok(_b(h), mx) != 0)
    for k in range(2000):
        t = [int(x) for x in rng.integers(0, 2**32, 5, dtype=np.uint64)]
        t[1] &= 0xFFFF
        t[3] &= 0xFFFF
        assert ref.ref_hash3(*t) == lib.oo_or_hash3(*t)
        assert ref.ref_hash2(*t) == lib.oo_or_hash2(*t)
