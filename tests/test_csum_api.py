# SPDX-License-Identifier: BSD-2-Clause
"""The boundary's host-pure checksum verifiers (include/oo_gpu_rx.h,
SURVEY.md §8(b)) against the reference's own verdicts.

tests/c/csum_api_check.c is compiled here with gcc against the header alone
(plus the system's wire-header structs) and linked with -loo_gpu_rx, the way a
reference-side C caller would use it; it replays tests/golden/
ref_csum_vectors.npz (verdicts of the reference's compiled checksum.c /
ip_csum_partial.c, tests/golden/make_golden.py) through every entry-point
shape.  No GPU is touched: these functions are host-pure."""
import ctypes
import json
import os
import struct
import subprocess

import numpy as np

from onload_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _write_vectors(tmp_path):
    d = np.load(os.path.join(GOLD, "ref_csum_vectors.npz"))
    meta, blob = d["meta"], d["blob"].tobytes()
    out = bytearray(struct.pack("<I", len(meta)))
    off = 0
    for m in meta:
        n3, n4, npay = int(m["l3len"]), int(m["l4len"]), int(m["paylen"])
        out += struct.pack("<6I", int(m["af"]), int(m["proto"]), n3, n4, npay, int(m["ok"]))
        out += blob[off: off + n3 + n4 + npay]
        off += n3 + n4 + npay
    assert off == len(blob)
    l4 = tmp_path / "l4.bin"
    l4.write_bytes(bytes(out))
    ip = bytearray(struct.pack("<I", len(d["ip_ok"])))
    for h, mx, ok in zip(d["ip_hdr"], d["ip_max"], d["ip_ok"]):
        ip += h.tobytes() + struct.pack("<iI", int(mx), int(ok))
    ipf = tmp_path / "ip.bin"
    ipf.write_bytes(bytes(ip))
    return l4, ipf, len(meta) * 4 + len(d["ip_ok"])


def test_c_caller_against_reference_verdicts(tmp_path):
    exe = tmp_path / "csum_api_check"
    libdir = os.path.dirname(_abi.LIB_PATH)
    subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "csum_api_check.c"), "-o", str(exe),
                    "-L", libdir, "-loo_gpu_rx", f"-Wl,-rpath,{libdir}"], check=True)
    l4, ip, n = _write_vectors(tmp_path)
    r = subprocess.run([str(exe), str(l4), str(ip)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == f"checked {n} mismatches 0"


def test_unit_test_known_answers_through_abi():
    """src/tests/unit/lib/ciul/checksum.c:13-62 through the product's
    verifiers: TCP SYN with options passes with check 0xffff and with 0
    (0 == 0xffff in one's complement); as UDP with an 8-B header it passes."""
    lib = _abi.load_library()
    d = json.load(open(os.path.join(GOLD, "ref_unit_checksum.json")))
    ip, tcp, udp = (bytearray(bytes.fromhex(d[k])) for k in ("ip", "tcp", "udp"))
    buf = ctypes.create_string_buffer
    iov = _abi.IoVec(None, 0)

    def tcp_ok():
        return lib.oo_rx_tcp_csum_ok(buf(bytes(ip)), buf(bytes(tcp)), ctypes.byref(iov), 1) != 0

    assert tcp_ok() == bool(d["expect"]["tcp_is_correct_check_ffff"])
    tcp[16:18] = b"\0\0"
    assert tcp_ok() == bool(d["expect"]["tcp_is_correct_check_0"])
    ip[9] = 17
    got = lib.oo_rx_udp_csum_ok(buf(bytes(ip)), buf(bytes(udp)), ctypes.byref(iov), 1) != 0
    assert got == bool(d["expect"]["udp_is_correct_proto17"])
