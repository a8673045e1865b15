# SPDX-License-Identifier: BSD-2-Clause
"""ctypes binding of the CPU oracle (oracle/liboorx_oracle.so) and of the
reference's own compiled checksum/hash code (oracle/_ref/libref_rx.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from onload_amd import _abi
from onload_amd.rx import addr_bytes, htons

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboorx_oracle.so")
REF_PATH = os.path.join(ROOT, "oracle", "_ref", "libref_rx.so")

_P, _U8, _U16, _U32, _I32 = (ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32,
                             ctypes.c_int32)
_or = None


def oracle():
    global _or
    if _or is None:
        if not os.path.exists(ORACLE_PATH):
            raise RuntimeError("oracle/liboorx_oracle.so missing: run `make`")
        lib = ctypes.CDLL(ORACLE_PATH)
        sig = {
            "oo_or_tables_new": (_P, [ctypes.c_int, ctypes.c_int, _U32, _P, ctypes.c_int]),
            "oo_or_tables_free": (None, [_P]),
            "oo_or_tables_clone": (_P, [_P]),
            "oo_or_insert": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8, _I32]),
            "oo_or_remove": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8, _I32]),
            "oo_or_lookup": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8]),
            "oo_or_slot": (ctypes.c_int, [_P, ctypes.c_int, _U32, ctypes.POINTER(_U32),
                                          ctypes.POINTER(_I32), ctypes.POINTER(_U16)]),
            "oo_or_sock_set": (ctypes.c_int, [_P, _I32, ctypes.POINTER(_abi.Sock)]),
            "oo_or_dump": (_U32, [_P, _P, _U32]),
            "oo_or_rx_one": (None, [_P, _P, ctypes.c_int, ctypes.c_int, _P]),
            "oo_or_walk4": (ctypes.c_int, [_P, _U32, _U32, _U32, _U32, _U32, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.POINTER(_I32)]),
            "oo_or_rx_batch": (None, [_P, _P, ctypes.c_uint64, _P, _U32, _P, ctypes.c_int]),
            "oo_or_ip4_hdr_ok": (ctypes.c_int, [_P, ctypes.c_int]),
            "oo_or_udp4_ok": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t]),
            "oo_or_udp6_ok": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t]),
            "oo_or_tcp4_ok": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t]),
            "oo_or_tcp6_ok": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t]),
            "oo_or_hash3": (_U32, [_U32] * 5),
            "oo_or_hash1": (_U32, [_U32] * 6),
            "oo_or_hash2": (_U32, [_U32] * 5),
            "oo_or_addr_xor": (_U32, [_P]),
            "oo_or_tx_fill_one": (None, [_P, ctypes.c_int]),
            "oo_or_tx_fill_batch": (None, [_P, ctypes.c_uint64, _P, _U32]),
            "oo_or_xdp_batch": (None, [_P, _P, ctypes.c_uint64, _P, _U32, _U32, _U32,
                                       ctypes.c_int, _P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _or = lib
    return _or


def ref_lib():
    """The reference's own checksum.c/ip_csum_partial.c/hash.h, or None."""
    if not os.path.exists(REF_PATH):
        return None
    lib = ctypes.CDLL(REF_PATH)
    for name in ("ref_hash3", "ref_hash2"):
        getattr(lib, name).restype = _U32
        getattr(lib, name).argtypes = [_U32] * 5
    lib.ref_hash1.restype = _U32
    lib.ref_hash1.argtypes = [_U32] * 6
    lib.ref_addr_xor.restype = _U32
    lib.ref_addr_xor.argtypes = [_P]
    lib.ref_onload_hash3.restype = _U32
    lib.ref_onload_hash3.argtypes = [_P, _U32, _P, _U32, _U32]
    lib.ref_ip_hdr_csum_ok.restype = ctypes.c_int
    lib.ref_ip_hdr_csum_ok.argtypes = [_P, ctypes.c_int]
    for name in ("ref_udp_ok", "ref_tcp_ok"):
        getattr(lib, name).restype = ctypes.c_int
        getattr(lib, name).argtypes = [ctypes.c_int, _P, _P, _P, ctypes.c_size_t]
    lib.ef_udp_checksum.restype = _U32
    lib.ef_udp_checksum.argtypes = [_P, _P, _P, ctypes.c_int]
    lib.ef_tcp_checksum.restype = _U32
    lib.ef_tcp_checksum.argtypes = [_P, _P, _P, ctypes.c_int]
    lib.ef_udp_checksum_is_correct.restype = ctypes.c_int
    lib.ef_udp_checksum_is_correct.argtypes = [_P, _P, _P, ctypes.c_int]
    lib.ef_tcp_checksum_is_correct.restype = ctypes.c_int
    lib.ef_tcp_checksum_is_correct.argtypes = [_P, _P, _P, ctypes.c_int]
    return lib


class OracleStack:
    """The oracle with the same surface as onload_amd.GpuRxStack."""

    def __init__(self, max_socks=8192, ip4_log2=16, ip6_log2=14, intf_hwport=(0,)):
        self._lib = oracle()
        hw = (ctypes.c_uint8 * _abi.MAX_INTF)(*intf_hwport)
        self._t = self._lib.oo_or_tables_new(ip4_log2, ip6_log2, max_socks, hw, len(intf_hwport))
        if not self._t:
            raise ValueError("bad oracle table config")

    def close(self):
        if self._t:
            self._lib.oo_or_tables_free(self._t)
            self._t = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def filter_insert(self, sock_id, af, laddr, lport, raddr, rport, protocol):
        return self._lib.oo_or_insert(self._t, af, addr_bytes(af, laddr), htons(lport),
                                      addr_bytes(af, raddr), htons(rport), protocol, sock_id)

    def filter_insert_raw(self, sock_id, af, laddr, lport_be, raddr, rport_be, protocol):
        return self._lib.oo_or_insert(self._t, af, laddr, lport_be, raddr, rport_be, protocol,
                                      sock_id)

    def filter_remove_raw(self, sock_id, af, laddr, lport_be, raddr, rport_be, protocol):
        return self._lib.oo_or_remove(self._t, af, laddr, lport_be, raddr, rport_be, protocol,
                                      sock_id)

    def filter_lookup_raw(self, af, laddr, lport_be, raddr, rport_be, protocol):
        return self._lib.oo_or_lookup(self._t, af, laddr, lport_be, raddr, rport_be, protocol)

    def filter_remove(self, sock_id, af, laddr, lport, raddr, rport, protocol):
        return self._lib.oo_or_remove(self._t, af, addr_bytes(af, laddr), htons(lport),
                                      addr_bytes(af, raddr), htons(rport), protocol, sock_id)

    def filter_lookup(self, af, laddr, lport, raddr, rport, protocol):
        return self._lib.oo_or_lookup(self._t, af, addr_bytes(af, laddr), htons(lport),
                                      addr_bytes(af, raddr), htons(rport), protocol)

    def table_slot(self, af, slot):
        st, rc_, lp = ctypes.c_uint32(), ctypes.c_int32(), ctypes.c_uint16()
        rc = self._lib.oo_or_slot(self._t, af, slot, ctypes.byref(st), ctypes.byref(rc_),
                                  ctypes.byref(lp))
        if rc:
            raise OSError(-rc, "oo_or_slot")
        return st.value, rc_.value, lp.value

    def sock_set(self, sock_id, sock):
        return self._lib.oo_or_sock_set(self._t, sock_id, ctypes.byref(sock))

    def dump(self) -> np.ndarray:
        """Sparse table rows (af, slot, a, b, c, d) as the table fixtures hold them."""
        n = self._lib.oo_or_dump(self._t, None, 0)
        rows = np.zeros((n, 6), dtype=np.int64)
        self._lib.oo_or_dump(self._t, rows.ctypes.data, n)
        return rows

    def walk4(self, laddr_be, lport_be, raddr_be, rport_be, proto, intf_i=0, vlan=0, stop=False):
        """One IPv4 lookup stage (ci_netif_filter_for_each_match restated):
        (match count, first socket id or -1)."""
        first = ctypes.c_int32(-1)
        n = self._lib.oo_or_walk4(self._t, laddr_be, lport_be, raddr_be, rport_be, proto, intf_i,
                                  vlan, int(stop), ctypes.byref(first))
        return n, first.value

    def load_world(self, filters, socks):
        for i, s in enumerate(socks):
            assert self.sock_set(i, s) == 0
        for f in filters:
            ra = None if f.raddr_any else bytes(f.raddr)[: 4 if f.af == 4 else 16]
            rc = self.filter_insert_raw(f.sock, f.af, bytes(f.laddr)[: 4 if f.af == 4 else 16],
                                        f.lport_be, ra, f.rport_be, f.proto)
            assert rc == 0, rc

    def handle_rx_batch(self, frames: np.ndarray, desc: np.ndarray, nthreads: int = 1,
                        frames_bytes: int | None = None):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=_abi.DESC_DTYPE)
        out = np.zeros(len(desc), dtype=_abi.RESULT_DTYPE)
        nb = frames.nbytes if frames_bytes is None else min(frames_bytes, frames.nbytes)
        self._lib.oo_or_rx_batch(self._t, frames.ctypes.data, nb, desc.ctypes.data, len(desc),
                                 out.ctypes.data, nthreads)
        return out


    def handle_xdp_batch(self, umem: np.ndarray, ring: np.ndarray, mask: int, cons: int,
                         n: int, intf_i: int):
        umem = np.ascontiguousarray(umem, dtype=np.uint8)
        ring = np.ascontiguousarray(ring, dtype=_abi.XDP_DESC_DTYPE)
        out = np.zeros(n, dtype=_abi.RESULT_DTYPE)
        self._lib.oo_or_xdp_batch(self._t, umem.ctypes.data, umem.nbytes, ring.ctypes.data,
                                  mask, cons, n, intf_i, out.ctypes.data)
        return out


def counters_of(results: np.ndarray) -> np.ndarray:
    return np.bincount(results["reason"], minlength=_abi.R_COUNT).astype(np.uint32)


def oracle_tx_fill(buf: np.ndarray, desc: np.ndarray) -> np.ndarray:
    """oo_pkt_calc_checksums over a batch (the oracle's restatement), on a copy."""
    out = np.ascontiguousarray(buf).copy()
    d = np.ascontiguousarray(desc)
    oracle().oo_or_tx_fill_batch(out.ctypes.data, out.nbytes, d.ctypes.data, len(d))
    return out


def tx_golden():
    """(frames_in, frames_out, desc) of tests/golden/ref_tx_fill.npz, packed
    back to back."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "ref_tx_fill.npz"))
    lens = g["lens"].astype(np.int64)
    desc = np.zeros(len(lens), dtype=_abi.DESC_DTYPE)
    desc["frame_off"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    desc["len"] = lens
    return g["frames_in"].copy(), g["frames_out"].copy(), desc
