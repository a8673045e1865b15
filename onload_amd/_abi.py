# SPDX-License-Identifier: BSD-2-Clause
"""ctypes/numpy mirror of the C ABI in include/oo_gpu_rx.h.

Loads the in-tree gfx950 library ``onload_amd/liboo_gpu_rx.so`` and fails
loudly when it is missing: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboo_gpu_rx.so")
PKTGEN_PATH = os.path.join(_HERE, "liboo_pktgen.so")

ABI_VERSION = 5
MAX_INTF = 32

# Reason codes (oo_gpu_rx.h), in the reference's check order.
R_DELIVER, R_NO_MATCH, R_IP4_FRAG, R_IP4_OPTS_BAD, R_TCP_SCATTERED = 0, 1, 2, 3, 4
R_DROP_BASE = 16
R_SHORT_L2, R_NOT_IP, R_IP4_LEN, R_IP4_CSUM, R_IP6_LEN = 16, 17, 18, 19, 20
R_PROTO_OTHER, R_TCP_SHORT, R_TCP_CSUM, R_UDP_SHORT, R_UDP_CSUM = 21, 22, 23, 24, 25
R_COUNT = 32
REASON_NAMES = {
    0: "DELIVER", 1: "NO_MATCH", 2: "IP4_FRAG", 3: "IP4_OPTS_BAD", 4: "TCP_SCATTERED",
    16: "SHORT_L2", 17: "NOT_IP", 18: "IP4_LEN", 19: "IP4_CSUM", 20: "IP6_LEN",
    21: "PROTO_OTHER", 22: "TCP_SHORT", 23: "TCP_CSUM", 24: "UDP_SHORT", 25: "UDP_CSUM",
}

F_IP6, F_VLAN, F_CSUM_OK, F_MCAST, F_MULTI, F_TSO = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
F_UDP_S2 = 0x40
SOCK_CONNECTED, SOCK_BIND2DEV = 0x1, 0x2

DESC_DTYPE = np.dtype([("frame_off", "<u8"), ("len", "<u2"), ("intf_i", "<i2"),
                       ("rsvd", "<u4")])
RESULT_DTYPE = np.dtype([
    ("reason", "u1"), ("flags", "u1"), ("stage", "u1"), ("proto", "u1"),
    ("vlan", "<u2"), ("l4_off", "<u2"), ("ip_paylen", "<u2"), ("sport_be", "<u2"),
    ("dport_be", "<u2"), ("nmatch", "<u2"), ("saddr_be", "<u4"), ("daddr_be", "<u4"),
    ("sock", "<i4"), ("hash3", "<u4")])
# struct xdp_desc (<linux/if_xdp.h>), an AF_XDP RX ring entry.
XDP_DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
assert DESC_DTYPE.itemsize == 16 and RESULT_DTYPE.itemsize == 32
assert XDP_DESC_DTYPE.itemsize == 16


class Sock(ctypes.Structure):
    """oo_gpu_rx_sock: the socket-side fields the demux reads."""
    _fields_ = [("raddr_be32", ctypes.c_uint32), ("rport_be16", ctypes.c_uint16),
                ("lport_be16", ctypes.c_uint16), ("protocol", ctypes.c_uint8),
                ("rsvd0", ctypes.c_uint8), ("flags", ctypes.c_uint16),
                ("bind2dev_vlan", ctypes.c_int16), ("rsvd1", ctypes.c_uint16),
                ("bind2dev_hwports", ctypes.c_uint64), ("raddr6", ctypes.c_uint8 * 16),
                ("rsvd2", ctypes.c_uint8 * 8)]


class Cfg(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_socks", ctypes.c_uint32),
                ("ip4_table_log2", ctypes.c_uint8), ("ip6_table_log2", ctypes.c_uint8),
                ("n_intf", ctypes.c_uint8), ("rsvd", ctypes.c_uint8),
                ("intf_hwport", ctypes.c_uint8 * MAX_INTF),
                ("host_stage_bytes", ctypes.c_uint64), ("host_stage_pkts", ctypes.c_uint32),
                ("rsvd2", ctypes.c_uint32)]


assert ctypes.sizeof(Sock) == 48


class Tuning(ctypes.Structure):
    """oo_gpu_rx_tuning (launch settings, results unchanged)."""
    _fields_ = [("path", ctypes.c_uint32), ("grid_pct", ctypes.c_uint32),
                ("groups", ctypes.c_uint32), ("gshift", ctypes.c_int32),
                ("static_tiles", ctypes.c_uint32), ("tail_tile", ctypes.c_uint32),
                ("tail_per_wave", ctypes.c_uint32), ("tstep", ctypes.c_uint32),
                ("body_bpc", ctypes.c_uint32), ("body_tail", ctypes.c_uint32),
                ("body_engine", ctypes.c_uint32), ("walks", ctypes.c_uint32)]


#: The measurement settings tests and tools pass through the environment of
#: the *Python* process (the C library reads none): variable -> field.
TUNING_ENV = {"OO_RX_KERNEL": "path", "OO_RX_GRID_PCT": "grid_pct", "OO_RX_GROUPS": "groups",
              "OO_RX_GSHIFT": "gshift", "OO_RX_STATIC": "static_tiles",
              "OO_RX_TAIL_TILE": "tail_tile", "OO_RX_TAIL_PER_WAVE": "tail_per_wave",
              "OO_RX_TSTEP": "tstep", "OO_RX_BODY_BPC": "body_bpc", "OO_RX_BODY_TAIL": "body_tail",
              "OO_RX_BODY_ENGINE": "body_engine", "OO_RX_WALKS": "walks"}


def tuning_from_env() -> "Tuning | None":
    t = Tuning()
    t.gshift = -1
    seen = False
    for var, field in TUNING_ENV.items():
        v = os.environ.get(var)
        if v:
            setattr(t, field, int(v, 0))
            seen = True
    return t if seen else None


class PgFilter(ctypes.Structure):
    """oo_pg_filter (onload_amd/csrc/oo_pktgen.h)."""
    _fields_ = [("sock", ctypes.c_int32), ("af", ctypes.c_uint8), ("proto", ctypes.c_uint8),
                ("lport_be", ctypes.c_uint16), ("rport_be", ctypes.c_uint16),
                ("raddr_any", ctypes.c_uint8), ("rsvd", ctypes.c_uint8),
                ("laddr", ctypes.c_uint8 * 16), ("raddr", ctypes.c_uint8 * 16)]


# struct iovec (<sys/uio.h>), for the host-pure verifiers.
class TableStats(ctypes.Structure):
    """oo_gpu_rx_table_stats."""
    _fields_ = [("flushes", ctypes.c_uint64), ("index_rebuilds", ctypes.c_uint64),
                ("index_updates", ctypes.c_uint64), ("index_on", ctypes.c_uint32),
                ("rsvd", ctypes.c_uint32)]


class IoVec(ctypes.Structure):
    _fields_ = [("iov_base", ctypes.c_void_p), ("iov_len", ctypes.c_size_t)]


# Table image header (oo_gpu_rx.h, oo_gpu_rx_table_export).
IMAGE_HDR_DTYPE = np.dtype([("magic", "<u4"), ("version", "<u4"), ("ip4_log2", "<u4"),
                            ("ip6_log2", "<u4"), ("max_socks", "<u4"), ("rsvd0", "<u4"),
                            ("off_slot4", "<u8"), ("off_rc4", "<u8"), ("off_slot6", "<u8"),
                            ("off_socks", "<u8"), ("total", "<u8")])
SLOT4_DTYPE = np.dtype([("id_state", "<u4"), ("laddr", "<u4"), ("raddr", "<u4"), ("lport", "<u2"),
                        ("rport", "<u2"), ("proto", "u1"), ("rsvd0", "u1"), ("sflags", "<u2"),
                        ("b2d_vlan", "<i2"), ("rsvd1", "<u2"), ("hwports", "<u8")])
SLOT6_DTYPE = np.dtype([("id", "<i4"), ("route_count", "<i4"), ("laddr", "<u4", 4),
                        ("raddr", "<u4", 4), ("lport", "<u2"), ("rport", "<u2"), ("proto", "u1"),
                        ("rsvd1", "u1"), ("sflags", "<u2"), ("b2d_vlan", "<i2"), ("rsvd2", "<u2"),
                        ("rsvd3", "<u4"), ("hwports", "<u8")])
assert IMAGE_HDR_DTYPE.itemsize == 64 and SLOT4_DTYPE.itemsize == 32 and SLOT6_DTYPE.itemsize == 64


def parse_image(img: np.ndarray) -> dict:
    """Split a table image (uint8 array) into its parts."""
    h = img[:64].view(IMAGE_HDR_DTYPE)[0]
    n4, n6 = 1 << int(h["ip4_log2"]), 1 << int(h["ip6_log2"])
    o4, orc, o6, os_ = (int(h[k]) for k in ("off_slot4", "off_rc4", "off_slot6", "off_socks"))
    return {"hdr": h,
            "slot4": img[o4:o4 + 32 * n4].view(SLOT4_DTYPE),
            "rc4": img[orc:orc + 4 * n4].view("<i4"),
            "slot6": img[o6:o6 + 64 * n6].view(SLOT6_DTYPE),
            "socks": img[os_:int(h["total"])]}


# Every symbol include/oo_gpu_rx.h declares, with its ctypes signature.
_P, _U8, _U16, _U32, _U64, _I32 = (ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16,
                                   ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32)
ABI_SYMBOLS = {
    "oo_gpu_rx_abi_version": (ctypes.c_int, []),
    "oo_gpu_rx_open": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(Cfg)]),
    "oo_gpu_rx_close": (ctypes.c_int, [_P]),
    "oo_gpu_rx_table_insert": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8, _I32]),
    "oo_gpu_rx_table_remove": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8, _I32]),
    "oo_gpu_rx_table_lookup": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8]),
    "oo_gpu_rx_table_slot": (ctypes.c_int, [_P, ctypes.c_int, _U32, ctypes.POINTER(_U32),
                                            ctypes.POINTER(_I32), ctypes.POINTER(_U16)]),
    "oo_gpu_rx_sock_set": (ctypes.c_int, [_P, _I32, ctypes.POINTER(Sock)]),
    "oo_gpu_rx_sync_tables": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_stream_done": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_table_gen": (ctypes.c_uint64, [_P]),
    "oo_gpu_rx_last_path": (ctypes.c_uint32, [_P]),
    "oo_gpu_rx_get_table_stats": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_set_len_hint": (ctypes.c_int, [_P, _U32]),
    "oo_gpu_rx_set_tuning": (ctypes.c_int, [_P, ctypes.POINTER(Tuning)]),
    "oo_gpu_rx_process_dev": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _P, _P, _P]),
    "oo_gpu_tx_fill_dev": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _P]),
    "oo_gpu_rx_xdp_dev": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _U32, _U32, ctypes.c_int,
                                         _P, _P, _P]),
    "oo_gpu_rx_xdp_poll": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _P, _P, _U32, ctypes.c_int,
                                          _P, _P, _P]),
    "oo_gpu_rx_batch": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _P, _P]),
    "oo_gpu_rx_submit": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _P, _P, ctypes.POINTER(_U64)]),
    "oo_gpu_rx_wait": (ctypes.c_int, [_P, _U64]),
    "oo_gpu_rx_submit_mapped": (ctypes.c_int, [_P, _P, _U64, _P, _U32, _P, ctypes.POINTER(_U64)]),
    "oo_gpu_rx_host_register": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_P)]),
    "oo_gpu_rx_host_unregister": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_host_registered": (ctypes.c_int, [_P]),
    "oo_gpu_rx_table_image_bytes": (_U64, [_P]),
    "oo_gpu_rx_table_export": (ctypes.c_int, [_P, _P, _U64, _P]),
    "oo_gpu_rx_table_import": (ctypes.c_int, [_P, _P, _U64, _P]),
    "oo_rx_ip_csum_ok": (ctypes.c_int, [_P, ctypes.c_int]),
    "oo_rx_udp_csum_ok": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "oo_rx_udp_csum_ok_ip6": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "oo_rx_tcp_csum_ok": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "oo_rx_tcp_csum_ok_ip6": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "oo_rx_udp_csum_ok_ipx": (ctypes.c_int, [ctypes.c_int, _P, _P, _P, ctypes.c_size_t]),
    "oo_rx_tcp_csum_ok_ipx": (ctypes.c_int, [ctypes.c_int, _P, _P, _P, ctypes.c_size_t]),
    "oo_gpu_rx_reason_str": (ctypes.c_char_p, [ctypes.c_int]),
    # multi-GPU group (onload_amd/group.py)
    "oo_gpu_rx_group_open": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(Cfg),
                                            ctypes.POINTER(_I32), _U32]),
    "oo_gpu_rx_group_rccl_id": (ctypes.c_int, [_P]),
    "oo_gpu_rx_group_join": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(Cfg), _U32, _U32,
                                            _P]),
    "oo_gpu_rx_group_join_transport": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(Cfg),
                                                      _U32, _U32, _P]),
    "oo_gpu_rx_group_close": (ctypes.c_int, [_P]),
    "oo_gpu_rx_group_size": (_U32, [_P]),
    "oo_gpu_rx_group_rank": (_U32, [_P]),
    "oo_gpu_rx_group_member": (_P, [_P, _U32]),
    "oo_gpu_rx_group_table_insert": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8,
                                                    _I32]),
    "oo_gpu_rx_group_table_remove": (ctypes.c_int, [_P, ctypes.c_int, _P, _U16, _P, _U16, _U8,
                                                    _I32]),
    "oo_gpu_rx_group_sock_set": (ctypes.c_int, [_P, _I32, ctypes.POINTER(Sock)]),
    "oo_gpu_rx_group_split": (ctypes.c_int, [_P, _P, _U32, _U32, ctypes.POINTER(_U32)]),
    "oo_gpu_rx_group_process": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_group_gather": (ctypes.c_int, [_P, _P, _P, _P]),
    "oo_gpu_rx_group_share_tables": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_group_share_ops": (ctypes.c_int, [_P, _P]),
    "oo_gpu_rx_group_gather_rccl": (ctypes.c_int, [_P, _P, _U32, _P, ctypes.POINTER(_U32), _P]),
    "oo_gpu_rx_group_sum_counters": (ctypes.c_int, [_P, _P, _P]),
    "oo_gpu_rx_group_uses_rccl": (ctypes.c_int, [_P]),
}

_lib = None


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load the gfx950 library.  Raises if it was not built (no fallback).

    OO_RX_LIB may name another build of the same library (the tuning
    variants of `make variants`)."""
    global _lib
    if _lib is not None:
        return _lib
    if path is None:
        path = os.environ.get("OO_RX_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(
            f"onload_amd: {path} is missing; build it with `make` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback for the receive transform.")
    try:  # share torch's HIP runtime when torch is present (same soname)
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    _lib = bind_library(path)
    return _lib


def bind_library(path: str) -> ctypes.CDLL:
    """dlopen one build of the library and declare its C ABI (a build with
    its own soname loads beside the product: tests/test_gpu_wait_variants.py)."""
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in ABI_SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.oo_gpu_rx_abi_version() != ABI_VERSION:
        raise RuntimeError("onload_amd: ABI version mismatch")
    return lib


_pg = None


def load_pktgen(path: str = PKTGEN_PATH) -> ctypes.CDLL:
    global _pg
    if _pg is not None:
        return _pg
    if not os.path.exists(path):
        raise RuntimeError(f"onload_amd: {path} is missing; run `make`")
    lib = ctypes.CDLL(path)
    lib.oo_pg_default_seed.restype = ctypes.c_uint64
    lib.oo_pg_default_seed.argtypes = [ctypes.c_int]
    lib.oo_pg_world.restype = ctypes.c_int
    lib.oo_pg_world.argtypes = [ctypes.c_int, ctypes.POINTER(PgFilter), ctypes.c_int,
                                ctypes.POINTER(Sock), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    lib.oo_pg_len.restype = ctypes.c_uint32
    lib.oo_pg_len.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
    lib.oo_pg_bytes.restype = ctypes.c_uint64
    lib.oo_pg_bytes.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                ctypes.c_uint32]
    lib.oo_pg_gen.restype = ctypes.c_uint64
    lib.oo_pg_gen.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                              ctypes.c_int]
    lib.oo_pg_split.restype = ctypes.c_int
    lib.oo_pg_split.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
    _pg = lib
    return lib
