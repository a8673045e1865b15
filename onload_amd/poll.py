# SPDX-License-Identifier: BSD-2-Clause
"""ctypes mirror of include/oo_rx_poll.h: the batched ci_netif_poll_evq RX
branch (src/shim/oo_rx_poll.c, onload_amd/liboo_rx_poll.so).

``RxPoll`` drives the C shim with a Python callback table, the way the tests
(and a host integration written in Python) use it.  The shim links
liboo_gpu_rx.so; there is no CPU path behind it."""
from __future__ import annotations

import ctypes
import errno
import os

import numpy as np

from . import _abi

POLL_PATH = os.path.join(_abi._HERE, "liboo_rx_poll.so")

EV_SOP, EV_CONT = 0x1, 0x2
DISCARD_L4_CSUM_ERR, DISCARD_L3_CSUM_ERR = 0x001, 0x002
DISCARD_ETH_FCS_ERR, DISCARD_ETH_LEN_ERR = 0x004, 0x008
DISCARD_L3_CLASS_OTHER = 0x100
MAX_EVS = 65536

EV_DTYPE = np.dtype([("rq_id", "<u4"), ("ofs", "<u2"), ("len", "<u2"), ("flags", "<u2"),
                     ("discard", "<u2"), ("intf_i", "<i2"), ("rsvd", "<u2")])
assert EV_DTYPE.itemsize == 16


class Future(ctypes.Structure):
    _fields_ = [("sock", ctypes.c_int32), ("hash", ctypes.c_uint32), ("seq", ctypes.c_uint32),
                ("ack", ctypes.c_uint32), ("pay_len", ctypes.c_uint32),
                ("l4_off", ctypes.c_uint16), ("ip_paylen", ctypes.c_uint16)]


STAT_NAMES = ("rx_evs", "rx_sw_csum_pass", "rx_discard_csum_bad", "rx_discard_len_err",
              "rx_discard_crc_bad", "rx_discard_other", "ip_options", "in_recvs", "in_hdr_errs",
              "in_delivers", "in6_recvs", "in6_hdr_errs", "in6_delivers", "tcp_in_segs",
              "udp_in_dgrams", "udp_in_errs", "n_future", "n_future_declined", "n_full",
              "n_pkt_handler", "n_release", "n_other", "n_batches", "n_resubmit",
              "n_handback")


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in STAT_NAMES]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n in STAT_NAMES}


class Result(ctypes.Structure):
    """oo_gpu_rx_result as a ctypes struct (the callbacks receive a pointer)."""
    _fields_ = [(n, {"u1": ctypes.c_uint8, "<u2": ctypes.c_uint16, "<u4": ctypes.c_uint32,
                     "<i4": ctypes.c_int32}[_abi.RESULT_DTYPE.fields[n][0].str.replace("|", "")])
                for n in _abi.RESULT_DTYPE.names]


assert ctypes.sizeof(Result) == 32 and ctypes.sizeof(Future) == 24

_RP, _FP = ctypes.POINTER(Result), ctypes.POINTER(Future)
_U8P = ctypes.POINTER(ctypes.c_uint8)
POST_FUTURE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, _U8P, _RP, _FP)
HANDLER = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, _U8P, _RP)
OTHER_EV = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)


class Ops(ctypes.Structure):
    _fields_ = [("post_future", POST_FUTURE), ("full_handler", HANDLER),
                ("pkt_handler", HANDLER), ("release", HANDLER), ("other_ev", OTHER_EV),
                ("arg", ctypes.c_void_p)]


class PollCfg(ctypes.Structure):
    _fields_ = [("pkt_bufs", ctypes.c_void_p), ("pkt_bufs_bytes", ctypes.c_uint64),
                ("buf_size", ctypes.c_uint32), ("evs_per_poll", ctypes.c_uint32),
                ("sw_verify", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("cpu_pkt_ps", ctypes.c_uint32), ("cpu_byte_ps", ctypes.c_uint32),
                ("gpu_fixed_ns", ctypes.c_uint32), ("gpu_pkt_ps", ctypes.c_uint32),
                ("gpu_byte_ps", ctypes.c_uint32)]


ZERO_COPY = 0x1  # OO_RX_POLL_ZERO_COPY
CROSSOVER = 0x2  # OO_RX_POLL_CROSSOVER


POLL_SYMBOLS = {
    "oo_rx_poll_open": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                       ctypes.POINTER(PollCfg), ctypes.POINTER(Ops)]),
    "oo_rx_poll_close": (None, [ctypes.c_void_p]),
    "oo_rx_poll_evs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.POINTER(Stats)]),
    "oo_rx_poll_zero_copy": (ctypes.c_int, [ctypes.c_void_p]),
}

_lib = None


def load_poll(path: str = POLL_PATH) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    _abi.load_library()  # the shim's liboo_gpu_rx.so dependency, loaded first
    if not os.path.exists(path):
        raise RuntimeError(f"onload_amd: {path} is missing; build it with `make`")
    lib = ctypes.CDLL(path)
    for name, (res, args) in POLL_SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _rec(r) -> dict | None:
    if not r:
        return None
    c = r.contents
    return {n: int(getattr(c, n)) for n in _abi.RESULT_DTYPE.names}


class RxPoll:
    """One stack's batched RX branch.  ``handlers`` provides post_future(id,
    rec, future) -> int, full_handler(id, rec), pkt_handler(id, rec),
    release(id, rec_or_None) and other_ev(ev dict); records and futures reach
    it as dicts.  ``pool`` is the packet-buffer pool (a uint8 array kept
    alive by this object)."""

    def __init__(self, stack, pool: np.ndarray, buf_size: int, evs_per_poll: int,
                 sw_verify: bool, handlers, zero_copy: bool = False,
                 crossover: dict | None = None):
        self._lib = load_poll()
        self.pool = pool
        self.stack = stack  # the shim's context outlives it (its registrations are the shim's)
        self.h = handlers
        h = handlers
        fut = lambda a, i, f, r, fu: int(h.post_future(  # noqa: E731
            i, _rec(r), {n: int(getattr(fu.contents, n)) for n, _ in Future._fields_}))
        self._cb = Ops(POST_FUTURE(fut),
                       HANDLER(lambda a, i, f, r: h.full_handler(i, _rec(r))),
                       HANDLER(lambda a, i, f, r: h.pkt_handler(i, _rec(r))),
                       HANDLER(lambda a, i, f, r: h.release(i, _rec(r))),
                       OTHER_EV(lambda a, e: h.other_ev(
                           np.frombuffer(ctypes.string_at(e, 16), EV_DTYPE)[0])),
                       None)
        cfg = PollCfg(pool.ctypes.data, pool.nbytes, buf_size, evs_per_poll, int(sw_verify),
                      (ZERO_COPY if zero_copy else 0) | (CROSSOVER if crossover is not None else 0))
        for k, v in (crossover or {}).items():  # cost-model fields (0: defaults)
            setattr(cfg, k, int(v))
        p = ctypes.c_void_p()
        rc = self._lib.oo_rx_poll_open(ctypes.byref(p), stack._ctx, ctypes.byref(cfg),
                                       ctypes.byref(self._cb))
        if rc != 0:
            raise OSError(-rc, f"oo_rx_poll_open: {errno.errorcode.get(-rc, rc)}")
        self._p = p
        self.stats = Stats()

    def poll(self, evs: np.ndarray) -> int:
        evs = np.ascontiguousarray(evs, dtype=EV_DTYPE)
        return self._lib.oo_rx_poll_evs(self._p, evs.ctypes.data, len(evs),
                                        ctypes.byref(self.stats))

    @property
    def zero_copy(self) -> bool:
        """Frames are read in place (the pool is registered with the device)."""
        return self._lib.oo_rx_poll_zero_copy(self._p) == 1

    def close(self) -> None:
        if self._p:
            self._lib.oo_rx_poll_close(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
