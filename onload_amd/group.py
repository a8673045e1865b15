# SPDX-License-Identifier: BSD-2-Clause
"""The multi-GPU group of the C ABI (include/oo_gpu_rx.h "Multi-GPU group";
SURVEY.md §8(b) "device ids", §8(e)) as a Python mirror.

One stack's batches spread over the GPUs of a node: every member holds a
replica of the filter tables, kept identical by applying the same changes
in the same order, and transforms a contiguous, byte-balanced share of each
batch.  In one process (``GpuRxGroup(devices=[...])``) the group drives
every member; across processes, one per GPU (``GpuRxGroup.join``), RCCL in
the library carries the table image, the changes and the records.
"""
from __future__ import annotations

import ctypes
import errno

import numpy as np

from . import _abi
from .rx import GpuRxStack

ID_BYTES = 128  # OO_GPU_RX_GROUP_ID_BYTES


class Shard(ctypes.Structure):
    """oo_gpu_rx_shard: one member's share of a batch."""
    _fields_ = [("d_frames", ctypes.c_void_p), ("frames_bytes", ctypes.c_uint64),
                ("d_desc", ctypes.c_void_p), ("n", ctypes.c_uint32), ("rsvd", ctypes.c_uint32),
                ("d_out", ctypes.c_void_p), ("d_counters", ctypes.c_void_p),
                ("stream", ctypes.c_void_p)]


assert ctypes.sizeof(Shard) == 56

# oo_gpu_rx_group_transport: a caller's collectives on host memory.
BCAST = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
REDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                          ctypes.c_uint32)
GATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                          ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))


class Transport(ctypes.Structure):
    _fields_ = [("arg", ctypes.c_void_p), ("bcast", BCAST), ("max_u32", REDUCE),
                ("sum_u32", REDUCE), ("gather", GATHER)]


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise OSError(-rc, f"{what}: {errno.errorcode.get(-rc, rc)}")
    return rc


def _cfg(device, max_socks, ip4_log2, ip6_log2, intf_hwport):
    cfg = _abi.Cfg()
    cfg.device = device
    cfg.max_socks = max_socks
    cfg.ip4_table_log2 = ip4_log2
    cfg.ip6_table_log2 = ip6_log2
    cfg.n_intf = len(intf_hwport)
    for i, h in enumerate(intf_hwport):
        cfg.intf_hwport[i] = h
    return cfg


class GpuRxGroup:
    def __init__(self, devices=(0,), max_socks: int = 8192, ip4_log2: int = 16,
                 ip6_log2: int = 14, intf_hwport=(0,), _join=None):
        self._lib = _abi.load_library()
        g = ctypes.c_void_p()
        if _join is not None and _join[0] == "transport":
            _, rank, nranks, t = _join
            cfg = _cfg(-1, max_socks, ip4_log2, ip6_log2, intf_hwport)
            self._transport = t  # the callbacks live as long as the group
            _check(self._lib.oo_gpu_rx_group_join_transport(ctypes.byref(g), ctypes.byref(cfg),
                                                            rank, nranks, ctypes.byref(t)),
                   "oo_gpu_rx_group_join_transport")
            self.devices = [-1]
        elif _join is None:
            devs = (ctypes.c_int32 * len(devices))(*devices)
            cfg = _cfg(0, max_socks, ip4_log2, ip6_log2, intf_hwport)
            _check(self._lib.oo_gpu_rx_group_open(ctypes.byref(g), ctypes.byref(cfg), devs,
                                                  len(devices)), "oo_gpu_rx_group_open")
            self.devices = list(devices)
        else:
            device, rank, nranks, gid = _join
            cfg = _cfg(device, max_socks, ip4_log2, ip6_log2, intf_hwport)
            buf = ctypes.create_string_buffer(bytes(gid), ID_BYTES)
            _check(self._lib.oo_gpu_rx_group_join(ctypes.byref(g), ctypes.byref(cfg), rank,
                                                  nranks, buf), "oo_gpu_rx_group_join")
            self.devices = [device]
        self._g = g
        self.max_socks = max_socks
        self.members = [GpuRxStack.wrap(self._lib.oo_gpu_rx_group_member(g, i), d, max_socks,
                                        self._lib)
                        for i, d in enumerate(self.devices)]

    @staticmethod
    def rccl_id() -> bytes:
        """Rank 0: a new communicator id (OO_GPU_RX_GROUP_ID_BYTES) to hand to
        every rank through the caller's own control plane."""
        lib = _abi.load_library()
        buf = ctypes.create_string_buffer(ID_BYTES)
        _check(lib.oo_gpu_rx_group_rccl_id(buf), "oo_gpu_rx_group_rccl_id")
        return buf.raw

    @classmethod
    def join(cls, device: int, rank: int, nranks: int, gid: bytes, **kw) -> "GpuRxGroup":
        """This process's member of a group across processes (one per GPU)."""
        return cls(_join=(device, rank, nranks, gid), **kw)

    @classmethod
    def join_transport(cls, rank: int, nranks: int, transport: Transport, **kw) -> "GpuRxGroup":
        """This process's host-only member of a group whose collectives run
        over the caller's transport (oo_gpu_rx_group_join_transport)."""
        return cls(_join=("transport", rank, nranks, transport), **kw)

    @property
    def rank(self) -> int:
        return int(self._lib.oo_gpu_rx_group_rank(self._g))

    @property
    def uses_rccl(self) -> bool:
        """True for a joined group: its collectives run over librccl."""
        return bool(self._lib.oo_gpu_rx_group_uses_rccl(self._g))

    def close(self) -> None:
        if self._g:
            rc = self._lib.oo_gpu_rx_group_close(self._g)
            if rc:  # -EBUSY: a member holds registered host memory; nothing closed
                raise OSError(-rc, "oo_gpu_rx_group_close: unregister host memory first")
            for m in self.members:
                m._ctx = None
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- table changes on every replica --------------------------------
    def filter_insert_raw(self, sock_id, af, laddr: bytes, lport_be, raddr, rport_be, proto):
        return self._lib.oo_gpu_rx_group_table_insert(self._g, af, laddr, lport_be, raddr,
                                                       rport_be, proto, sock_id)

    def filter_remove_raw(self, sock_id, af, laddr: bytes, lport_be, raddr, rport_be, proto):
        return self._lib.oo_gpu_rx_group_table_remove(self._g, af, laddr, lport_be, raddr,
                                                       rport_be, proto, sock_id)

    def sock_set(self, sock_id: int, sock: _abi.Sock) -> int:
        return self._lib.oo_gpu_rx_group_sock_set(self._g, sock_id, ctypes.byref(sock))

    def load_world(self, filters, socks) -> None:
        """Install a generator world (onload_amd.pktgen.world) on every replica."""
        GpuRxStack.load_world(self, filters, socks)

    # -- batches --------------------------------------------------------
    def split(self, desc: np.ndarray, parts: int | None = None) -> list[tuple[int, int]]:
        """Byte-balanced contiguous shares of a batch: [(first, count)]."""
        parts = parts or len(self.members)
        d = np.ascontiguousarray(desc)
        first = (ctypes.c_uint32 * (parts + 1))()
        _check(self._lib.oo_gpu_rx_group_split(self._g, d.ctypes.data, len(d), parts, first),
               "oo_gpu_rx_group_split")
        return [(int(first[k]), int(first[k + 1] - first[k])) for k in range(parts)]

    def process(self, shards) -> None:
        arr = (Shard * len(shards))(*shards)
        _check(self._lib.oo_gpu_rx_group_process(self._g, arr), "oo_gpu_rx_group_process")

    def gather(self, shards, dst: int, counters: np.ndarray | None = None) -> None:
        arr = (Shard * len(shards))(*shards)
        c = None if counters is None else counters.ctypes.data
        _check(self._lib.oo_gpu_rx_group_gather(self._g, arr, dst, c), "oo_gpu_rx_group_gather")

    # -- across processes -------------------------------------------------
    def share_tables(self, stream: int = 0) -> None:
        _check(self._lib.oo_gpu_rx_group_share_tables(self._g, stream),
               "oo_gpu_rx_group_share_tables")

    def share_ops(self, stream: int = 0) -> int:
        return _check(self._lib.oo_gpu_rx_group_share_ops(self._g, stream),
                      "oo_gpu_rx_group_share_ops")

    def gather_rccl(self, d_out: int, n: int, d_dst: int = 0, counts=None, stream: int = 0):
        c = None if counts is None else (ctypes.c_uint32 * len(counts))(*counts)
        _check(self._lib.oo_gpu_rx_group_gather_rccl(self._g, d_out, n, d_dst, c, stream),
               "oo_gpu_rx_group_gather_rccl")

    def sum_counters(self, d_counters: int, stream: int = 0) -> None:
        _check(self._lib.oo_gpu_rx_group_sum_counters(self._g, d_counters, stream),
               "oo_gpu_rx_group_sum_counters")
