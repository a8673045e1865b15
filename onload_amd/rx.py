# SPDX-License-Identifier: BSD-2-Clause
"""Host-side mirror of Onload's RX-transform interface over the gfx950 library.

The reference's own entry points for this path are C:

* ``ci_netif_filter_insert`` / ``ci_netif_filter_remove``
  (src/lib/transport/ip/netif_table.c:436-503) -> :meth:`GpuRxStack.filter_insert`
  / :meth:`GpuRxStack.filter_remove` (same slot placement, ``-ENOBUFS`` when full);
* the socket fields the demux reads (``sock_raddr_be32`` ...,
  src/include/ci/internal/ip.h:1315-1340) -> :meth:`GpuRxStack.sock_set`;
* ``handle_rx_csum_bad`` (src/lib/transport/ip/netif_event.c:1014) run over a
  batch -> :meth:`GpuRxStack.handle_rx_batch` (host buffers) and
  :meth:`GpuRxStack.handle_rx_batch_dev` (HBM-resident buffers).  Its return
  value (1 = consumed, 0 = caller releases the packet) is
  ``results["reason"] < R_DROP_BASE``.

Addresses are network-order bytes (``bytes`` of length 4/16, or a dotted /
colon string); ports are host-order ints and are converted to the
network-order-in-host-integer form the reference uses.
"""
from __future__ import annotations

import ctypes
import errno
import ipaddress
import mmap
from typing import Optional, Union

import numpy as np

from . import _abi

Addr = Union[bytes, str, None]
PAGE = mmap.PAGESIZE


def htons(port: int) -> int:
    return ((port & 0xFF) << 8) | ((port >> 8) & 0xFF)


def addr_bytes(af: int, a: Addr) -> Optional[bytes]:
    if a is None:
        return None
    if isinstance(a, str):
        return ipaddress.ip_address(a).packed
    b = bytes(a)
    if len(b) != (4 if af == 4 else 16):
        raise ValueError(f"address length {len(b)} does not match af {af}")
    return b


class GpuRxStack:
    """One Onload stack's receive transform on one MI355X.

    ``ip4_log2`` >= 16 (netif_table.c:280), default 16 (ip.h:1790-1804);
    ``ip6_log2`` default 14 (netif_init.c:107-108); ``max_socks`` default 8192
    (EF_MAX_ENDPOINTS, opts_netif_def.h:1095-1108).
    """

    def __init__(self, device: int = 0, max_socks: int = 8192, ip4_log2: int = 16,
                 ip6_log2: int = 14, intf_hwport=(0,), host_stage_bytes: int = 0,
                 host_stage_pkts: int = 0, lib=None):
        self._lib = lib if lib is not None else _abi.load_library()
        cfg = _abi.Cfg()
        cfg.device = device
        cfg.max_socks = max_socks
        cfg.ip4_table_log2 = ip4_log2
        cfg.ip6_table_log2 = ip6_log2
        cfg.n_intf = len(intf_hwport)
        for i, h in enumerate(intf_hwport):
            cfg.intf_hwport[i] = h
        cfg.host_stage_bytes = host_stage_bytes
        cfg.host_stage_pkts = host_stage_pkts
        ctx = ctypes.c_void_p()
        rc = self._lib.oo_gpu_rx_open(ctypes.byref(ctx), ctypes.byref(cfg))
        if rc != 0:
            raise OSError(-rc, f"oo_gpu_rx_open: {errno.errorcode.get(-rc, rc)}")
        self._ctx = ctx
        self.device = device
        self.max_socks = max_socks
        self.host_stage_bytes = host_stage_bytes
        self.host_stage_pkts = host_stage_pkts
        t = _abi.tuning_from_env() if device >= 0 else None
        if t is not None:  # measurement settings of the Python process (tests, tools)
            self.set_tuning(t)

    def set_tuning(self, t: "_abi.Tuning | None") -> None:
        """oo_gpu_rx_set_tuning: launch settings (None: the defaults)."""
        rc = self._lib.oo_gpu_rx_set_tuning(self._ctx, ctypes.byref(t) if t is not None else None)
        if rc != 0:
            raise OSError(-rc, "oo_gpu_rx_set_tuning")

    @classmethod
    def wrap(cls, ctx, device: int, max_socks: int, lib) -> "GpuRxStack":
        """A view of a context another object owns (a group member): its
        calls work as for any stack; closing it is the owner's."""
        self = cls.__new__(cls)
        self._lib = lib
        self._ctx = ctypes.c_void_p(ctx)
        self._owned = False
        self.device = device
        self.max_socks = max_socks
        self.host_stage_bytes = self.host_stage_pkts = 0
        return self

    # -- lifetime -------------------------------------------------------
    def close(self) -> None:
        if not getattr(self, "_owned", True):
            self._ctx = None
            return
        if self._ctx:
            rc = self._lib.oo_gpu_rx_close(self._ctx)
            if rc:  # -EBUSY: host memory still registered; the context stays open
                raise OSError(-rc, "oo_gpu_rx_close: unregister host memory first")
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- filter table (ci_netif_filter_insert/remove) -------------------
    def _tuple(self, af, laddr, raddr):
        la = addr_bytes(af, laddr)
        ra = addr_bytes(af, raddr)
        return la, (None if ra is None else ra)

    def filter_insert(self, sock_id: int, af: int, laddr: Addr, lport: int,
                      raddr: Addr, rport: int, protocol: int) -> int:
        la, ra = self._tuple(af, laddr, raddr)
        return self._lib.oo_gpu_rx_table_insert(self._ctx, af, la, htons(lport), ra,
                                                 htons(rport), protocol, sock_id)

    def filter_insert_raw(self, sock_id, af, laddr: bytes, lport_be: int, raddr: Optional[bytes],
                          rport_be: int, protocol: int) -> int:
        return self._lib.oo_gpu_rx_table_insert(self._ctx, af, laddr, lport_be, raddr, rport_be,
                                                 protocol, sock_id)

    def filter_remove(self, sock_id: int, af: int, laddr: Addr, lport: int,
                      raddr: Addr, rport: int, protocol: int) -> int:
        la, ra = self._tuple(af, laddr, raddr)
        return self._lib.oo_gpu_rx_table_remove(self._ctx, af, la, htons(lport), ra,
                                                 htons(rport), protocol, sock_id)

    def filter_remove_raw(self, sock_id, af, laddr: bytes, lport_be: int,
                          raddr: Optional[bytes], rport_be: int, protocol: int) -> int:
        return self._lib.oo_gpu_rx_table_remove(self._ctx, af, laddr, lport_be, raddr, rport_be,
                                                 protocol, sock_id)

    def filter_lookup_raw(self, af, laddr: bytes, lport_be: int, raddr: Optional[bytes],
                          rport_be: int, protocol: int) -> int:
        return self._lib.oo_gpu_rx_table_lookup(self._ctx, af, laddr, lport_be, raddr, rport_be,
                                                 protocol)

    def filter_lookup(self, af: int, laddr: Addr, lport: int, raddr: Addr, rport: int,
                      protocol: int) -> int:
        la, ra = self._tuple(af, laddr, raddr)
        return self._lib.oo_gpu_rx_table_lookup(self._ctx, af, la, htons(lport), ra,
                                                 htons(rport), protocol)

    def table_slot(self, af: int, slot: int):
        st, rc_, lp = ctypes.c_uint32(), ctypes.c_int32(), ctypes.c_uint16()
        rc = self._lib.oo_gpu_rx_table_slot(self._ctx, af, slot, ctypes.byref(st),
                                            ctypes.byref(rc_), ctypes.byref(lp))
        if rc != 0:
            raise OSError(-rc, "oo_gpu_rx_table_slot")
        return st.value, rc_.value, lp.value

    def sock_set(self, sock_id: int, sock: "_abi.Sock") -> int:
        return self._lib.oo_gpu_rx_sock_set(self._ctx, sock_id, ctypes.byref(sock))

    def load_world(self, filters, socks) -> None:
        """Install a generator world (onload_amd.pktgen.world)."""
        for i, s in enumerate(socks):
            rc = self.sock_set(i, s)
            if rc:
                raise OSError(-rc, "sock_set")
        for f in filters:
            ra = None if f.raddr_any else bytes(f.raddr)[: 4 if f.af == 4 else 16]
            rc = self.filter_insert_raw(f.sock, f.af, bytes(f.laddr)[: 4 if f.af == 4 else 16],
                                        f.lport_be, ra, f.rport_be, f.proto)
            if rc:
                raise OSError(-rc, "filter_insert")

    def sync(self, stream: int = 0) -> None:
        rc = self._lib.oo_gpu_rx_sync_tables(self._ctx, ctypes.c_void_p(stream))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_sync_tables")

    def table_gen(self) -> int:
        """oo_gpu_rx_table_gen: table and socket changes made so far."""
        return int(self._lib.oo_gpu_rx_table_gen(self._ctx))

    def table_stats(self) -> dict:
        """oo_gpu_rx_get_table_stats: flushes, index rebuilds / incremental
        updates, and whether the key index is on (waits for the device)."""
        st = _abi.TableStats()
        rc = self._lib.oo_gpu_rx_get_table_stats(self._ctx, ctypes.byref(st))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_get_table_stats")
        return {n: int(getattr(st, n)) for n, _ in st._fields_ if n != "rsvd"}

    def last_path(self) -> int:
        """oo_gpu_rx_last_path: the last batch's kernels (1 / 2 rx_kernel
        instances, 3 / 4 the split transform with the lockstep / sequences
        body engine, 5 the poll instance, 0 none yet)."""
        return int(self._lib.oo_gpu_rx_last_path(self._ctx))

    def set_len_hint(self, mean_frame_len: int) -> None:
        """Mean frame length of the batches to come (0: inferred from the
        buffer bytes per packet); picks the kernel instance."""
        rc = self._lib.oo_gpu_rx_set_len_hint(self._ctx, int(mean_frame_len))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_set_len_hint")

    def stream_done(self, stream: int) -> None:
        """The caller is about to destroy `stream` (oo_gpu_rx_stream_done)."""
        rc = self._lib.oo_gpu_rx_stream_done(self._ctx, ctypes.c_void_p(stream))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_stream_done")

    # -- the transform --------------------------------------------------
    def handle_rx_batch_dev(self, frames_ptr: int, frames_bytes: int, desc_ptr: int, n: int,
                            out_ptr: int, counters_ptr: int = 0, stream: int = 0) -> None:
        """Enqueue the transform over HBM-resident buffers (device addresses)."""
        rc = self._lib.oo_gpu_rx_process_dev(self._ctx, ctypes.c_void_p(frames_ptr),
                                             frames_bytes, ctypes.c_void_p(desc_ptr), n,
                                             ctypes.c_void_p(out_ptr),
                                             ctypes.c_void_p(counters_ptr or None),
                                             ctypes.c_void_p(stream or None))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_process_dev")

    def tx_fill_dev(self, frames_ptr: int, frames_bytes: int, desc_ptr: int, n: int,
                    stream: int = 0) -> None:
        """Enqueue the TX checksum fill (oo_pkt_calc_checksums,
        src/lib/transport/ip/pkt_checksum.c:20-102) over HBM-resident frames,
        in place."""
        rc = self._lib.oo_gpu_tx_fill_dev(self._ctx, ctypes.c_void_p(frames_ptr), frames_bytes,
                                          ctypes.c_void_p(desc_ptr), n,
                                          ctypes.c_void_p(stream or None))
        if rc:
            raise OSError(-rc, "oo_gpu_tx_fill_dev")

    def xdp_dev(self, umem_ptr: int, umem_bytes: int, ring_ptr: int, ring_mask: int,
                cons: int, n: int, intf_i: int, out_ptr: int, counters_ptr: int = 0,
                stream: int = 0) -> None:
        """Enqueue the transform of n AF_XDP RX ring entries from consumer
        index cons (efxdp_ef_eventq_poll, src/lib/ciul/efxdp_vi.c:309-358);
        record i for entry (cons + i) & ring_mask."""
        rc = self._lib.oo_gpu_rx_xdp_dev(self._ctx, ctypes.c_void_p(umem_ptr), umem_bytes,
                                         ctypes.c_void_p(ring_ptr), ring_mask, cons, n,
                                         intf_i, ctypes.c_void_p(out_ptr),
                                         ctypes.c_void_p(counters_ptr or None),
                                         ctypes.c_void_p(stream or None))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_xdp_dev")

    def xdp_poll(self, umem_ptr: int, umem_bytes: int, ring_ptr: int, ring_mask: int,
                 consumer: np.ndarray, producer: np.ndarray, max_n: int, intf_i: int,
                 out_ptr: int, counters_ptr: int = 0, stream: int = 0) -> int:
        """One batched ring poll: consumes min(producer - consumer, max_n)
        entries, advances consumer[0] after the device has read them, returns
        the count."""
        assert consumer.dtype == np.uint32 and producer.dtype == np.uint32
        rc = self._lib.oo_gpu_rx_xdp_poll(self._ctx, ctypes.c_void_p(umem_ptr), umem_bytes,
                                          ctypes.c_void_p(ring_ptr), ring_mask,
                                          consumer.ctypes.data_as(ctypes.c_void_p),
                                          producer.ctypes.data_as(ctypes.c_void_p), max_n,
                                          intf_i, ctypes.c_void_p(out_ptr),
                                          ctypes.c_void_p(counters_ptr or None),
                                          ctypes.c_void_p(stream or None))
        if rc < 0:
            raise OSError(-rc, "oo_gpu_rx_xdp_poll")
        return rc

    # -- table image (replication across ranks) ----------
    def image_bytes(self) -> int:
        return int(self._lib.oo_gpu_rx_table_image_bytes(self._ctx))

    def table_export(self, dst_ptr: int, nbytes: int, stream: int = 0) -> None:
        """Copy the table image to dst (device memory; host memory for a
        host-only stack), asynchronously on `stream`."""
        rc = self._lib.oo_gpu_rx_table_export(self._ctx, ctypes.c_void_p(dst_ptr), nbytes,
                                              ctypes.c_void_p(stream or None))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_table_export")

    def table_import(self, src_ptr: int, nbytes: int, stream: int = 0) -> None:
        rc = self._lib.oo_gpu_rx_table_import(self._ctx, ctypes.c_void_p(src_ptr), nbytes,
                                              ctypes.c_void_p(stream or None))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_table_import")

    def image_host(self) -> np.ndarray:
        """The table image in host memory (host-only stacks)."""
        img = np.zeros(self.image_bytes(), dtype=np.uint8)
        self.table_export(img.ctypes.data, img.nbytes)
        return img

    # -- host memory the device reads directly --------------------------
    def host_register(self, arr: np.ndarray, nbytes: Optional[int] = None) -> int:
        """oo_gpu_rx_host_register: hipHostRegister (mapped) the whole pages
        holding the array -- from its first byte, which must start a page,
        through the page holding its last (nbytes: that many bytes instead,
        a multiple of the page size).  Those pages must be the caller's own
        (tests/hostmem.page_buffer); returns the device address."""
        if nbytes is None:
            nbytes = -(-arr.nbytes // PAGE) * PAGE
        d = ctypes.c_void_p()
        rc = self._lib.oo_gpu_rx_host_register(self._ctx, ctypes.c_void_p(arr.ctypes.data),
                                               nbytes, ctypes.byref(d))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_host_register")
        return int(d.value or 0)

    def host_unregister(self, arr: np.ndarray) -> None:
        rc = self._lib.oo_gpu_rx_host_unregister(self._ctx, ctypes.c_void_p(arr.ctypes.data))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_host_unregister")

    def host_registered(self) -> int:
        """oo_gpu_rx_host_registered: ranges the context holds."""
        return int(self._lib.oo_gpu_rx_host_registered(self._ctx))

    # -- asynchronous host-memory batches -------------------------------
    def submit(self, frames: np.ndarray, desc: np.ndarray, out: np.ndarray,
               delta: Optional[np.ndarray] = None) -> int:
        """Enqueue one host-memory batch; returns its ticket.  frames, desc,
        out (and delta) must stay alive and unchanged until wait()."""
        assert out.dtype == _abi.RESULT_DTYPE and len(out) >= len(desc)
        assert desc.dtype == _abi.DESC_DTYPE and desc.flags.c_contiguous
        t = ctypes.c_uint64()
        rc = self._lib.oo_gpu_rx_submit(
            self._ctx, ctypes.c_void_p(frames.ctypes.data), frames.nbytes,
            ctypes.c_void_p(desc.ctypes.data), len(desc), ctypes.c_void_p(out.ctypes.data),
            ctypes.c_void_p(None if delta is None else delta.ctypes.data), ctypes.byref(t))
        if rc:
            raise OSError(-rc, "oo_gpu_rx_submit")
        return t.value

    def wait(self, ticket: int) -> int:
        rc = self._lib.oo_gpu_rx_wait(self._ctx, ticket)
        if rc < 0:
            raise OSError(-rc, "oo_gpu_rx_wait")
        return rc

    def handle_rx_batch(self, frames: np.ndarray, desc: np.ndarray):
        """Host buffers in, (results, per-reason counters) out."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=_abi.DESC_DTYPE)
        n = len(desc)
        out = np.zeros(n, dtype=_abi.RESULT_DTYPE)
        ctr = np.zeros(_abi.R_COUNT, dtype=np.uint32)
        rc = self._lib.oo_gpu_rx_batch(self._ctx, frames.ctypes.data_as(ctypes.c_void_p),
                                       frames.nbytes, desc.ctypes.data_as(ctypes.c_void_p), n,
                                       out.ctypes.data_as(ctypes.c_void_p),
                                       ctr.ctypes.data_as(ctypes.c_void_p))
        if rc < 0:
            raise OSError(-rc, "oo_gpu_rx_batch")
        return out, ctr


def handled(results: np.ndarray) -> np.ndarray:
    """handle_rx_csum_bad's return value per packet (1 = consumed)."""
    return results["reason"] < _abi.R_DROP_BASE
