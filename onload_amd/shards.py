# SPDX-License-Identifier: BSD-2-Clause
"""How a packet stream is spread over the GPUs of one node.

Packets are independent and the filter table is read-only during a batch,
so each rank (one process per GPU) owns a contiguous packet range and no
collective touches the data path.  What does move between ranks:

* the filter tables: built once on rank 0 (the stack that owns the socket
  world), broadcast as one table image (oo_gpu_rx_table_export / _import,
  ~3.4 MB at the default sizes) over RCCL, then kept current incrementally:
  rank 0 broadcasts each batch of filter ops (insert / remove / socket
  fields, 96 B each, broadcast_ops) and every rank applies it in order --
  the ops are deterministic, so the tables stay identical, return codes
  included (`oof` applies its deferred ops at the same serialisation point,
  oof_interface.c:184-217);
* optionally the frames, when they arrive on one ingest GPU: a scatter;
* optionally the 32-B records, gathered back to one rank.

Ranges are contiguous: equal packet counts for fixed-size traffic, equal
packed bytes (oo_pg_split) for IMIX / jumbo mixes so that every GPU streams
the same number of bytes.  These helpers take torch tensors and a
torch.distributed process group, so the same code runs over RCCL on GPUs and
over gloo on CPU tensors (tests/test_dist.py).
"""
from __future__ import annotations

import os

import numpy as np

from . import _abi

#: configurations whose frame sizes vary (byte-balanced shards)
MIXED_CONFIGS = (4, 5)


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """(first, count) of rank's contiguous, equal-count share of n_total."""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def split_bytes(config: int, seed: int, n_total: int, world: int, align: int = 64,
                nthreads: int | None = None) -> list[tuple[int, int]]:
    """Every rank's (first, count) when n_total packets of a configuration
    are split into contiguous ranges of equal packed bytes."""
    pg = _abi.load_pktgen()
    firsts = np.zeros(world + 1, dtype=np.uint64)
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    rc = pg.oo_pg_split(config, seed, n_total, world, align, firsts.ctypes.data, nthreads)
    if rc != 0:
        raise ValueError("oo_pg_split failed")
    return [(int(firsts[r]), int(firsts[r + 1] - firsts[r])) for r in range(world)]


def shard_for(config: int, seed: int, n_total: int, rank: int, world: int,
              align: int = 64) -> tuple[int, int]:
    """The shard bench.py and the tests use: by bytes for mixed sizes, by
    count otherwise."""
    if world > 1 and config in MIXED_CONFIGS:
        return split_bytes(config, seed, n_total, world, align)[rank]
    return shard_range(n_total, rank, world)


def broadcast_tables(stack, torch, dist, device, src: int = 0, stream: int = 0) -> int:
    """Replicate rank src's filter tables on every rank: src exports its
    table image into a tensor on `device`, one broadcast (RCCL on GPUs,
    gloo on CPU), every other rank imports it.  Returns the image size."""
    nbytes = stack.image_bytes()
    img = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if dist.get_rank() == src:
        stack.table_export(img.data_ptr(), nbytes, stream)
        if img.is_cuda:
            torch.cuda.current_stream(device).synchronize()
    dist.broadcast(img, src=src)
    if dist.get_rank() != src:
        if img.is_cuda:
            torch.cuda.current_stream(device).synchronize()
        stack.table_import(img.data_ptr(), nbytes, stream)
    return nbytes


#: one filter-table op as it travels between ranks
OP_INSERT, OP_REMOVE, OP_SOCK = 0, 1, 2
OP_DTYPE = np.dtype([("kind", "u1"), ("af", "u1"), ("proto", "u1"), ("raddr_any", "u1"),
                     ("lport_be", "<u2"), ("rport_be", "<u2"), ("sock", "<i4"), ("rsvd", "<u4"),
                     ("laddr", "u1", 16), ("raddr", "u1", 16), ("fields", "u1", 48)])
assert OP_DTYPE.itemsize == 96


def pack_ops(ops) -> np.ndarray:
    """Filter-table ops as OP_DTYPE records.  An op is
    ("insert" | "remove", sock_id, af, laddr bytes, lport_be, raddr bytes | None,
    rport_be, proto) -- ci_netif_filter_insert / _remove's arguments -- or
    ("sock", sock_id, _abi.Sock) -- the socket fields the demux reads."""
    out = np.zeros(len(ops), dtype=OP_DTYPE)
    for i, o in enumerate(ops):
        r = out[i]
        if o[0] == "sock":
            r["kind"], r["sock"] = OP_SOCK, o[1]
            r["fields"] = np.frombuffer(bytes(o[2]), dtype=np.uint8)
            continue
        kind, sock, af, la, lport_be, ra, rport_be, proto = o
        r["kind"] = OP_INSERT if kind == "insert" else OP_REMOVE
        r["sock"], r["af"], r["proto"] = sock, af, proto
        r["lport_be"], r["rport_be"] = lport_be, rport_be
        r["laddr"][: len(la)] = np.frombuffer(la, dtype=np.uint8)
        if ra is None:
            r["raddr_any"] = 1
        else:
            r["raddr"][: len(ra)] = np.frombuffer(ra, dtype=np.uint8)
    return out


def apply_ops(stack, recs: np.ndarray) -> list[int]:
    """Applies packed ops to a stack in order; returns their return codes."""
    rcs = []
    for r in recs:
        kind = int(r["kind"])
        if kind == OP_SOCK:
            rcs.append(stack.sock_set(int(r["sock"]), _abi.Sock.from_buffer_copy(r["fields"].tobytes())))
            continue
        n = 4 if int(r["af"]) == 4 else 16
        la = r["laddr"][:n].tobytes()
        ra = None if r["raddr_any"] else r["raddr"][:n].tobytes()
        f = stack.filter_insert_raw if kind == OP_INSERT else stack.filter_remove_raw
        rc = f(int(r["sock"]), int(r["af"]), la, int(r["lport_be"]), ra, int(r["rport_be"]),
               int(r["proto"]))
        rcs.append(0 if rc is None else int(rc))
    return rcs


def broadcast_ops(stack, ops, torch, dist, device, src: int = 0) -> list[int]:
    """One incremental table update on every rank: rank src packs its ops
    (pack_ops), one broadcast of the count and one of the records, and every
    rank -- src too -- applies them in order (apply_ops).  Other ranks pass
    ops=None.  Returns this rank's return codes (identical on every rank)."""
    cnt = torch.tensor([len(ops) if dist.get_rank() == src else 0], dtype=torch.int64,
                       device=device)
    dist.broadcast(cnt, src=src)
    n = int(cnt.item())
    buf = torch.zeros(n * OP_DTYPE.itemsize, dtype=torch.uint8, device=device)
    if dist.get_rank() == src and n:
        buf.copy_(torch.from_numpy(pack_ops(ops).view(np.uint8)))
    if n:
        dist.broadcast(buf, src=src)
    return apply_ops(stack, buf.cpu().numpy().view(OP_DTYPE))


def gather_records(records, count: int, torch, dist, dst: int = 0):
    """Gather every rank's records (a uint8 tensor of >= 32*count bytes) on
    rank dst in rank order; ranks may hold different counts.  Returns the
    concatenated uint8 tensor on dst, None elsewhere."""
    world = dist.get_world_size()
    dev = records.device
    counts = torch.tensor([count], dtype=torch.int64, device=dev)
    all_counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(all_counts, counts)
    cmax = int(max(int(c.item()) for c in all_counts))
    pad = torch.zeros(cmax * 32, dtype=torch.uint8, device=dev)
    pad[: count * 32] = records[: count * 32]
    if dist.get_rank() == dst:
        bufs = [torch.empty(cmax * 32, dtype=torch.uint8, device=dev) for _ in range(world)]
        dist.gather(pad, bufs, dst=dst)
        return torch.cat([b[: int(c.item()) * 32] for b, c in zip(bufs, all_counts)])
    dist.gather(pad, None, dst=dst)
    return None


def scatter_frames(shards, slab: int, torch, dist, device, src: int = 0):
    """Scatter per-rank frame buffers from rank src (a list of uint8
    tensors on src, one per rank, each <= slab bytes) into a slab on every
    rank; returns this rank's slab."""
    recv = torch.empty(slab, dtype=torch.uint8, device=device)
    send = None
    if dist.get_rank() == src:
        send = []
        for t in shards:
            s = torch.zeros(slab, dtype=torch.uint8, device=device)
            s[: t.numel()] = t
            send.append(s)
    dist.scatter(recv, send, src=src)
    return recv


def host_cores() -> int:
    """The host cores this process may use: its CPU affinity, bounded by a
    cgroup v2 CPU quota when one is set."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


__all__ = ["shard_range", "split_bytes", "shard_for", "broadcast_tables", "gather_records",
           "scatter_frames", "host_cores", "MIXED_CONFIGS", "pack_ops", "apply_ops",
           "broadcast_ops", "OP_DTYPE"]
