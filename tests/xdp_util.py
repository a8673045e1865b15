# SPDX-License-Identifier: BSD-2-Clause
"""AF_XDP layouts for the ring tests: a UMEM of 2048-B buffers with the
frames at varying headroom, and RX rings of struct xdp_desc entries
(efxdp_vi.c:309-358; buffer = addr / 2048, offset = addr & 2047)."""
from __future__ import annotations

import numpy as np

from onload_amd import _abi

CHUNK = 2048


def to_umem(frames: list[bytes], seed: int = 0, headroom=(192, 256)):
    """Frames into consecutive buffers, each at a random offset in
    [headroom[0], headroom[1]) of its first buffer (odd offsets included); a
    frame longer than the rest of its buffer runs on into the next ones, as a
    contiguous UMEM lays it out.  Returns (umem, entries in frame order)."""
    rng = np.random.default_rng(seed)
    ents = np.zeros(len(frames), dtype=_abi.XDP_DESC_DTYPE)
    parts = []
    chunk = 0
    for i, f in enumerate(frames):
        ofs = int(rng.integers(headroom[0], headroom[1]))
        nchunks = (ofs + len(f) + CHUNK - 1) // CHUNK
        blob = bytearray(rng.integers(0, 256, nchunks * CHUNK, dtype=np.uint8).tobytes())
        blob[ofs:ofs + len(f)] = f
        parts.append(bytes(blob))
        ents[i]["addr"] = chunk * CHUNK + ofs
        ents[i]["len"] = len(f)
        ents[i]["options"] = int(rng.integers(0, 1 << 32))
        chunk += nchunks
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy(), ents


def frames_of(buf: np.ndarray, desc: np.ndarray) -> list[bytes]:
    """The frames a packed (buffer, oo_gpu_pkt_desc[]) batch holds."""
    b = buf.tobytes()
    return [b[int(d["frame_off"]):int(d["frame_off"]) + int(d["len"])] for d in desc]


def ring_of(ents: np.ndarray, log2: int, cons: int, seed: int = 1):
    """A ring of 2^log2 entries holding ents at (cons + i) & mask, the other
    entries garbage."""
    size = 1 << log2
    assert len(ents) <= size
    rng = np.random.default_rng(seed)
    ring = np.zeros(size, dtype=_abi.XDP_DESC_DTYPE)
    ring["addr"] = rng.integers(0, 1 << 62, size, dtype=np.uint64)
    ring["len"] = rng.integers(0, 1 << 32, size, dtype=np.uint64).astype(np.uint32)
    idx = (cons + np.arange(len(ents), dtype=np.uint64)) & np.uint64(size - 1)
    ring[idx] = ents
    return ring, size - 1
