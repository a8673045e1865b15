# SPDX-License-Identifier: BSD-2-Clause
"""Synthetic workloads of BASELINE.json's configurations (onload_amd/csrc/oo_pktgen.c)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _abi

MAX_FILTERS = 8192


def default_seed(config: int) -> int:
    return _abi.load_pktgen().oo_pg_default_seed(config)


def world(config: int):
    """(filters, socks) of a configuration's socket world."""
    pg = _abi.load_pktgen()
    filters = (_abi.PgFilter * MAX_FILTERS)()
    socks = (_abi.Sock * 8192)()
    n_socks = ctypes.c_int()
    nf = pg.oo_pg_world(config, filters, MAX_FILTERS, socks, 8192, ctypes.byref(n_socks))
    if nf < 0:
        raise ValueError(f"unknown config {config}")
    return list(filters[:nf]), list(socks[: n_socks.value])


def nbytes(config: int, seed: int, first: int, n: int, align: int = 64) -> int:
    return _abi.load_pktgen().oo_pg_bytes(config, seed, first, n, align)


def generate(config: int, n: int, seed: int | None = None, first: int = 0, align: int = 64,
             nthreads: int | None = None, out: np.ndarray | None = None):
    """Generate packets [first, first+n): returns (frames uint8 array, descriptors)."""
    pg = _abi.load_pktgen()
    if seed is None:
        seed = default_seed(config)
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    size = pg.oo_pg_bytes(config, seed, first, n, align)
    frames = out if out is not None else np.empty(size, dtype=np.uint8)
    if frames.nbytes < size:
        raise ValueError("frame buffer too small")
    desc = np.empty(n, dtype=_abi.DESC_DTYPE)
    used = pg.oo_pg_gen(config, seed, first, n, align, frames.ctypes.data, frames.nbytes,
                        desc.ctypes.data, nthreads)
    if used != size:
        raise RuntimeError("oo_pg_gen failed")
    return frames[:size], desc
