# SPDX-License-Identifier: BSD-2-Clause
"""Key-index placement statistics of a configuration's world (diagnostic).

Needs an experiment build (``make variants VARIANTS="exp:-DOO_RX_EXPERIMENTS"``,
selected with OO_RX_LIB): it exports the device index (oo_gpu_rx_debug_kx)
and prints, per region, the entries in use, each key's distance from its
home bucket / entry, and the share of home positions another key holds.

    OO_RX_LIB=build/var_exp.so python tools/kx_probe.py --config 5
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

M = 0xFFFFFFFF
KX_OVF = 64
KX_PAD4, KX_PAD6 = KX_OVF + 2, KX_OVF + 1


def kx_mix(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x7FEB352D) & M
    h ^= h >> 15
    h = (h * 0x846CA68B) & M
    h ^= h >> 16
    return h


def kx_fold(w: int) -> int:
    return w ^ (w >> 16)


def kx_hash(la, ra, ports, pw) -> int:
    """oo_rx_device.h kx_hash (each word folded, then the weighted sum mixed)."""
    c = (0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D, 0x27D4EB2F, 0x165667B1, 0xD3A2646D, 0xFD7046C5,
         0xB55A4F09)
    s = sum(kx_fold(x) * k for x, k in zip(list(la) + list(ra), c))
    s += kx_fold(ports) * 0x2545F491 + kx_fold(pw) * 0x9E3779B9
    return kx_mix(s & M)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    args = ap.parse_args()
    from onload_amd import pktgen
    from onload_amd.rx import GpuRxStack

    filters, socks = pktgen.world(args.config)
    g = GpuRxStack(device=0)
    g.load_world(filters, socks)
    lib = g._lib
    f = lib.oo_gpu_rx_debug_kx
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                  ctypes.POINTER(ctypes.c_uint32)]
    sizes = (ctypes.c_uint32 * 2)()
    probe4 = np.zeros(8, np.uint32)
    rc = f(g._ctx, probe4.ctypes.data, 0, probe4.ctypes.data, 0, sizes)
    assert rc == 0, rc
    nb4, ne6 = int(sizes[0]), int(sizes[1])
    k4 = np.zeros(2 * (nb4 + KX_PAD4) * 8, np.uint32)
    k6 = np.zeros((ne6 + KX_PAD6) * 16, np.uint32)
    assert f(g._ctx, k4.ctypes.data, k4.nbytes, k6.ctypes.data, k6.nbytes, sizes) == 0
    res = {"nb4": nb4, "ne6": ne6}
    # IPv4: two regions of buckets of two 16-B entries {la, ra, ports, val}
    for reg, name in ((0, "udp4"), (1, "tcp4")):
        e = k4[reg * (nb4 + KX_PAD4) * 8:(reg + 1) * (nb4 + KX_PAD4) * 8].reshape(-1, 2, 4)
        used = np.argwhere(e[:, :, 3] != 0)
        dist = collections.Counter()
        homes = collections.Counter()
        for b, j in used:
            la, ra, ports = int(e[b, j, 0]), int(e[b, j, 1]), int(e[b, j, 2])
            h = kx_hash((la, 0, 0, 0), (ra, 0, 0, 0), ports, 0) & (nb4 - 1)
            dist[int(b) - h] += 1
            homes[h] += 1
        res[name] = {"keys": int(len(used)), "dist_hist": dict(sorted(dist.items())[:8]),
                     "max_keys_per_home": max(homes.values()) if homes else 0,
                     "homes_with_2plus": sum(1 for v in homes.values() if v >= 2)}
    # IPv6: 64-B entries {la[4], ra[4], ports, pw, val, ...}
    e6 = k6.reshape(-1, 16)
    used = np.nonzero(e6[:, 10])[0]
    dist = collections.Counter()
    homes = collections.Counter()
    for i in used:
        r = e6[i]
        h = kx_hash(tuple(int(x) for x in r[0:4]), tuple(int(x) for x in r[4:8]), int(r[8]), int(r[9])) & (ne6 - 1)
        dist[int(i) - h] += 1
        homes[h] += 1
    res["ip6"] = {"keys": int(len(used)), "dist_hist": dict(sorted(dist.items())[:12]),
                  "max_keys_per_home": max(homes.values()) if homes else 0,
                  "homes_with_2plus": sum(1 for v in homes.values() if v >= 2)}
    print(json.dumps(res))
    g.close()


if __name__ == "__main__":
    main()
