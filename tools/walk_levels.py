# SPDX-License-Identifier: BSD-2-Clause
"""Filter-table walk lengths of a configuration's packets (diagnostic, CPU).

For every packet that reaches the lookups (the oracle's records say which),
replays the kernel's walks over the oracle's tables: per lookup stage, the
occupied slots visited before the walk ends (an EMPTY slot, a full cycle, or
-- TCP -- the deciding match).  Per 64-packet wave it prints the sum over
stages of the wave's longest walk (what stage-by-stage walks cost in
dependent loads) and the longest per-packet total (what the per-lane state
machine, lookup_fsm, costs).

    python tools/walk_levels.py --config 5 --n 65536
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--n", type=int, default=65536)
    args = ap.parse_args()
    from onload_amd import pktgen
    from oracle_lib import OracleStack  # the checker (test infrastructure)

    filters, socks = pktgen.world(args.config)
    o = OracleStack()
    o.load_world(filters, socks)
    buf, desc = pktgen.generate(args.config, args.n)
    rec = o.handle_rx_batch(buf, desc, nthreads=4)
    lib = o._lib
    lib.oo_or_hash1.restype = lib.oo_or_hash2.restype = ctypes.c_uint32
    lib.oo_or_hash1.argtypes = [ctypes.c_uint32] * 6
    lib.oo_or_hash2.argtypes = [ctypes.c_uint32] * 5
    masks = {4: (1 << 16) - 1, 6: (1 << 14) - 1}
    cache: dict = {}

    def slot(af, i):
        if (af, i) not in cache:
            st = o.table_slot(af, i)[0]
            empty = (st & 0xc0000000) == 0x80000000 if af == 4 else st == 0xfffffffe
            ident = st & 0x3fffffff if af == 4 else st
            cache[(af, i)] = (empty, ident)
        return cache[(af, i)]

    def visits(af, key, stop_sock):
        mask = masks[af]
        h1 = lib.oo_or_hash1(mask, *key)
        h2 = lib.oo_or_hash2(*key)
        first, n = h1, 0
        for _ in range(mask + 1):
            empty, ident = slot(af, h1)
            if empty:
                break
            n += 1
            if stop_sock is not None and ident == stop_sock:
                break
            h1 = (h1 + h2) & mask
            if h1 == first:
                break
        return n

    per = np.zeros((len(rec), 3), dtype=np.int32)
    for i in np.nonzero((rec["reason"] == 0) | (rec["reason"] == 1))[0]:
        r = rec[i]
        af = 6 if r["l4_off"] == 54 else 4  # the generator's IPv6 frames: L4 at 54
        pr = int(r["proto"])
        dx, sx = int(r["daddr_be"]), int(r["saddr_be"])
        dp, sp = int(r["dport_be"]), int(r["sport_be"])
        keys = [(dx, dp, sx, sp, pr), (dx, dp, 0, 0, pr), (0, dp, 0, 0, pr)]
        for s in range(3 if pr == 6 else 2):
            dec = r["reason"] == 0 and r["stage"] == s + 1
            per[i, s] = visits(af, keys[s], int(r["sock"]) if (pr == 6 and dec) else None)
            if dec:
                break
    nw = len(rec) // 64
    P = per[: nw * 64].reshape(nw, 64, 3)
    print({"config": args.config, "packets": args.n,
           "mean_visits_per_stage": [round(float(x), 3) for x in per.mean(0)],
           "wave_max_per_stage": [round(float(x), 3) for x in P.max(1).mean(0)],
           "sum_of_stage_maxima": round(float(P.max(1).sum(1).mean()), 3),
           "max_of_lane_totals": round(float(P.sum(2).max(1).mean()), 3)})


if __name__ == "__main__":
    main()
