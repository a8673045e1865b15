# SPDX-License-Identifier: BSD-2-Clause
"""GPU diagnosis of a record mismatch: config samples through the default
(split) path and the single-kernel path, with jumbo frames kept or left out,
each against the oracle; prints per-case mismatch counts and the first
records that differ.  Usage: python tools/r04_diag.py [config n ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from gpu_util import run_dev  # noqa: E402
from onload_amd import _abi, pktgen  # noqa: E402
from onload_amd.rx import GpuRxStack  # noqa: E402
from oracle_lib import OracleStack  # noqa: E402


def report(tag, got, want, desc, limit=6):
    A = got.view(np.uint8).reshape(-1, 32)
    B = want.view(np.uint8).reshape(-1, 32)
    bad = np.nonzero((A != B).any(1))[0]
    print(f"{tag}: {len(bad)} of {len(got)} differ", flush=True)
    if len(bad):
        cols = np.nonzero((A[bad] != B[bad]).any(0))[0]
        print(f"  differing byte columns: {cols.tolist()}")
        print(f"  lens of bad: min {desc['len'][bad].min()} max {desc['len'][bad].max()};"
              f" tiles {sorted(set((bad // 64).tolist()))[:12]}")
        for i in bad[:limit]:
            print(f"  [{i}] len={desc[i]['len']} off={desc[i]['frame_off']}\n    gpu={got[i]}\n    ora={want[i]}")


def main():
    args = [int(a) for a in sys.argv[1:]] or [4, 12000, 4, 1 << 14, 5, 40000]
    for config, n in zip(args[::2], args[1::2]):
        filters, socks = pktgen.world(config)
        buf, desc = pktgen.generate(config, n)
        o = OracleStack()
        o.load_world(filters, socks)
        for label, d in (("all", desc), ("le1514", desc[desc["len"] <= 1514]),
                         ("jumbo", desc[desc["len"] > 1514])):
            if len(d) == 0:
                continue
            want = o.handle_rx_batch(buf, d, nthreads=8)
            for path in (0, 1):
                g = GpuRxStack(device=0)
                g.load_world(filters, socks)
                if path:
                    t = _abi.Tuning()
                    t.gshift = -1
                    t.path = path
                    g.set_tuning(t)
                got, ctr = run_dev(g, buf, d)
                report(f"config {config} n={len(d)} {label} path={path}", got, want, d)
                g.close()


if __name__ == "__main__":
    main()
