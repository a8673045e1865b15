# SPDX-License-Identifier: BSD-2-Clause
"""Debug helper: run one config sample through the GPU library twice and
against the oracle; print which tiles/lanes differ (pattern + determinism)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from gpu_util import run_dev  # noqa: E402
from onload_amd import pktgen  # noqa: E402
from onload_amd.rx import GpuRxStack  # noqa: E402
from oracle_lib import OracleStack  # noqa: E402

config = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
filters, socks = pktgen.world(config)
g = GpuRxStack(device=0)
o = OracleStack()
g.load_world(filters, socks)
o.load_world(filters, socks)
buf, desc = pktgen.generate(config, n, first=12345 * config)
want = o.handle_rx_batch(buf, desc, nthreads=16)
for rep in range(2):
    got, _ = run_dev(g, buf, desc)
    A = got.view(np.uint8).reshape(-1, 32)
    B = want.view(np.uint8).reshape(-1, 32)
    bad = np.nonzero((A != B).any(1))[0]
    tiles = np.unique(bad // 64)
    print(f"rep {rep}: {len(bad)} bad; tiles {tiles[:20].tolist()} ({len(tiles)} tiles)")
    for t in tiles[:4]:
        lanes = (bad[bad // 64 == t] % 64).tolist()
        print(f"  tile {t}: lanes {lanes}")
    if len(bad):
        i = bad[0]
        print("  gpu", got[i], "\n  ora", want[i])
