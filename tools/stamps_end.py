# SPDX-License-Identifier: BSD-2-Clause
"""How a launch ends, from the raw per-wave stamps of tools/stamps.py --raw.

    python tools/stamps_end.py gpurun_out/r03/r/stamps_c2_raw.npz

Slots per tile (oo_rx_kernel.hip STAMP): 0 tile start, 1 header windows
landed, 2 parse done, 3 demux done, 4 body streamed, 5 records stored,
6 the tile's first packet, 7 its body rounds.  Prints the end spread, the
time every wave would end at if the work were shared out evenly, when the
waves' last tiles started and how long they took, and the wave speeds.
"""
from __future__ import annotations

import json
import sys

import numpy as np


def main() -> None:
    z = np.load(sys.argv[1])
    a = z["stamps"].astype(np.int64)
    used = a[:, :, 0] != 0
    t0 = a[:, :, 0][used].min()
    us = (a[:, :, :6] - t0) * 10.0 / 1e3  # s_memrealtime: 100 MHz
    ntile = used.sum(1)
    live = ntile > 0
    w = np.nonzero(live)[0]
    last = ntile[w] - 1
    end = us[w, last, 5]
    start = us[w, 0, 0]
    busy = np.array([np.sum(us[i, :ntile[i], 5] - us[i, :ntile[i], 0]) for i in w])
    rounds = np.array([a[i, :ntile[i], 7].sum() for i in w])
    last_start = us[w, last, 0]
    last_rounds = a[w, last, 7]
    last_dur = end - last_start
    res = {
        "waves": int(len(w)),
        "end_us": {"max": round(float(end.max()), 1), "mean": round(float(end.mean()), 1),
                   "pct_0_10_25_50_75_90": [round(float(np.percentile(end, q)), 1) for q in (0, 10, 25, 50, 75, 90)]},
        # every wave busy until the same moment, the same total busy time
        "even_end_us": round(float(start.mean() + busy.mean()), 1),
        "last_tile": {
            "start_pct_0_25_50_75_100": [round(float(np.percentile(last_start, q)), 1) for q in (0, 25, 50, 75, 100)],
            "rounds_hist": {str(int(k)): int(v) for k, v in zip(*np.unique(last_rounds, return_counts=True))},
            "dur_us_by_rounds": {str(int(k)): round(float(last_dur[last_rounds == k].mean()), 2)
                                 for k in np.unique(last_rounds)},
            "header_us_mean": round(float((us[w, last, 3] - us[w, last, 0]).mean()), 2),
        },
        "tiles_per_wave": {str(int(k)): int(v) for k, v in zip(*np.unique(ntile[w], return_counts=True))},
        # body KiB per us of stream phase, per wave
        "wave_stream_GBps_pct_10_50_90": [round(float(np.percentile(
            rounds * 1.024 / np.maximum(np.array([np.sum(us[i, :ntile[i], 4] - us[i, :ntile[i], 3]) for i in w]), 1e-3),
            q)), 2) for q in (10, 50, 90)],
        "busy_us_pct_10_50_90": [round(float(np.percentile(busy, q)), 1) for q in (10, 50, 90)],
        "rounds_pct_10_50_90": [int(np.percentile(rounds, q)) for q in (10, 50, 90)],
    }
    # Which waves end last: their tile count and their last tile's size.
    late = end >= np.percentile(end, 95)
    res["latest_5pct"] = {"tiles": {str(int(k)): int(v) for k, v in zip(*np.unique(ntile[w][late], return_counts=True))},
                          "last_rounds_mean": round(float(last_rounds[late].mean()), 1),
                          "last_start_mean": round(float(last_start[late].mean()), 1)}
    early = end <= np.percentile(end, 5)
    res["earliest_5pct"] = {"tiles": {str(int(k)): int(v) for k, v in zip(*np.unique(ntile[w][early], return_counts=True))},
                            "last_rounds_mean": round(float(last_rounds[early].mean()), 1),
                            "rounds_total_mean": round(float(rounds[early].mean()), 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
