# SPDX-License-Identifier: BSD-2-Clause
"""Summarise rocprofv3 --pmc passes of bench.py into profiles/pmc_config<N>.json
(the file bench.py reads for roofline.traffic).

  python tools/pmc_summary.py --config 2 --dir gpurun_out/ev2/pmc_c2 [--out profiles/pmc_config2.json]

Each pass directory (fetch/, write/, sq/, tcc/) holds one rocprofv3 run with
--kernel-trace and its counters; values are averaged over each kernel's
launches and summed over the kernels one batch runs (--kernels, or the bench
line's roofline.kernels: rx_kernel, or win_kernel + body_kernel for the split
transform).  FETCH_SIZE is doubled: on gfx950 it counts a 128-B request as 64 B
(MI355X_MICROARCH.md, HBM/rocprofv3 section); WRITE_SIZE is taken as read.
Both are in KiB."""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counters(path: str, kernel: str = "rx_kernel") -> dict:
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    vals: dict = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if not r["Kernel_Name"].startswith(kernel + "("):
                continue
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            vals.setdefault(r["Counter_Name"], {}).setdefault(key[0], 0.0)
            vals[r["Counter_Name"]][key[0]] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in vals.items()}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--dir", required=True)
    ap.add_argument("--out")
    ap.add_argument("--bench-json", help="a bench.py line of the same configuration: "
                    "its roofline.achieved x kernel_ms gives the algorithmic bytes")
    ap.add_argument("--kernels", help="comma-separated kernel names (default: the bench "
                    "line's roofline.kernels, else oo_rx::rx_kernel)")
    a = ap.parse_args()
    from bench import DEFAULT_N  # noqa: E402
    bench = None
    if a.bench_json:
        line = [x for x in open(a.bench_json).read().splitlines() if x.startswith("{")][-1]
        bench = json.loads(line)
    kernels = (a.kernels.split(",") if a.kernels else
               (bench or {}).get("roofline", {}).get("kernels") or ["oo_rx::rx_kernel"])
    res = {"config": a.config, "packets_per_launch": DEFAULT_N[a.config],
           "kernel": " + ".join(kernels)}
    allc: dict = {}
    for p in sorted(os.listdir(a.dir)):
        d = os.path.join(a.dir, p)
        if not os.path.isdir(d):
            continue
        for k in kernels:
            for name, (v, n) in counters(d, k).items():
                tot, cnt = allc.get(name, (0.0, 0))
                allc[name] = (tot + v, max(cnt, n))
    for name, (v, n) in sorted(allc.items()):
        res[name] = v
        res[name + "_launches"] = n
    if "FETCH_SIZE" in allc and "WRITE_SIZE" in allc:
        rd = allc["FETCH_SIZE"][0] * 2 * 1024
        wr = allc["WRITE_SIZE"][0] * 1024
        alg = None
        if bench is not None:
            r = bench["roofline"]
            alg = r["achieved"] * r["kernel_ms"] * 1e6
        res.update({
            "correction": "FETCH_SIZE x2 (gfx950 counts 128-B requests as 64 B, MI355X_MICROARCH.md "
                          "HBM/rocprofv3 section); WRITE_SIZE as read; both KiB",
            "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
            "hbm_bytes_per_launch": int(rd + wr)})
        if alg:
            res.update({"algorithmic_bytes_per_launch": int(alg),
                        "traffic_over_algorithmic": round((rd + wr) / alg, 4)})
    if "SQ_WAIT_INST_ANY" in allc and "SQ_WAVE_CYCLES" in allc:
        res["wait_inst_frac"] = allc["SQ_WAIT_INST_ANY"][0] / max(1.0, allc["SQ_WAVE_CYCLES"][0])
    if "SQ_BUSY_CYCLES" in allc and "GRBM_GUI_ACTIVE" in allc:
        res["sq_busy_frac"] = allc["SQ_BUSY_CYCLES"][0] / max(1.0, allc["GRBM_GUI_ACTIVE"][0])
    if "TCC_HIT_sum" in allc and "TCC_MISS_sum" in allc:
        h, m = allc["TCC_HIT_sum"][0], allc["TCC_MISS_sum"][0]
        res["tcc_hit_rate"] = h / max(1.0, h + m)
    res["command"] = ("rocprofv3 --kernel-trace --pmc <one pass each: FETCH_SIZE | WRITE_SIZE | "
                      "SQ_* | TCC_*> -- python3 bench.py --config %d --steps 5 --warmup 1 "
                      "--no-cpu-baseline" % a.config)
    text = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
