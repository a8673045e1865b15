#!/bin/bash
# Bench sweep over launch knobs (env vars read by oo_gpu_rx_open):
#   SWEEP="OO_RX_GRID_PCT=100 OO_RX_GRID_PCT=50" CONFIG=2 bash tools/sweep.sh
# Each item is a space-free ';'-joined list of VAR=VALUE settings.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
CONFIG="${CONFIG:-2}"
for item in ${SWEEP:-OO_RX_GRID_PCT=100}; do
  envs=$(echo "$item" | tr ';' ' ')
  out=$(env $envs timeout -k 10 300 python bench.py --config "$CONFIG" --steps "${STEPS:-20}" \
        --warmup 3 --no-cpu-baseline 2> gpurun_out/sweep_last.err)
  rc=$?
  if [ $rc -ne 0 ]; then echo "$item rc=$rc"; tail -5 gpurun_out/sweep_last.err; exit $rc; fi
  echo "$item $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"
done
