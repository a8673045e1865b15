#!/bin/bash
# rocprofv3 kernel trace + stats of the driver-shaped config-2 bench command
# (--steps 20 --warmup 5) and of other configs: per-kernel average durations
# (win_kernel + body_kernel for the split transform) under gpurun_out/prof_c*.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-2}; do
  OUT="$ROOT/gpurun_out/prof_c$c"
  mkdir -p "$OUT"
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config "$c" --steps "${STEPS:-20}" --warmup "${WARMUP:-5}" \
     --no-cpu-baseline ${EXTRA:-} > "$OUT/bench.log" 2>&1)
  rc=$?
  echo "prof c$c rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/bench.log"; exit $rc; fi
  grep '^{' "$OUT/bench.log" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("c'$c'", r["kernel_ms"], r["frac"], d.get("steady"))'
  find "$OUT" -name '*kernel_stats.csv' -exec cat {} \; | head -12
done
