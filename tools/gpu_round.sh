#!/bin/bash
# One GPU-box session: parity tests, bench lines, and a rocprofv3 kernel
# trace of the config-2 bench command.  Stops at the first GPU fault / abort /
# timeout (exit codes other than 0 and 1).  Usage (from the repo root):
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh [tests|bench|prof|all]
#   CONFIGS="2 3" STEPS=20 ... bench configs (default 2)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
WHAT="${1:-all}"
STEPS="${STEPS:-20}"
CONFIGS="${CONFIGS:-2}"

stop_if_fault() {
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping after $what (rc=$rc)"
    exit "$rc"
  fi
}

if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/gpu_tests.log
  stop_if_fault $rc pytest
  [ $rc -ne 0 ] && exit $rc
fi

if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  for c in $CONFIGS; do
    timeout -k 10 300 python bench.py --config "$c" --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-} \
      > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err
    rc=$?
    cat gpurun_out/bench_c$c.json
    tail -3 gpurun_out/bench_c$c.err
    stop_if_fault $rc "bench c$c"
    [ $rc -ne 0 ] && exit $rc
  done
fi

if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  export TMPDIR=/tmp
  c=${PROF_CONFIG:-2}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_c$c" \
      -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$c" --steps "$STEPS" \
      --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_c$c.log" 2>&1)
  rc=$?
  tail -3 gpurun_out/prof_c$c.log
  find gpurun_out/prof_c$c -name "*kernel_stats*" -exec cat {} \;
  stop_if_fault $rc rocprof
fi
echo done
