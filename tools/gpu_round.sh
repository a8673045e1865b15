#!/bin/bash
# One GPU-box session: parity tests, a bench line, and a rocprofv3 kernel
# trace of the same bench command.  Stops at the first GPU fault / abort /
# timeout (exit codes other than 0 and 1).  Usage (from the repo root):
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh [tests|bench|prof|all]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
WHAT="${1:-all}"
STEPS="${STEPS:-20}"
CONFIG="${CONFIG:-2}"

stop_if_fault() {
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping after $what (rc=$rc)"
    exit "$rc"
  fi
}

if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/gpu_tests.log
  stop_if_fault $rc pytest
fi

if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  timeout -k 10 400 python bench.py --config "$CONFIG" --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-} \
    > gpurun_out/bench_c${CONFIG}.json 2> gpurun_out/bench_c${CONFIG}.err
  rc=$?
  cat gpurun_out/bench_c${CONFIG}.json
  tail -5 gpurun_out/bench_c${CONFIG}.err
  stop_if_fault $rc bench
fi

if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_c${CONFIG}" \
      -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$CONFIG" --steps "$STEPS" \
      --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/prof_c${CONFIG}.log" 2>&1)
  rc=$?
  tail -5 gpurun_out/prof_c${CONFIG}.log
  find gpurun_out/prof_c${CONFIG} -name "*stats*" | head
  stop_if_fault $rc rocprof
fi
echo done
