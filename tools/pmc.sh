#!/bin/bash
# PMC passes for the RX kernel on one bench configuration (MI355X_MICROARCH.md
# "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE in separate passes, SQ
# counters in their own pass; --kernel-trace only, never with sys/runtime
# traces).  Writes gpurun_out/pmc_c$CONFIG/<pass>/... and the HBM ceiling
# microbenchmark output.  Usage: gpurun -- bash tools/pmc.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
CONFIG="${CONFIG:-2}"
STEPS="${STEPS:-10}"
OUT="$ROOT/gpurun_out/pmc_c${CONFIG}"
mkdir -p "$OUT"
export TMPDIR=/tmp

if [ -x tools/hbm_ceiling ] && [ "${CEILING:-1}" = 1 ]; then
  timeout -k 10 120 tools/hbm_ceiling > gpurun_out/hbm_ceiling.json 2>&1
  rc=$?; echo "ceiling rc=$rc"; cat gpurun_out/hbm_ceiling.json
  if [ $rc -ne 0 ]; then exit $rc; fi
fi

run_pass() {
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run \
     --output-format csv -- python3 "$ROOT/bench.py" --config "$CONFIG" --steps "$STEPS" \
     --warmup 2 --no-cpu-baseline > "$OUT/$name.log" 2>&1)
  local rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}

run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
run_pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
echo done
