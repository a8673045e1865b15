#!/bin/bash
# SQ instruction-mix passes (one --pmc pass each, --kernel-trace only) of the
# bench on CONFIGS under each OO_RX_KERNEL path in PATHS; per-dispatch rows
# under gpurun_out/sq_c<config>_p<path>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-3}; do
  for p in ${PATHS:-2 3}; do
    OUT="$ROOT/gpurun_out/sq_c${c}_p${p}"
    mkdir -p "$OUT"
    (cd /tmp && OO_RX_KERNEL=$p timeout -s KILL 120 rocprofv3 --kernel-trace --pmc \
       ${COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY} \
       -d "$OUT" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$c" --steps 3 \
       --warmup 1 --steady 0 --no-cpu-baseline > "$OUT/bench.log" 2>&1)
    rc=$?
    echo "sq c$c p$p rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/bench.log"; exit $rc; fi
  done
done
