#!/bin/bash
# The round's GPU evidence under gpurun_out/ev2/, in phases (one gpurun call
# each; every GPU step under its own time limit, the script stops at the
# first failure):
#   A  the -m gpu suite, bench lines for configs 2-5 (config 2 with the CPU
#      baseline, the host-memory paths, TX fill and the AF_XDP ring paths),
#      and a rocprofv3 --kernel-trace --stats run of the config-2 bench;
#   B  PMC passes per configuration (CONFIGS, default 2 3 4 5): FETCH_SIZE,
#      WRITE_SIZE, an SQ pass and a TCC pass, each its own rocprofv3 run with
#      --kernel-trace only, summarised by tools/pmc_summary.py;
#   C  per-wave phase stamps (build/var_st.so, a -DOO_RX_STAMPS build).
#   gpurun --timeout 1200 -- bash tools/evidence_r02.sh A
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT=gpurun_out/ev2
mkdir -p "$OUT"
export TMPDIR=/tmp
PHASE="${1:-A}"
step() {  # name, then the command
  local name=$1; shift
  echo "== $name"
  "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}

if [ "$PHASE" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?
  tail -3 "$OUT/gpu_tests.log"
  [ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; exit $rc; }
  step bench2 timeout -k 10 300 sh -c "python bench.py --config 2 --steps 50 --warmup 5 --host-path --tx --xdp --xdp-host > $OUT/bench_config2.json 2> $OUT/bench_config2.err"
  cat "$OUT/bench_config2.json"
  for c in 3 4 5; do
    step bench$c timeout -k 10 300 sh -c "python bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 5 > $OUT/bench_config$c.json 2> $OUT/bench_config$c.err"
    cat "$OUT/bench_config$c.json"
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
     --output-format csv -- python3 "$ROOT/bench.py" --config 2 --steps 50 --warmup 5 \
     --no-cpu-baseline > "$ROOT/$OUT/prof.log" 2>&1) || { echo "rocprof failed"; tail -5 "$OUT/prof.log"; exit 1; }
  grep -h '^{' "$OUT/prof.log" | tail -1
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
fi

if [ "$PHASE" = B ]; then
  for c in ${CONFIGS:-2 3 4 5}; do
    d="$ROOT/$OUT/pmc_c$c"
    mkdir -p "$d"
    timeout -k 10 200 python bench.py --config "$c" --steps 5 --warmup 1 --no-cpu-baseline \
      > "$d/bench.json" 2> "$d/bench.err" || { echo "bench c$c failed"; exit 1; }
    for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" \
                "sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
                "tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
      set -- $pass
      name=$1; shift
      (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" -d "$d/$name" -o run \
         --output-format csv -- python3 "$ROOT/bench.py" --config "$c" --steps 5 --warmup 1 \
         --no-cpu-baseline > "$d/$name.log" 2>&1)
      rc=$?
      echo "c$c pass $name rc=$rc"
      if [ $rc -ne 0 ]; then tail -5 "$d/$name.log"; exit $rc; fi
    done
    python3 tools/pmc_summary.py --config "$c" --dir "$d" --bench-json "$d/bench.json" \
      --out "$d/pmc_config$c.json" | tail -30
  done
fi

if [ "$PHASE" = C ]; then
  for c in ${CONFIGS:-2 3 4 5}; do
    OO_RX_LIB=build/var_st.so timeout -k 10 200 python tools/stamps.py --config "$c" \
      > "$OUT/stamps_c$c.json" 2> "$OUT/stamps_c$c.err"
    rc=$?; echo "stamps c$c rc=$rc"; cat "$OUT/stamps_c$c.json"
    [ $rc -ne 0 ] && { tail -5 "$OUT/stamps_c$c.err"; exit $rc; }
  done
fi
echo done
