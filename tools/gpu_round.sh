#!/bin/bash
# One GPU-box driver for a round's measurements (run through gpurun from the
# repo root).  Steps, in the order given in STEPS (default "tests bench"):
#   tests     the -m gpu suite (TESTS files, TESTS_K -k filter; HIP_LOG sets
#             AMD_LOG_LEVEL, default 1: HIP's errors) -> gpu_tests.log
#   smoke     __graft_entry__.smoke()
#   bench     the driver-shaped bench line (--steps 20 --warmup 5) per config in
#             CONFIGS (config 2 with its cpu_baseline) -> bench_c<N>.json
#   group     config-5 bench through a joined group of one rank (--group)
#   prof      rocprofv3 --kernel-trace --stats of that command -> prof_c<N>/
#   hbm       FETCH_SIZE and WRITE_SIZE passes, one run each -> pmc_c<N>/
#   sq        SQ instruction-mix pass (COUNTERS overrides) -> sq_c<N>/
#   ta        texture-path pass (TA/TD/TCP) -> ta_c<N>/
#   ab        same-box A/B of LIBS entries (tools/ab.sh) -> ab.log
#   poll      tools/poll_bench per poll size (EPP) -> poll.jsonl
#   stamps    the OO_RX_STAMPS build on STAMP_CONFIG via tools/stamps.py
# Every GPU step runs under its own time limit; the first failure ends the
# call (no retries).  Output under gpurun_out/$TAG (default "round").
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${TAG:-round}"
mkdir -p "$OUT"
CONFIGS="${CONFIGS:-2 3 4 5}"

fail() { echo "step $1 failed (rc=$2)"; [ -f "$3" ] && tail -20 "$3"; exit "$2"; }

summ() {  # one line per bench JSON
  python3 -c 'import json,sys
d=json.load(open(sys.argv[1])); r=d["roofline"]
print(sys.argv[1].split("/")[-1], d["value"], r["kernel_ms"], r["frac"], r.get("kernels"),
      (d.get("steady") or {}).get("frac"), d.get("path"), (d.get("cpu_baseline") or {}).get("value"))' "$1"
}

for step in ${STEPS:-tests bench}; do
  case $step in
    tests)
      AMD_LOG_LEVEL=${HIP_LOG:-1} timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 \
        --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > "$OUT/gpu_tests.log" 2>&1 \
        || fail tests $? "$OUT/gpu_tests.log"
      tail -2 "$OUT/gpu_tests.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || fail smoke $? "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      for c in $CONFIGS; do
        extra="--no-cpu-baseline"; [ "$c" = 2 ] && extra=""
        timeout -k 10 300 python bench.py --config "$c" --steps 20 --warmup 5 $extra ${EXTRA:-} \
          > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || fail "bench c$c" $? "$OUT/bench_c$c.err"
        summ "$OUT/bench_c$c.json"
      done ;;
    group)
      timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline --group \
        > "$OUT/bench_group_c5.json" 2> "$OUT/bench_group_c5.err" || fail group $? "$OUT/bench_group_c5.err"
      summ "$OUT/bench_group_c5.json"
      python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d.get("table_broadcast"), d.get("record_gather"))' \
        "$OUT/bench_group_c5.json" ;;
    prof)
      for c in $CONFIGS; do
        mkdir -p "$OUT/prof_c$c"
        (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run \
           --output-format csv -- python3 "$ROOT/bench.py" --config "$c" --steps 20 --warmup 5 --steady 0 \
           --no-cpu-baseline ${EXTRA:-} > "$OUT/prof_c$c/bench.log" 2>&1) || fail "prof c$c" $? "$OUT/prof_c$c/bench.log"
        find "$OUT/prof_c$c" -name '*kernel_stats.csv' -exec head -4 {} \;
      done ;;
    hbm)
      for c in $CONFIGS; do
        for pass in FETCH_SIZE WRITE_SIZE; do
          mkdir -p "$OUT/pmc_c$c/$pass"
          (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $pass -d "$OUT/pmc_c$c/$pass" -o run \
             --output-format csv -- python3 "$ROOT/bench.py" --config "$c" --steps 5 --warmup 1 --steady 0 \
             --no-cpu-baseline ${EXTRA:-} > "$OUT/pmc_c$c/$pass.log" 2>&1) || fail "hbm c$c $pass" $? "$OUT/pmc_c$c/$pass.log"
        done
        echo "hbm c$c done"
      done ;;
    sq|ta)
      if [ "$step" = sq ]; then
        ctr="${COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY}"
      else
        ctr="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
      fi
      for c in $CONFIGS; do
        mkdir -p "$OUT/${step}_c$c"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/${step}_c$c" -o run \
           --output-format csv -- python3 "$ROOT/bench.py" --config "$c" --steps 3 --warmup 1 --steady 0 \
           --no-cpu-baseline ${EXTRA:-} > "$OUT/${step}_c$c/bench.log" 2>&1) || fail "$step c$c" $? "$OUT/${step}_c$c/bench.log"
        echo "$step c$c done"
      done ;;
    ab)
      REPS=${REPS:-1} CONFIGS="$CONFIGS" STEPS=20 LIBS="${LIBS:-onload_amd/liboo_gpu_rx.so}" \
        bash tools/ab.sh > "$OUT/ab.log" 2>&1 || fail ab $? "$OUT/ab.log"
      cat "$OUT/ab.log" ;;
    poll)
      : > "$OUT/poll.jsonl"
      for c in ${POLL_CONFIGS:-2 3}; do
        timeout -k 10 300 tools/poll_bench "$c" ${FRAMES:-262144} ${EPP:-16 64 1024 65536} >> "$OUT/poll.jsonl" \
          2> "$OUT/poll.err" || fail "poll c$c" $? "$OUT/poll.err"
      done
      python3 -c 'import json
for l in open("'"$OUT"'/poll.jsonl"):
    d = json.loads(l)
    print({k: d.get(k) for k in ("config", "evs_per_poll", "mode", "poll_us_median", "mpps", "cpu_poll_us_equiv", "handed_back", "fit")})' ;;
    stamps)
      OO_RX_LIB="${OO_RX_LIB:-build/var_st.so}" timeout -k 10 300 python tools/stamps.py --config ${STAMP_CONFIG:-3} \
        > "$OUT/stamps.txt" 2> "$OUT/stamps.err" \
        || fail stamps $? "$OUT/stamps.err"
      tail -c 600 "$OUT/stamps.txt"; echo ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
