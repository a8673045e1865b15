#!/bin/bash
# Round-3 GPU experiments, one phase per gpurun call.  Every GPU step runs
# under its own time limit; the script stops at the first failure.
#   gpurun --timeout 1200 -- bash tools/exp_r03.sh <phase>
# Output under gpurun_out/r03/<phase>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
PHASE="${1:-a}"
OUT=gpurun_out/r03/$PHASE
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # name, limit (s), command...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc" >&2; exit $rc; fi
}

tests() {  # a test failure (rc 1) is reported; a fault, abort or timeout stops the script
  echo "== tests $(date +%T)"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > "$OUT/gpu_tests.log" 2>&1
  local rc=$?
  tail -3 "$OUT/gpu_tests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
}

# bench line summary: kernel ms, frac, value
ab() {  # reps, configs, libs...
  local reps=$1 configs=$2; shift 2
  for rep in $(seq 1 "$reps"); do
    for c in $configs; do
      for spec in "$@"; do
        lib=${spec%%@*}; envs=""
        [ "$spec" != "$lib" ] && envs=$(echo "${spec#*@}" | tr ',' ' ')
        env $envs OO_RX_LIB="$lib" timeout -k 10 300 python bench.py --config "$c" \
          --steps "${STEPS:-30}" --warmup 5 --no-cpu-baseline ${EXTRA:-} \
          > "$OUT/ab_last.json" 2> "$OUT/ab_last.err"
        rc=$?
        if [ $rc -ne 0 ]; then echo "$spec c$c rc=$rc"; tail -5 "$OUT/ab_last.err"; exit $rc; fi
        echo "rep$rep c$c $spec $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(r["kernel_ms"], r["frac"], d["value"])' "$OUT/ab_last.json")" | tee -a "$OUT/ab.log"
      done
    done
  done
}

case "$PHASE" in
a)  # baseline of the round: tests, store ablations, stamps, batch-size sweep
  tests
  ab 3 2 onload_amd/liboo_gpu_rx.so build/var_nost.so build/var_hot.so
  step stamps 300 env OO_RX_LIB=build/var_st.so python tools/stamps.py --config 2 > "$OUT/stamps_c2.json" 2> "$OUT/stamps.err"
  cat "$OUT/stamps_c2.json"
  for n in 524288 1048576 2097152; do
    step n$n 300 python bench.py --config 2 --n $n --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/n$n.json" 2>/dev/null
    python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[1], r["kernel_ms"], r["frac"])' "$OUT/n$n.json"
  done
  step counters 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
  grep -i -E "utcl|tlb|translation" "$OUT/counters.txt" | head -40
  ;;
*)
  echo "unknown phase $PHASE"; exit 2 ;;
esac
echo "done $(date +%T)"
