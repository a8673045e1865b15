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
        echo "rep$rep c$c $spec $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(r["kernel_ms"], r["frac"], d["value"], "steady", (d.get("steady") or {}).get("kernel_ms"))' "$OUT/ab_last.json")" | tee -a "$OUT/ab.log"
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
b)  # tests, driver-shaped bench lines, kernel trace, TLB counters at 2^20 / 2^21
  tests
  for r in 1 2; do
    step bench$r 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench$r.json" 2> "$OUT/bench$r.err"
    cat "$OUT/bench$r.json"
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
     --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline \
     > "$ROOT/$OUT/prof.log" 2>&1) || { echo "rocprof failed"; tail -5 "$OUT/prof.log"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
  for n in 1048576 2097152; do
    for pass in "tlb1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
                "tlb2 TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
      set -- $pass; name=$1; shift
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$ROOT/$OUT/${name}_$n" \
         -o run --output-format csv -- python3 "$ROOT/bench.py" --n $n --steps 5 --warmup 1 \
         --no-cpu-baseline > "$ROOT/$OUT/${name}_$n.log" 2>&1) || { echo "pmc $name $n failed"; tail -3 "$OUT/${name}_$n.log"; exit 1; }
    done
  done
  python3 -c "import sys, glob, os; sys.path.insert(0, 'tools'); from pmc_summary import counters; [print(d, counters(d)) for d in sorted(glob.glob('$OUT/tlb*_*')) if os.path.isdir(d)]" > "$OUT/tlb_summary.txt" 2>&1
  cat "$OUT/tlb_summary.txt"
  ;;
c)  # steps / profiler sensitivity of the config-2 line; table maintenance timing
  TESTS_K="table or poll or stream or l4" tests
  for spec in "20 a" "50 a" "200 a" "20 b" "50 b"; do
    set -- $spec
    step s$1$2 300 python bench.py --steps $1 --warmup 5 --no-cpu-baseline > "$OUT/s$1$2.json" 2>/dev/null
    echo "steps $1 ($2): $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(r["kernel_ms"], d["ms_per_step"], r["frac"])' "$OUT/s$1$2.json")"
  done
  for st in 20 50; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof$st" -o run \
       --output-format csv -- python3 "$ROOT/bench.py" --steps $st --warmup 5 --no-cpu-baseline \
       > "$ROOT/$OUT/prof$st.log" 2>&1) || { echo "rocprof failed"; tail -5 "$OUT/prof$st.log"; exit 1; }
    echo "rocprof steps $st: $(grep -o '"kernel_ms": [0-9.]*' "$OUT/prof$st.log")"
  done
  step tableops 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --table-ops > "$OUT/tableops.json" 2> "$OUT/tableops.err"
  grep -o '"table_ops": {[^}]*}' "$OUT/tableops.json"
  for kv in "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
    step kernarg 300 env $kv python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/ka.json" 2>/dev/null
    echo "$kv: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(r["kernel_ms"], d["ms_per_step"], r["frac"])' "$OUT/ka.json")"
  done
  step poll 300 tools/poll_bench 2 262144 64 1024 65536 > "$OUT/poll_c2.jsonl" 2> "$OUT/poll.err"
  cat "$OUT/poll_c2.jsonl"
  step poll3 300 tools/poll_bench 3 262144 64 1024 65536 > "$OUT/poll_c3.jsonl" 2>> "$OUT/poll.err"
  cat "$OUT/poll_c3.jsonl"
  ;;
d)  # claim sets alternating per launch (no end-of-launch reset) vs HEAD; I-cache and VMEM level counters
  TESTS_K="table or stream or claim or parity or wait_variants or dist" tests
  ab 3 "2 3" onload_amd/liboo_gpu_rx.so build/var_ref.so
  for pass in "ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
              "lv SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"; do
    set -- $pass; name=$1; shift
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$ROOT/$OUT/$name" \
       -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 \
       --no-cpu-baseline > "$ROOT/$OUT/$name.log" 2>&1) || { echo "pmc $name failed"; tail -3 "$OUT/$name.log"; exit 1; }
  done
  python3 -c "import sys, glob, os; sys.path.insert(0, 'tools'); from pmc_summary import counters; [print(d, counters(d)) for d in sorted(glob.glob('$OUT/*')) if os.path.isdir(d)]" > "$OUT/pmc_summary.txt" 2>&1
  cat "$OUT/pmc_summary.txt"
  ;;
e)  # deep turns through the header rows: parity of the check builds, then depth A/B
  TESTS_K="wait_variants or gpu_parity or l4_ref" tests
  ab 3 "2 4" onload_amd/liboo_gpu_rx.so build/var_d8.so build/var_d16.so build/var_d32.so
  ab 1 "3 5" onload_amd/liboo_gpu_rx.so build/var_d8.so build/var_d16.so
  ;;
f)  # fewer bytes in flight: smaller grids, fewer extra rounds (config 2)
  L=onload_amd/liboo_gpu_rx.so
  ab 3 2 $L $L@OO_RX_GRID_PCT=80 $L@OO_RX_GRID_PCT=90 $L@OO_RX_GRID_PCT=60 build/var_e4.so build/var_e6.so
  ;;
g)  # AF_XDP ring path in the 2048-B UMEM layout for the short-frame configs, with and without the length hint
  for c in 3 5 2; do
    step xdp$c 600 python bench.py --config $c --xdp --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/xdp_c$c.json" 2> "$OUT/xdp_c$c.err"
    python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print("c", sys.argv[2], "packed", r["kernel_ms"], r["frac"], "xdp", json.dumps(d["xdp_ring"]))' "$OUT/xdp_c$c.json" $c
  done
  ;;
h)  # the launch's end in the stamps (config 2); HBM bytes of config 3 on the AF_XDP ring path
  step stamps 300 env OO_RX_LIB=build/var_st.so python tools/stamps.py --config 2 > "$OUT/stamps_c2.json" 2> "$OUT/stamps.err"
  cat "$OUT/stamps_c2.json"
  for pass in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
    set -- $pass; name=$1; shift
    (cd /tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc "$@" -d "$ROOT/$OUT/xdp3_$name" \
       -o run --output-format csv -- python3 "$ROOT/bench.py" --config 3 --xdp --steps 5 --warmup 1 \
       --no-cpu-baseline > "$ROOT/$OUT/xdp3_$name.log" 2>&1) || { echo "pmc $name failed"; tail -3 "$OUT/xdp3_$name.log"; exit 1; }
  done
  ;;
i)  # deep turns for each wave's last tile (product) vs none (dl0)
  TESTS_K="wait_variants or gpu_parity or l4_ref or tx or xdp" tests
  ab 3 2 onload_amd/liboo_gpu_rx.so build/var_dl0.so
  ab 1 "3 4 5" onload_amd/liboo_gpu_rx.so build/var_dl0.so
  ;;
j)  # deep-last on config 2 with more reps; deep-all + deep-last on config 4
  ab 5 2 onload_amd/liboo_gpu_rx.so build/var_dl0.so
  ab 2 4 onload_amd/liboo_gpu_rx.so build/var_d8dl.so build/var_d32dl.so build/var_dl0.so
  ;;
k)  # deep turns only for tiles longer than a threshold (config 4's jumbo tiles)
  ab 3 4 onload_amd/liboo_gpu_rx.so build/var_t100.so build/var_t200.so build/var_t400.so build/var_d8dl.so
  ab 2 2 onload_amd/liboo_gpu_rx.so build/var_t100.so build/var_t200.so
  ab 1 5 onload_amd/liboo_gpu_rx.so build/var_t100.so build/var_t200.so
  ;;
l)  # a wave's last long tile through one R + E-row ring (product) vs not (w0)
  TESTS_K="wait_variants or gpu_parity or l4_ref or tx or xdp or table" tests
  ab 5 2 onload_amd/liboo_gpu_rx.so build/var_w0.so
  ab 1 "3 4 5" onload_amd/liboo_gpu_rx.so build/var_w0.so
  ;;
m)  # config 2: claim groups spanning XCDs (runs of 2^gshift waves = 2^(gshift-1) blocks)
  L=onload_amd/liboo_gpu_rx.so
  ab 3 2 $L $L@OO_RX_GSHIFT=2 $L@OO_RX_GSHIFT=3 $L@OO_RX_GSHIFT=4 $L@OO_RX_GSHIFT=4,OO_RX_GROUPS=32
  ;;
n)  # bench lines and PMC passes (FETCH/WRITE/SQ/TCC) of configs 2-5 on the current kernel
  for c in ${CONFIGS:-2 3 4 5}; do
    step bench$c 300 python bench.py --config $c --steps 20 --warmup 5 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
    python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[1], r["kernel_ms"], r["frac"], d["value"])' "$OUT/bench_c$c.json"
    CONFIG=$c CEILING=0 STEPS=5 bash tools/pmc.sh > "$OUT/pmc_c$c.log" 2>&1 || { echo "pmc c$c failed"; tail -5 "$OUT/pmc_c$c.log"; exit 1; }
  done
  ;;
o)  # split tail tiles (last part to finish combines) vs whole tail tiles (OO_RX_SPLIT=0) vs HEAD
  tests
  L=onload_amd/liboo_gpu_rx.so
  ab 5 2 $L $L@OO_RX_SPLIT=0 build/var_ref.so
  ab 2 4 $L $L@OO_RX_SPLIT=0 build/var_ref.so
  ab 1 "3 5" $L build/var_ref.so
  ;;
p)  # HEAD check after the restart; write-cost and half-line (sector) probes
  tests
  for r in 1 2; do
    step bench$r 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench$r.json" 2> "$OUT/bench$r.err"
    cat "$OUT/bench$r.json"
  done
  step probe 600 tools/ring_probe 1610612736 w > "$OUT/wr_probe.jsonl" 2> "$OUT/wr_probe.err"
  [ -n "${PROBE_ONLY:-}" ] && { cat "$OUT/wr_probe.jsonl"; }
  cat "$OUT/wr_probe.jsonl"
  step counters 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
  grep -o -E "TCC_EA0?_RDREQ[A-Z0-9_]*|TCC_BUBBLE[A-Z0-9_]*|TCC_EA0?_WRREQ[A-Z0-9_]*" "$OUT/counters.txt" | sort -u | tr '\n' ' '; echo
  for v in h0 h1; do
    for pass in "fetch FETCH_SIZE" "rq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
      set -- $pass; name=$1; shift
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$ROOT/$OUT/${v}_$name" \
         -o run --output-format csv -- "$ROOT/tools/ring_probe" 1610612736 $v \
         > "$ROOT/$OUT/${v}_$name.log" 2>&1) || { echo "pmc $v $name failed"; tail -3 "$OUT/${v}_$name.log"; }
    done
  done
  python3 -c "import sys, glob, os; sys.path.insert(0, 'tools'); from pmc_summary import counters; [print(d, counters(d, 'ring_split')) for d in sorted(glob.glob('$OUT/h*_*')) if os.path.isdir(d)]" > "$OUT/sector_summary.txt" 2>&1
  cat "$OUT/sector_summary.txt"
  # per-launch clock: GRBM_GUI_ACTIVE cycles per dispatch over 50 launches
  (cd /tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$ROOT/$OUT/clk" \
     -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline \
     > "$ROOT/$OUT/clk.log" 2>&1) || { echo "pmc clk failed"; tail -3 "$OUT/clk.log"; }
  ;;
q)  # write cost by read/store cache policy; half-line reads (HBM request size)
  step probe 600 tools/ring_probe 1610612736 w > "$OUT/wr_probe.jsonl" 2> "$OUT/wr_probe.err"
  cat "$OUT/wr_probe.jsonl"
  [ -n "${SECTOR:-}" ] || { echo "done $(date +%T)"; exit 0; }
  for v in h0 h1; do
    for pass in "fetch FETCH_SIZE" "rq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
      set -- $pass; name=$1; shift
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$ROOT/$OUT/${v}_$name" \
         -o run --output-format csv -- "$ROOT/tools/ring_probe" 1610612736 $v \
         > "$ROOT/$OUT/${v}_$name.log" 2>&1) || { echo "pmc $v $name failed"; tail -3 "$OUT/${v}_$name.log"; exit 1; }
      grep -h '"tag"' "$OUT/${v}_$name.log" || true
    done
  done
  python3 -c "import sys, glob, os; sys.path.insert(0, 'tools'); from pmc_summary import counters; [print(d, counters(d, 'ring_split')) for d in sorted(glob.glob('$OUT/h*_*')) if os.path.isdir(d)]" > "$OUT/sector_summary.txt" 2>&1
  cat "$OUT/sector_summary.txt"
  ;;
r)  # raw per-wave stamps of config 2 (the launch's end); kernel arguments in device memory or not
  step stamps 300 env OO_RX_LIB=build/var_st.so python tools/stamps.py --config 2 --raw "$OUT/stamps_c2_raw.npz" > "$OUT/stamps_c2.json" 2> "$OUT/stamps.err"
  cat "$OUT/stamps_c2.json"
  L=onload_amd/liboo_gpu_rx.so
  ab 3 2 $L $L@HIP_FORCE_DEV_KERNARG=0
  ;;
s)  # per-tile hwport byte + branch-free slot compares vs HEAD: full GPU suite, then A/B
  tests
  ab 2 "2 3 5" onload_amd/liboo_gpu_rx.so build/var_ref.so
  ab 1 4 onload_amd/liboo_gpu_rx.so build/var_ref.so
  ;;
t)  # 8 waves per CU (the check builds: ring 6 / 8, LDS allows 4 blocks per CU) vs the product
  ab 3 2 onload_amd/liboo_gpu_rx.so build/check/liboo_gpu_rx_r8e2.so build/check/liboo_gpu_rx_r6e4.so
  ;;
u)  # per-group job sequences (OO_RX_GSEQ): parity of the variant, then A/B
  for v in gseq; do
    OO_RX_LIB=build/var_$v.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py \
      tests/test_gpu_tx.py tests/test_gpu_l4_ref.py tests/test_gpu_xdp.py -x -q -p no:cacheprovider \
      --timeout 300 --timeout-method thread > "$OUT/${v}_parity.log" 2>&1
    rc=$?; echo "$v parity:"; tail -2 "$OUT/${v}_parity.log"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
  ab 4 2 onload_amd/liboo_gpu_rx.so build/var_gseq.so
  ab 2 "4 5" onload_amd/liboo_gpu_rx.so build/var_gseq.so
  ;;
v)  # smoke(); the N>1 bench flow rehearsed on one GPU (two ranks sharing it over gloo)
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step rehearsal 600 env OO_BENCH_SHARE_GPU=1 OO_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 10 --warmup 3 \
    --steady 20 > "$OUT/rehearsal_2ranks.json" 2> "$OUT/rehearsal_2ranks.err"
  cat "$OUT/rehearsal_2ranks.json"
  ;;
w)  # the tile iteration as a template: lockstep only (d0) and per tile (d2) vs HEAD (ref)
  for v in d0 d2; do
    OO_RX_LIB=build/var_$v.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py \
      tests/test_gpu_tx.py tests/test_gpu_l4_ref.py tests/test_gpu_xdp.py -x -q -p no:cacheprovider \
      --timeout 300 --timeout-method thread > "$OUT/${v}_parity.log" 2>&1
    rc=$?; echo "$v parity:"; tail -2 "$OUT/${v}_parity.log"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
  ab 4 2 build/var_ref.so build/var_d0.so build/var_d2.so
  ab 2 "4 5" build/var_ref.so build/var_d0.so build/var_d2.so
  ab 1 3 build/var_ref.so build/var_d0.so build/var_d2.so
  ;;
x)  # per-launch clock of the streaming probe alone (is the clock dip the workload's or the GPU's?)
  (cd /tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$ROOT/$OUT/clk_probe" \
     -o run --output-format csv -- "$ROOT/tools/ring_probe" 1610612736 c > "$ROOT/$OUT/clk_probe.log" 2>&1) \
     || { echo "pmc clk_probe failed"; tail -3 "$OUT/clk_probe.log"; exit 1; }
  grep -h '"tag"' "$OUT/clk_probe.log"
  ;;
y)  # the short-frame instance with per-group job sequences (product) vs HEAD (ref): parity, then A/B
  tests
  ab 3 "5 3" onload_amd/liboo_gpu_rx.so build/var_ref.so
  ab 1 "2 4" onload_amd/liboo_gpu_rx.so build/var_ref.so
  ;;
z)  # ablation: the ring loop without its per-lane bookkeeping (results wrong), timed window and settled
  ab 3 2 onload_amd/liboo_gpu_rx.so build/var_lean.so
  ;;
fa)  # wave-uniform fast path for the body rounds (product) vs HEAD (ref): full suite, then A/B
  tests
  ab 4 2 onload_amd/liboo_gpu_rx.so build/var_ref.so
  ab 2 4 onload_amd/liboo_gpu_rx.so build/var_ref.so
  ab 1 5 onload_amd/liboo_gpu_rx.so build/var_ref.so
  ;;
fb)  # group 0's slot job by readlane instead of three bpermutes (product) vs HEAD (ref)
  tests
  ab 4 2 onload_amd/liboo_gpu_rx.so build/var_ref.so
  ab 1 "4 5" onload_amd/liboo_gpu_rx.so build/var_ref.so
  ;;
final)  # the round's evidence: full GPU suite, driver-shaped bench lines, rocprof of the same command
  tests
  for r in 1 2; do
    step bench$r 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_c2_$r.json" 2> "$OUT/bench_c2_$r.err"
    cat "$OUT/bench_c2_$r.json"
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
     --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 \
     > "$ROOT/$OUT/prof.log" 2>&1) || { echo "rocprof failed"; tail -5 "$OUT/prof.log"; exit 1; }
  find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
  for c in 3 4 5; do
    step bench_c$c 300 python bench.py --config $c --steps 20 --warmup 5 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
    python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[1], r["kernel_ms"], r["frac"], d["value"])' "$OUT/bench_c$c.json"
  done
  ;;
*)
  echo "unknown phase $PHASE"; exit 2 ;;
esac
echo "done $(date +%T)"
