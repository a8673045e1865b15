#!/bin/bash
# Round-4 evidence for each configuration: the driver-shaped bench line, the
# rocprofv3 kernel-trace stats of the same command, and the HBM PMC passes
# (FETCH_SIZE and WRITE_SIZE, one pass each, --kernel-trace only) of a short
# run.  Output under gpurun_out/final/; tools/pmc_summary.py turns the
# passes into profiles/pmc_config<N>.json.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/final"; mkdir -p "$OUT"
for c in ${CONFIGS:-2 3 4 5}; do
  extra=""; [ "$c" != 2 ] && extra="--no-cpu-baseline"
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 $extra \
    > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { tail -5 "$OUT/bench_c$c.err"; exit 1; }
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config $c --steps 20 --warmup 5 --steady 0 --no-cpu-baseline \
     > "$OUT/prof_c$c.log" 2>&1) || { tail -5 "$OUT/prof_c$c.log"; exit 1; }
  for pass in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $pass -d "$OUT/pmc_c$c/$pass" -o run \
       --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --steady 0 \
       --no-cpu-baseline > "$OUT/pmc_c$c.$pass.log" 2>&1) || { tail -5 "$OUT/pmc_c$c.$pass.log"; exit 1; }
  done
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print("c'$c'", d["value"], r["kernel_ms"], r["frac"], r.get("kernels"), (d.get("steady") or {}).get("frac"))' "$OUT/bench_c$c.json"
done
