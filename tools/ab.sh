#!/bin/bash
# Same-box A/B of library builds: bench lines for each OO_RX_LIB in LIBS,
# configs in CONFIGS, REPS rounds interleaved (boxes differ by several
# percent; compare only within one call).  A LIBS entry may carry
# environment settings: path@VAR=val,VAR2=val.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for c in ${CONFIGS:-2}; do
    for spec in ${LIBS:-onload_amd/liboo_gpu_rx.so}; do
      lib=${spec%%@*}; envs=""
      [ "$spec" != "$lib" ] && envs=$(echo "${spec#*@}" | tr ',' ' ')
      out=$(env $envs OO_RX_LIB=$lib timeout -k 10 300 python bench.py --config "$c" --steps "${STEPS:-30}" \
            --warmup 5 --no-cpu-baseline ${EXTRA:-} 2> gpurun_out/ab_last.err)
      rc=$?
      if [ $rc -ne 0 ]; then echo "$spec c$c rc=$rc"; tail -5 gpurun_out/ab_last.err; exit $rc; fi
      echo "rep$rep c$c $spec $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms"], r["frac"], d["value"])')"
    done
  done
done
