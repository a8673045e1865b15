#!/bin/bash
# Round-4 GPU pass: the -m gpu suite, then bench lines -- the driver's shape
# on config 2, configs 3-5, and config 3 in the AF_XDP UMEM layout.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline ${EXTRA:-} \
    > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || exit 1
done
timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --steady 0 --xdp \
  > gpurun_out/bench_c3_xdp.json 2> gpurun_out/bench_c3_xdp.err || exit 1
for f in gpurun_out/bench_c*.json; do
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[1], d["value"], r["kernel_ms"], r["frac"], (d.get("steady") or {}).get("frac"), d.get("xdp_ring"), (d.get("cpu_baseline") or {}).get("value"))' $f
done
