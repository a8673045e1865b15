#!/bin/bash
# TX fill A/B: the product against ALT on config 2 (same box, interleaved).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for lib in onload_amd/liboo_gpu_rx.so $ALT; do
    OO_RX_LIB=$lib timeout -k 10 300 python bench.py --config 2 --steps 30 --warmup 5 --no-cpu-baseline --tx \
      2> gpurun_out/txab.err | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$lib'", d["roofline"]["kernel_ms"], d["tx_fill"]["kernel_ms"], d["tx_fill"]["frac"])' || exit 1
  done
done
