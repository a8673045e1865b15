#!/bin/bash
# The -m gpu suite, then a same-box A/B of LIBS (tools/ab.sh) -- one call.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 180 \
  --timeout-method thread > gpurun_out/gpu_full.log 2>&1 || { tail -30 gpurun_out/gpu_full.log; exit 1; }
tail -1 gpurun_out/gpu_full.log
bash tools/ab.sh
