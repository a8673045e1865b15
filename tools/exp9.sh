#!/bin/bash
# GPU tests on the product, then a same-box A/B against ALT over CONFIGS.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/exp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/exp_tests.log; [ $rc -ne 0 ] && exit $rc
L=onload_amd/liboo_gpu_rx.so
REPS=${REPS:-2} CONFIGS="${CONFIGS:-2 3 4 5}" STEPS=20 LIBS="$L ${ALT}" bash tools/ab.sh
