#!/bin/bash
# Round-4 check on a GPU box: the -m gpu suite, then same-box bench lines of
# the product's auto path against the split transform (OO_RX_KERNEL=3) on
# configs 2-5 (LIBS: other builds or settings, path@VAR=val).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    ${TESTS_K:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
REPS=${REPS:-1} CONFIGS="${CONFIGS:-2 3 4 5}" STEPS=${STEPS:-20} \
  LIBS="${LIBS:-onload_amd/liboo_gpu_rx.so onload_amd/liboo_gpu_rx.so@OO_RX_KERNEL=3}" \
  bash tools/ab.sh 2>&1 | tee gpurun_out/ab.log
