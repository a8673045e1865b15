#!/bin/bash
# Timing experiment: the split transform's two kernels concurrently on two
# streams (build/var_concur.so, results wrong) against the product's paths.
# LIBS entries as tools/ab.sh; the concurrent build needs OO_RX_KERNEL=3.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
REPS=${REPS:-1} CONFIGS="${CONFIGS:-2 4 5}" STEPS=${STEPS:-20} \
  LIBS="${LIBS:-onload_amd/liboo_gpu_rx.so build/var_concur.so@OO_RX_KERNEL=3 build/var_concur.so@OO_RX_KERNEL=3,OO_RX_GRID_PCT=67,OO_RX_BODY_BPC=3 build/var_concur.so@OO_RX_KERNEL=3,OO_RX_GRID_PCT=34,OO_RX_BODY_BPC=4}" \
  bash tools/ab.sh 2>&1 | tee gpurun_out/concur.log
