#!/bin/bash
# Claim-group mapping A/B: parity of the mappings first, then bench lines for
# each mapping (tools/ab.sh).  OO_RX_GSHIFT=32: contiguous wave ranges.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  -k "tile_partitions" --timeout 120 --timeout-method thread > gpurun_out/groups_tests.log 2>&1 \
  || { tail -20 gpurun_out/groups_tests.log; exit 1; }
tail -2 gpurun_out/groups_tests.log
L=onload_amd/liboo_gpu_rx.so
LIBS="${LIBS:-$L $L@OO_RX_GSHIFT=32 $L@OO_RX_GSHIFT=32,OO_RX_GROUPS=32 $L@OO_RX_GSHIFT=32,OO_RX_GROUPS=16 $L@OO_RX_GSHIFT=4,OO_RX_GROUPS=32}" \
  CONFIGS="${CONFIGS:-2 3 5}" REPS=${REPS:-2} STEPS=30 bash tools/ab.sh
