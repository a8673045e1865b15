#!/bin/bash
# Config-2 launch overhead and tail-tile knobs (one box).
set -u
L=onload_amd/liboo_gpu_rx.so
REPS=2 CONFIGS=2 LIBS="$L $L@OO_RX_TAIL_TILE=16,OO_RX_TAIL_PER_WAVE=2 $L@OO_RX_TAIL_TILE=8,OO_RX_TAIL_PER_WAVE=2 $L@OO_RX_TAIL_TILE=64 $L@OO_RX_STATIC=1" bash tools/ab.sh || exit $?
for n in 524288 2097152; do
  EXTRA="--n $n" REPS=1 CONFIGS=2 LIBS="$L" bash tools/ab.sh || exit $?
done
