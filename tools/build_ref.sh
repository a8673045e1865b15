#!/bin/bash
# Builds the product library of git revision REV (default HEAD) as
# build/var_<NAME>.so (default NAME=ref), for same-box A/B sweeps
# (OO_RX_LIB=build/var_ref.so) -- run-to-run differences between GPU boxes
# are a few percent, more than many of the changes being measured.
# EXTRA adds compiler flags (EXTRA=-DOO_RX_STAMPS for a stamps build);
# every such build is an experiments build (-DOO_RX_EXPERIMENTS).
set -eu
REV="${1:-HEAD}"; NAME="${2:-ref}"
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" onload_amd/csrc include | tar -x -C "$T"
mkdir -p "$ROOT/build"
SRCS=$(ls "$T"/onload_amd/csrc/*.hip "$T"/onload_amd/csrc/oo_gpu_rx.cpp "$T"/onload_amd/csrc/oo_gpu_rx_group.cpp "$T"/onload_amd/csrc/oo_rx_csum.cpp 2>/dev/null)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -DOO_RX_EXPERIMENTS ${EXTRA:-} -shared -Wl,-soname,liboo_gpu_rx.so \
  -o "$ROOT/build/var_$NAME.so" $SRCS
rm -rf "$T"
echo "build/var_$NAME.so <- $REV"
