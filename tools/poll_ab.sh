#!/bin/bash
# Same-box A/B of library builds under the deployed poll shape:
# tools/poll_bench (CONFIGS, FRAMES, EPP) once per VARIANTS entry
# name:hipcc-flags (flags comma-separated; "base" = the product build), the
# variant loaded in place of onload_amd/liboo_gpu_rx.so through
# LD_LIBRARY_PATH (the shim's RUNPATH yields to it).  One JSON line per run,
# with "variant" added, on stdout.  Builds are made here on the CPU side
# (make poll-variants) and travel with the tree.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-base}; do
    name=${v%%:*}
    dir="build/pollvar/$name"
    [ "$name" = base ] && dir="onload_amd"
    [ -f "$dir/liboo_gpu_rx.so" ] || { echo "missing $dir/liboo_gpu_rx.so" >&2; exit 2; }
    for c in ${CONFIGS:-2 3}; do
      LD_LIBRARY_PATH="$ROOT/$dir" timeout -k 10 300 tools/poll_bench "$c" ${FRAMES:-262144} ${EPP:-16 64 1024} \
        > gpurun_out/poll_ab_last.jsonl 2> gpurun_out/poll_ab_last.err || { tail -5 gpurun_out/poll_ab_last.err; exit 1; }
      python3 -c 'import json,sys
for l in open(sys.argv[1]):
    d = json.loads(l); d["variant"] = sys.argv[2]; d["rep"] = int(sys.argv[3]); print(json.dumps(d))' \
        gpurun_out/poll_ab_last.jsonl "$name" "$rep"
    done
  done
done
