#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of bench.py for each library
# variant named in LIBS (default: the product library).  Prints per-launch
# averages for the rx kernel.  Usage: LIBS="build/var_a.so ..." CONFIG=2 bash tools/fetch_pass.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
CONFIG="${CONFIG:-2}"
mkdir -p gpurun_out/fetch
for lib in ${LIBS:-onload_amd/liboo_gpu_rx.so}; do
  for ctr in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
    name=$(basename "$lib" .so)_$ctr
    (cd /tmp && OO_RX_LIB="$ROOT/$lib" timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr \
       -d "$ROOT/gpurun_out/fetch/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" \
       --config "$CONFIG" --steps 5 --warmup 1 --no-cpu-baseline > "$ROOT/gpurun_out/fetch/$name.log" 2>&1)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 "$ROOT/gpurun_out/fetch/$name.log"; exit $rc; fi
    f=$(find "$ROOT/gpurun_out/fetch/$name" -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$name" <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "rx_kernel" in r["Kernel_Name"]]
print(sys.argv[2], "launches", len(v), "avg", sum(v) / max(1, len(v)))
PY
  done
done
