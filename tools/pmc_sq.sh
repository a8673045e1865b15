#!/bin/bash
# SQ counter passes (instruction mix / activity) for bench.py on CONFIG with
# the library OO_RX_LIB (default: product) and kernel OO_RX_KERNEL.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; export TMPDIR=/tmp
CONFIG="${CONFIG:-2}"; OUT="$ROOT/gpurun_out/pmc_sq_${TAG:-x}"; mkdir -p "$OUT"
pass() {
  local name=$1; shift
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run \
     --output-format csv -- python3 "$ROOT/bench.py" --config "$CONFIG" --steps 5 --warmup 1 \
     --no-cpu-baseline > "$OUT/$name.log" 2>&1) || { echo "pass $name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "rx_" in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(" ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(d.items())))
PY
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
