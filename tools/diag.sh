#!/bin/bash
# Diagnostics for the weak configurations: per-wave phase stamps (a
# -DOO_RX_STAMPS build, build/var_st.so) and the PMC passes of tools/pmc.sh
# per configuration.  Usage: gpurun -- bash tools/diag.sh   (CONFIGS="3 4 5")
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/diag
for c in ${STAMP_CONFIGS:-2 3 4 5}; do
  OO_RX_LIB=build/var_st.so timeout -k 10 200 python tools/stamps.py --config "$c" \
    > gpurun_out/diag/stamps_c$c.json 2> gpurun_out/diag/stamps_c$c.err
  rc=$?; echo "stamps c$c rc=$rc"; cat gpurun_out/diag/stamps_c$c.json
  [ $rc -ne 0 ] && { tail -5 gpurun_out/diag/stamps_c$c.err; exit $rc; }
done
for c in ${PMC_CONFIGS-3 4 5}; do
  CEILING=0 CONFIG=$c STEPS=5 bash tools/pmc.sh || exit $?
done
echo done
