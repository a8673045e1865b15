#!/bin/bash
# GPU tests on the product, then a same-box A/B against build/var_nolast.so,
# then phase stamps (build/var_st.so) for configs 5 and 3.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/exp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/exp_tests.log; [ $rc -ne 0 ] && exit $rc
L=onload_amd/liboo_gpu_rx.so
REPS=2 CONFIGS="${CONFIGS:-2 3 4 5}" STEPS=20 LIBS="$L ${ALT:-build/var_nolast.so}" bash tools/ab.sh || exit $?
[ -n "${STAMPS:-}" ] && CONFIGS="$STAMPS" bash tools/evidence_r02.sh C
exit 0
