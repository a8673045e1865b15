#!/bin/bash
# Diagnostic order of the -m gpu suite: test_gpu_tables.py first, then every
# other GPU test file; HIP error logging on (AMD_LOG_LEVEL=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/diag
files="tests/test_gpu_tables.py $(ls tests/test_gpu_*.py | grep -v test_gpu_tables.py | tr '\n' ' ')"
AMD_LOG_LEVEL=1 timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/diag/tests.log 2>&1
rc=$?
tail -5 gpurun_out/diag/tests.log
exit $rc
