set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
OO_RX_TSTEP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_l.log 2>&1; rc=$?; tail -2 gpurun_out/t_l.log; [ $rc -ne 0 ] && exit $rc
for c in 2 4 5; do SWEEP="OO_RX_TSTEP=8 OO_RX_TSTEP=1 OO_RX_LIB=build/var_prev.so" CONFIG=$c STEPS=40 bash tools/sweep.sh || exit $?; done
