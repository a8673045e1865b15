set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_xdp.py tests/test_gpu_tx.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_l.log 2>&1; rc=$?; tail -2 gpurun_out/t_l.log; [ $rc -ne 0 ] && exit $rc
for c in 2 5 2; do SWEEP="OO_RX_KERNEL=lanes OO_RX_LIB=build/var_prev.so" CONFIG=$c STEPS=40 bash tools/sweep.sh || exit $?; done
