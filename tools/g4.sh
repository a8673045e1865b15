set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
OO_RX_KERNEL=split timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_split.log 2>&1
rc=$?; tail -3 gpurun_out/t_split.log; [ $rc -ne 0 ] && exit $rc
SWEEP="OO_RX_KERNEL=split OO_RX_KERNEL=split;OO_RX_LIB=build/var_noparse.so" CONFIG=2 STEPS=100 bash tools/sweep.sh || exit $?
SWEEP="OO_RX_KERNEL=split" CONFIG=3 STEPS=50 bash tools/sweep.sh || exit $?
OO_RX_KERNEL=split OO_RX_LIB=build/var_noparse.so TAG=splitnp bash tools/pmc_sq.sh || exit $?
OO_RX_KERNEL=lanes OO_RX_LIB=build/var_nohp.so TAG=lanesnhp bash tools/pmc_sq.sh || exit $?
