set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for k in lanes split; do OO_RX_KERNEL=$k timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$k.log 2>&1; rc=$?; tail -2 gpurun_out/t_$k.log; [ $rc -ne 0 ] && exit $rc; done
S="OO_RX_KERNEL=lanes OO_RX_KERNEL=lanes;OO_RX_LIB=build/var_nohp.so OO_RX_KERNEL=split;OO_RX_LIB=build/var_s4.so OO_RX_KERNEL=split;OO_RX_LIB=build/var_s4np.so"
SWEEP="$S" CONFIG=2 STEPS=100 bash tools/sweep.sh || exit $?
for c in 3 4 5; do SWEEP="OO_RX_KERNEL=lanes OO_RX_KERNEL=split;OO_RX_LIB=build/var_s4.so" CONFIG=$c STEPS=30 bash tools/sweep.sh || exit $?; done
OO_RX_KERNEL=lanes LIBS="onload_amd/liboo_gpu_rx.so" COUNTERS=FETCH_SIZE CONFIG=2 bash tools/fetch_pass.sh || exit $?
