set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for k in lanes split; do
  OO_RX_KERNEL=$k timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_$k.log 2>&1
  rc=$?; tail -4 gpurun_out/t_$k.log; echo "tests $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
SWEEP="OO_RX_KERNEL=split OO_RX_KERNEL=lanes" CONFIG=2 STEPS=100 bash tools/sweep.sh || exit $?
for c in 3 4 5; do SWEEP="OO_RX_KERNEL=split OO_RX_KERNEL=lanes" CONFIG=$c STEPS=30 bash tools/sweep.sh || exit $?; done
for c in 2 3; do OO_RX_LIB=build/var_st.so OO_RX_KERNEL=lanes timeout -k 10 200 python tools/stamps.py --config $c || exit $?; done
