set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for c in 2 3; do OO_RX_LIB=build/var_st.so OO_RX_KERNEL=lanes timeout -k 10 200 python tools/stamps.py --config $c || exit $?; done
OO_RX_LIB=build/var_st.so OO_RX_KERNEL=split timeout -k 10 200 python tools/split_stamps.py --config 2 || exit $?
SWEEP="OO_RX_KERNEL=split OO_RX_KERNEL=lanes" CONFIG=2 STEPS=100 bash tools/sweep.sh || exit $?
