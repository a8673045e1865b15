set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
S=""
for v in ${VARS:-noparse s4 s12 s16 ws3 ws1}; do S="$S OO_RX_KERNEL=${KER:-split};OO_RX_LIB=build/var_$v.so"; done
SWEEP="OO_RX_KERNEL=${KER:-split} $S" CONFIG=${CONFIG:-2} STEPS=100 bash tools/sweep.sh || exit $?
