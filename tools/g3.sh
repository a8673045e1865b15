set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
LIBS="onload_amd/liboo_gpu_rx.so build/var_prev.so" CONFIG=2 bash tools/fetch_pass.sh || exit 1
for c in 2 2 2; do SWEEP="OO_RX_KERNEL=lanes OO_RX_LIB=build/var_prev.so" CONFIG=$c STEPS=60 bash tools/sweep.sh || exit $?; done
