set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for l in s4 w3s4 w3s2 w1s8 w1s12 r2 w3r4 w4r2; do python3 -c "import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); print(sys.argv[1], L.oo_rx_blocks_per_cu(0), L.oo_rx_blocks_per_cu(1))" build/var_$l.so; done
S=""; for v in s6 s4 s6np w3s4 w3s2 w1s8 w1s12; do S="$S OO_RX_KERNEL=split;OO_RX_LIB=build/var_$v.so"; done; for v in r4 r2 w3r4 w4r2; do S="$S OO_RX_KERNEL=lanes;OO_RX_LIB=build/var_$v.so"; done
SWEEP="$S" CONFIG=2 STEPS=100 bash tools/sweep.sh || exit $?
