set -u
mkdir -p gpurun_out/r06b
OO_RX_LIB=build/var_deepall.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_l4_ref.py tests/test_gpu_xdp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06b/deep_tests.log 2>&1 || { tail -30 gpurun_out/r06b/deep_tests.log; exit 1; }
tail -2 gpurun_out/r06b/deep_tests.log
TAG=r06b STEPS=ab CONFIGS="5 2" LIBS="onload_amd/liboo_gpu_rx.so build/var_deeps.so build/var_deepall.so" REPS=2 bash tools/gpu_round.sh
