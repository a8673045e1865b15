set -u
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
TESTS="tests/test_gpu_parity.py tests/test_gpu_l4_ref.py tests/test_gpu_wait_variants.py tests/test_gpu_poll.py" CONFIGS="5 4" LIBS="onload_amd/liboo_gpu_rx.so onload_amd/liboo_gpu_rx.so@OO_RX_KERNEL=3,OO_RX_BODY_ENGINE=2 build/var_mt0.so@OO_RX_KERNEL=3,OO_RX_BODY_ENGINE=2" bash tools/r04_check.sh || exit 1
SKIP_TESTS=1 REPS=2 CONFIGS="3" LIBS="onload_amd/liboo_gpu_rx.so build/var_hx1.so build/var_hx2.so build/var_hx3.so" bash tools/r04_check.sh
