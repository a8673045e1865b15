set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_tx.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_l.log 2>&1; rc=$?; tail -2 gpurun_out/t_l.log; [ $rc -ne 0 ] && exit $rc
for lib in onload_amd/liboo_gpu_rx.so build/var_prev.so onload_amd/liboo_gpu_rx.so build/var_prev.so; do
  OO_RX_LIB=$lib timeout -k 10 200 python bench.py --config 2 --steps 30 --warmup 3 --no-cpu-baseline --tx > gpurun_out/tx.json 2> gpurun_out/tx.err || { tail -5 gpurun_out/tx.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/tx.json')); print('$lib', d['roofline']['kernel_ms'], d['tx_fill'])"
done
