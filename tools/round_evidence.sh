#!/bin/bash
# One GPU call that regenerates the round's evidence under gpurun_out/ev/:
# the -m gpu suite, bench lines for configs 2-5 (config 2 with the CPU
# baseline and the host-memory path), a rocprofv3 kernel-trace/stats run of
# the config-2 bench, and FETCH_SIZE / WRITE_SIZE passes for the HBM traffic.
#   gpurun --timeout 1200 -- bash tools/round_evidence.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT=gpurun_out/ev
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, then the command; stops the script on any failure
  local name=$1; shift
  echo "== $name"
  "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; exit $rc; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && { echo "gpu tests failed rc=$rc"; exit $rc; }
step bench2 timeout -k 10 300 sh -c "python bench.py --config 2 --steps 50 --warmup 5 --host-path --tx --xdp > $OUT/bench_config2.json 2> $OUT/bench_config2.err"
cat "$OUT/bench_config2.json"
for c in 3 4 5; do
  step bench$c timeout -k 10 300 sh -c "python bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 5 > $OUT/bench_config$c.json 2> $OUT/bench_config$c.err"
  cat "$OUT/bench_config$c.json"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run \
   --output-format csv -- python3 "$ROOT/bench.py" --config 2 --steps 50 --warmup 5 \
   --no-cpu-baseline > "$ROOT/$OUT/prof.log" 2>&1) || { echo "rocprof failed"; tail -5 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
LIBS="onload_amd/liboo_gpu_rx.so" CONFIG=2 bash tools/fetch_pass.sh || exit 1
echo done
