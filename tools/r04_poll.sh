#!/bin/bash
# The batched RX branch per poll on the GPU box (tools/poll_bench): configs
# 2 and 3, 16 / 64 / 1024 / 65536 events per poll, gather, zero-copy and
# zero-copy with the crossover; JSON lines to gpurun_out/poll_r04.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
: > gpurun_out/poll_r04.jsonl
for c in ${CONFIGS:-2 3}; do
  timeout -k 10 300 tools/poll_bench $c ${FRAMES:-262144} ${EPP:-16 64 1024 65536} >> gpurun_out/poll_r04.jsonl \
    2> gpurun_out/poll_r04.err || { tail -5 gpurun_out/poll_r04.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/poll_r04.jsonl"):
    d = json.loads(l)
    print({k: d.get(k) for k in ("config", "evs_per_poll", "mode", "poll_us_median", "mpps", "cpu_poll_us_equiv", "handed_back", "fit")})
PY
