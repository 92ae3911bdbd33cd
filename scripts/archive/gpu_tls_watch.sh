#!/usr/bin/env bash
# GPU-box pass: https API server (every real cluster) — the watch decrypted by
# the reader hub's OpenSSL session vs by asyncio's ssl on the event loop,
# cluster-wide watch and 64 namespace watches, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tls
for rep in 1 2; do
  for v in "native cluster" "asyncio cluster" "native discover" "asyncio discover"; do
    set -- $v
    name="$1-$2-$rep"
    timeout -k 10 300 python bench.py --api-tls --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 \
      --watch-reader $1 --watch-scope $2 --json-out gpurun_out/tls/$name.json > gpurun_out/tls/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/tls/$name.log; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/tls/$name.json')); h=d['latency_high_rate']
print('$name', round(d['value']), 'cpu', d['cpu_util_rank0'], 'ev/watcher-cpu-s', d['events_per_watcher_cpu_second'], '| p50 100/s', d['p50_latency_ms'], '1k/s', h['p50_ms'], 'exactly_once', d['verify']['exactly_once'])"
  done
done
echo done
