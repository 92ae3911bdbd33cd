#!/usr/bin/env bash
# GPU-box pass: event->notify latency at 100 and 1,000 ev/s (production
# profile) for watch reader x thread pinning, alternating, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lat
for rep in 1 2; do
  for v in "native auto" "native none" "asyncio auto" "asyncio none"; do
    set -- $v
    name="$1-$2-$rep"
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --ref-events 0 --latency-seconds 20 --latency-seconds-high 10 \
      --watch-reader $1 --thread-pinning $2 --json-out gpurun_out/lat/$name.json > gpurun_out/lat/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/lat/$name.log; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/lat/$name.json')); h=d['latency_high_rate']
print('$name', round(d['value']), '| 100/s p50', d['p50_latency_ms'], 'p99', d['p99_latency_ms'], 'n', d['latency_samples'], '| 1k/s p50', h['p50_ms'], 'p90', h['p90_ms'], 'p99', h['p99_ms'], 'n', h['samples'])"
  done
done
echo done
