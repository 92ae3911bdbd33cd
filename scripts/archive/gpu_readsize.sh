#!/usr/bin/env bash
# A/B of watcher.watch_read_bytes (bytes per socket read on the watch), alternating runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rs
for i in 1 2 3; do
  for rb in 262144 1048576 4194304; do
    timeout -k 10 300 python bench.py --ref-events 0 --watch-read-bytes $rb > gpurun_out/rs/$rb-$i.json 2> gpurun_out/rs/$rb-$i.err || { echo "$rb $i failed"; tail -5 gpurun_out/rs/$rb-$i.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rs/$rb-$i.json').read().strip().splitlines()[-1]);print($rb,$i,d['value'],d['p50_latency_ms'],d['cpu_util_rank0'])"
  done
done
