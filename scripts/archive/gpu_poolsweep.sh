#!/usr/bin/env bash
# notifier pool shape sweep (loop-thread bound regime): connections x pipeline depth
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ps
for cfg in "16 4" "4 16" "8 8" "4 32" "2 64" "16 4"; do
  set -- $cfg
  n=c$1d$2
  timeout -k 10 300 python bench.py --ref-events 0 --connections $1 --pipeline-depth $2 > gpurun_out/ps/$n.json 2> gpurun_out/ps/$n.err || { echo "$n failed"; tail -5 gpurun_out/ps/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ps/$n.json').read().strip().splitlines()[-1]);print('$n',d['value'],d['p50_latency_ms'],d['saturated_p50_latency_ms'],d['cpu_util_rank0'])"
done
