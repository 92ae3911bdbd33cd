#!/usr/bin/env bash
# Three headline bench runs (default flags) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/b3
for i in 1 2 3; do
  a=""; [ $i -gt 1 ] && a="--ref-events 0"
  timeout -k 10 300 python bench.py $a > gpurun_out/b3/run$i.json 2> gpurun_out/b3/run$i.err || { echo "run $i failed"; tail -5 gpurun_out/b3/run$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b3/run$i.json').read().strip().splitlines()[-1]);print($i,d['value'],d['vs_baseline'],d['p50_latency_ms'],d['cpu_util_rank0'],d.get('cpu_other_threads_rank0'))"
done
