#!/usr/bin/env bash
# A/B: native notifier on its own I/O thread (default) vs driven from the event loop, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/io
for i in 1 2 3; do
  for m in thread loop; do
    a=""; [ $m = thread ] && a="--io-thread"
    timeout -k 10 300 python bench.py --ref-events 0 $a > gpurun_out/io/$m-$i.json 2> gpurun_out/io/$m-$i.err || { echo "$m $i failed"; tail -5 gpurun_out/io/$m-$i.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/io/$m-$i.json').read().strip().splitlines()[-1]);print('$m',$i,d['value'],d['p50_latency_ms'],d['cpu_util_rank0'],d['cpu_other_threads_rank0'][:5])"
  done
done
