#!/usr/bin/env bash
# https clusterapi (production.yaml's scheme): native TLS core vs asyncio pool, and plain http for scale.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tls
run() { name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/tls/$name.json 2> gpurun_out/tls/$name.err || { echo "$name failed"; tail -5 gpurun_out/tls/$name.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/tls/$name.json').read().strip().splitlines()[-1]);r=d['reference_equiv'] or {};print('$name',d['value'],'p50',d['p50_latency_ms'],'p99',d['p99_latency_ms'],'ref',r.get('events_per_s'),d['cpu_util_rank0'])"
}
run https-native --tls
run https-python --tls --python-pool --ref-events 0
run http-native --ref-events 0
