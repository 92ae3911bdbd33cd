#!/usr/bin/env bash
# GPU-box pass: every-event-notified configs #2/#3 (benchmarks.suite) with the
# default pool and with pipelined pools, plus the N=1 headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in ${DEPTHS:-1 4 8 16}; do
  timeout -k 10 300 python -m benchmarks.suite --only 2,3 --set clusterapi.pool.pipeline_depth=$d --out gpurun_out/suite23_d$d.json > gpurun_out/suite23_d$d.md 2> gpurun_out/suite23_d$d.err || { echo "suite depth $d failed"; tail -20 gpurun_out/suite23_d$d.err; exit 1; }
  echo "depth $d"; tail -2 gpurun_out/suite23_d$d.md
done
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_n1.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n1.json')); print(d['value'], d['p50_latency_ms'], d['cpu_util_rank0'], d['verify']['exactly_once'])"
echo done
