#!/usr/bin/env bash
# GPU-box pass: latency vs offered load (staging: every event notified;
# production: ~20% notified, capped at 90 s per rate), then the sharded bench
# N=1/2/4 on the current fixture. Every step prints as it goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_STAGING" ]; then
  timeout -k 10 500 python -m benchmarks.latency_curve --out gpurun_out/latency_curve_staging.json > gpurun_out/latency_curve_staging.md || { echo "latency curve failed"; exit 1; }
  cat gpurun_out/latency_curve_staging.md
fi
timeout -k 10 700 python -m benchmarks.latency_curve --profile production --ref-rates 100,1000 --out gpurun_out/latency_curve_production.json > gpurun_out/latency_curve_production.md || { echo "latency curve prod failed"; exit 1; }
cat gpurun_out/latency_curve_production.md
for n in ${SHARD_NS:-1 2 4}; do
  if [ "$n" = 1 ]; then
    timeout -k 10 300 python bench.py --json-out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || { echo "bench n1 failed"; tail -30 gpurun_out/bench_n1.log; exit 1; }
  else
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29400 + n)) bench.py --gpus $n --ref-events 0 --json-out gpurun_out/bench_n$n.json > gpurun_out/bench_n$n.log 2>&1 || { echo "bench n$n failed"; tail -30 gpurun_out/bench_n$n.log; exit 1; }
  fi
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_n$n.json')); print($n, d['value'], d['p50_latency_ms'], d['latency_samples'], d['verify']['exactly_once'], d['cpu_util_rank0'])"
done
echo done
