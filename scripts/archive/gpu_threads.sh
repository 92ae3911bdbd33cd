#!/usr/bin/env bash
# Decode-thread sweep on the GPU box host: headline bench (default = auto
# threads) plus --decode-threads 0..7 and --sink-workers variants, one JSON
# line each into gpurun_out/threads.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ nproc; python -c "import os;print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > gpurun_out/host_cpus.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
: > gpurun_out/threads.jsonl
DEFAULT_SWEEP="--decode-threads 0|--decode-threads 2|--decode-threads 3|--decode-threads 3 --decode-affinity none|--decode-threads 5"
IFS='|' read -r -a SWEEP_ARGS <<< "${SWEEP:-$DEFAULT_SWEEP}"
for args in "${SWEEP_ARGS[@]}"; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --ref-events 0 $args --json-out gpurun_out/t.json \
    > gpurun_out/t.log 2>&1 || { echo "failed: $args"; tail -20 gpurun_out/t.log; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/t.json')); print(json.dumps({'args': sys.argv[1], 'value': d['value'], 'p50': d['p50_latency_ms'], 'sat_p50': d['saturated_p50_latency_ms'], 'cpu': d['cpu_util_rank0']}))" "$args" | tee -a gpurun_out/threads.jsonl
done
echo done
