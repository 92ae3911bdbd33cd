#!/usr/bin/env bash
# Notifier concurrency sweep on the GPU box (host CPU = the deployment CPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 600 python bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
i=0
for cfg in "--connections 16 --pipeline-depth 1" "--connections 32 --pipeline-depth 1" "--connections 16 --pipeline-depth 4" \
           "--connections 32 --pipeline-depth 8" "--connections 64 --pipeline-depth 4" "--sink-workers 8 --connections 32 --pipeline-depth 4"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --ref-events 0 $cfg --json-out gpurun_out/sweep/$i.json > gpurun_out/sweep/$i.log 2>&1 || echo "sweep $i failed"
  echo "$cfg => $(python -c "import json;d=json.load(open('gpurun_out/sweep/$i.json'));print(d['value'], d['p50_latency_ms'], d['saturated_p50_latency_ms'])" 2>/dev/null)"
done
timeout -k 10 300 python -m cProfile -o gpurun_out/bench.prof bench.py --steps 6 --warmup 1 --ref-events 0 --latency-seconds 0.2 > /dev/null 2>&1 || echo "profile failed"
python -c "import pstats; pstats.Stats('gpurun_out/bench.prof').sort_stats('tottime').print_stats(30)" > gpurun_out/bench_prof.txt 2>&1
echo done
