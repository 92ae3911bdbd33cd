#!/usr/bin/env bash
# GPU-box pass: cProfile of the watcher process under bench.py, one
# cluster-wide watch vs 64 per-namespace watches (namespace_scope: discover).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for scope in cluster discover; do
  timeout -k 10 300 python -m cProfile -o gpurun_out/prof_$scope.prof bench.py --watch-scope $scope --steps 6 --warmup 1 --ref-events 0 --latency-seconds 1 --json-out gpurun_out/prof_$scope.json > gpurun_out/prof_$scope.log 2>&1 || { echo "prof $scope failed"; tail -20 gpurun_out/prof_$scope.log; exit 1; }
  python -c "
import json, pstats, io
d = json.load(open('gpurun_out/prof_$scope.json'))
print('$scope', d['value'], d['cpu_util_rank0'], d['cpu_other_threads_rank0'])
s = io.StringIO(); p = pstats.Stats('gpurun_out/prof_$scope.prof', stream=s); p.sort_stats('tottime').print_stats(25); print(s.getvalue()[:6000])" | tee gpurun_out/prof_$scope.txt
done
echo done
