#!/usr/bin/env bash
# Host-tier tests, headline bench (twice), five-config suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --json-out gpurun_out/bench_$i.json > gpurun_out/bench_$i.log 2>&1 || { tail -30 gpurun_out/bench_$i.log; exit 1; }
  cat gpurun_out/bench_$i.json
done
timeout -k 10 1000 python -m benchmarks.suite --out gpurun_out/suite.json > gpurun_out/suite.md 2> gpurun_out/suite.err || { echo "suite failed"; tail -40 gpurun_out/suite.err; exit 1; }
cat gpurun_out/suite.md
