#!/usr/bin/env bash
# Full five-config suite on the GPU box host CPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -m benchmarks.suite --out gpurun_out/suite.json > gpurun_out/suite.md 2> gpurun_out/suite.err || { echo "suite failed"; tail -40 gpurun_out/suite.err; exit 1; }
cat gpurun_out/suite.md
