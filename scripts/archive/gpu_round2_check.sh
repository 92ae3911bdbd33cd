#!/usr/bin/env bash
# GPU-box pass: staging + production latency curves (tail check after the
# thread-placement change), then the https-API-server comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -m benchmarks.latency_curve --rates 100,1000,10000,100000 --out gpurun_out/latency_curve_staging.json > gpurun_out/latency_curve_staging.md || { echo "latency curve failed"; exit 1; }
cat gpurun_out/latency_curve_staging.md
bash scripts/gpu_tls_watch.sh
