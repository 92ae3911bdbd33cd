#!/usr/bin/env bash
# Flakiness hunt on the box's host: the CPU tier 10x (xdist), failures collected.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/flaky
for i in $(seq 1 10); do
  timeout -k 10 300 python -m pytest tests -m "not gpu" -q -n 8 --timeout 120 -rf -p no:cacheprovider > gpurun_out/flaky/run$i.log 2>&1
  echo "run $i rc=$? $(tail -1 gpurun_out/flaky/run$i.log)"
  grep -E "^FAILED" gpurun_out/flaky/run$i.log || true
done
