#!/usr/bin/env bash
# GPU-box pass: restart soak at 100k pods (SIGKILL + checkpoint resume),
# production latency curve, sharded bench N=1/2/4. Prints as it goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m benchmarks.restart_soak --pods 100000 --rounds 6 --kills 4 --round-seconds-hint 1.0 --out gpurun_out/restart_soak_100k.json > gpurun_out/restart_soak_100k.log 2>&1 || { echo "restart soak failed"; tail -40 gpurun_out/restart_soak_100k.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/restart_soak_100k.json')); print({k: d[k] for k in ('lost','duplicates','checkpoint_stall_ms_max','checkpoint_write_ms_max','checkpoint_bytes','watcher_peak_rss_mb','kills')})"
SKIP_STAGING=1 SHARD_NS="${SHARD_NS:-1 2 4}" bash scripts/gpu_latency_shard.sh
