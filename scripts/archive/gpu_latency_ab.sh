#!/usr/bin/env bash
# GPU-box A/B of the staging latency curve at high offered load: the current
# extension vs another build ($PREV_SO, loaded through $K8S_WATCHER_KWCORE_SO),
# interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/latab
for rep in 1 2; do
  for v in prev cur; do
    if [ $v = prev ]; then export K8S_WATCHER_KWCORE_SO=$PREV_SO; else unset K8S_WATCHER_KWCORE_SO; fi
    timeout -k 10 300 python -m benchmarks.latency_curve --rates ${RATES:-10000,100000,500000} --ref-rates "" \
      --out gpurun_out/latab/${v}_$rep.json > gpurun_out/latab/${v}_$rep.md 2> gpurun_out/latab/${v}_$rep.err || { echo "$v failed"; tail -20 gpurun_out/latab/${v}_$rep.err; exit 1; }
    echo "== $v $rep"; grep -E "^\| [0-9]" gpurun_out/latab/${v}_$rep.md
  done
done
echo done
