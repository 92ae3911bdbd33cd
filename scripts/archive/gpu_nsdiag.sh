#!/usr/bin/env bash
# Namespace-watch diagnosis on the box: perf availability, then the loop probe
# (split / decode wait / apply per line, data age at first touch) for one
# cluster watch vs 64 and 1000 namespace watches at N=1, and the staging
# (every event notified) shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/nsdiag}
mkdir -p "$OUT"
{ which perf; perf --version; cat /proc/sys/kernel/perf_event_paranoid; nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"; lscpu | grep -E "Model name|L3|L2"; } > "$OUT/host.txt" 2>&1
B="--steps 6 --warmup 2 --rounds-per-step ${ROUNDS:-4} --latency-seconds 0 --latency-seconds-high 0 --ref-events 0 --apart off --staging off --probe"
run() { name=$1; shift; timeout -k 10 300 python bench.py $B --json-out "$OUT/$name.json" "$@" > "$OUT/$name.log" 2>&1 || { echo "FAILED $name"; tail -20 "$OUT/$name.log"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); p=d.get('loop_probe_rank0') or {}; l=max(1,p.get('lines',1)); print('$name', d['value'], 'split/wait/apply ns', round(p.get('split_ns',0)/l), round(p.get('wait_ns',0)/l), round(p.get('apply_ns',0)/l), 'lines/call', round(l/max(1,p.get('calls',1))), 'age_us', round(p.get('data_age_us',0)), 'io_ns', round(p.get('notifier_io_ns',0)/l), 'cpu', d['cpu_util_rank0'], 'hub', {k: d.get('watch_reader_rank0', {}).get(k) for k in ('reads', 'signals', 'starved', 'hub_dispatch_watches')})"; }
# default: the pieces given on the command line after OUT, else the whole set
if [ $# -gt 1 ]; then shift; for spec in "$@"; do IFS=: read -r name rest <<< "$spec"; run "$name" ${rest//,/ }; done; echo done; exit 0; fi
run cluster --watch-scope cluster
run ns64 --watch-scope discover
run ns64_off --watch-scope discover --hub-dispatch off
run ns1000 --watch-scope discover --namespaces 1000
run ns1000_off --watch-scope discover --namespaces 1000 --hub-dispatch off
run ns1000_bufs --watch-scope discover --namespaces 1000 --watch-reader-buffers 512 --watch-read-bytes 1048576
run staging --profile staging
run staging_io --profile staging --io-thread
echo done
