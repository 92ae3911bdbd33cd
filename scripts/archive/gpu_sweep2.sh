#!/usr/bin/env bash
# decode-thread sweep at the current defaults + a cProfile of the watcher process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sw
for t in 1 2 3 5 7; do
  timeout -k 10 300 python bench.py --ref-events 0 --decode-threads $t > gpurun_out/sw/t$t.json 2> gpurun_out/sw/t$t.err || { echo "t=$t failed"; tail -5 gpurun_out/sw/t$t.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sw/t$t.json').read().strip().splitlines()[-1]);print('threads',$t,d['value'],d['cpu_util_rank0'],d['events_per_watcher_cpu_second'])"
done
timeout -k 10 300 python -m cProfile -o gpurun_out/sw/bench.prof bench.py --steps 10 --warmup 2 --ref-events 0 --latency-seconds 1 > gpurun_out/sw/prof.log 2>&1 || { echo "profile failed"; exit 1; }
python -c "
import pstats; p=pstats.Stats('gpurun_out/sw/bench.prof'); p.sort_stats('tottime').print_stats(25)" > gpurun_out/sw/prof.txt 2>&1
tail -1 gpurun_out/sw/prof.log | cut -c1-200
