#!/usr/bin/env bash
# cProfile of the headline bench's watcher process (Python-level view of the event-loop thread).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
timeout -k 10 300 python -m cProfile -o gpurun_out/prof/bench.prof bench.py --steps 20 --warmup 2 --ref-events 0 --latency-seconds 1 > gpurun_out/prof/run.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/prof/run.log; exit 1; }
python -c "
import pstats; p=pstats.Stats('gpurun_out/prof/bench.prof'); p.sort_stats('tottime').print_stats(30)" > gpurun_out/prof/prof.txt 2>&1
tail -1 gpurun_out/prof/run.log | cut -c1-300
