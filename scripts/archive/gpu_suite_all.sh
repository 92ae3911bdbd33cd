#!/usr/bin/env bash
# GPU-box pass: the five BASELINE configurations (benchmarks.suite), the
# every-event configs with the asyncio watch read for comparison, and the
# host's CPU quota (what an N-rank rehearsal on this box shares).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; nproc; } > gpurun_out/cgroup.txt 2>&1
timeout -k 10 900 python -m benchmarks.suite --out gpurun_out/suite.json > gpurun_out/suite.md 2> gpurun_out/suite.err || { echo "suite failed"; tail -30 gpurun_out/suite.err; exit 1; }
cat gpurun_out/suite.md
timeout -k 10 300 python -m benchmarks.suite --only 2,3 --set watcher.watch_reader=asyncio --out gpurun_out/suite23_asyncio.json > gpurun_out/suite23_asyncio.md 2> gpurun_out/suite23_asyncio.err || { echo "suite asyncio failed"; tail -20 gpurun_out/suite23_asyncio.err; exit 1; }
tail -4 gpurun_out/suite23_asyncio.md
cat gpurun_out/cgroup.txt
echo done
