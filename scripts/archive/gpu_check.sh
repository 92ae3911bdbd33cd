#!/usr/bin/env bash
# One GPU-box pass: host-tier tests, the headline bench, a CPU profile of the
# watcher process and a rocprofv3 kernel trace (expected: no GPU kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ nproc; lscpu | head -20; python -c "import torch;print(torch.__version__, torch.cuda.device_count())"; } > gpurun_out/host.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest -m gpu failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 600 python bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python -m cProfile -o gpurun_out/bench.prof bench.py --steps 3 --warmup 1 --ref-events 0 > gpurun_out/bench_prof.log 2>&1 || echo "profile run failed"
python -c "
import pstats; p=pstats.Stats('gpurun_out/bench.prof'); p.sort_stats('tottime').print_stats(30)" > gpurun_out/bench_prof.txt 2>&1
echo done
