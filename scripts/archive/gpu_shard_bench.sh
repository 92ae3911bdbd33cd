#!/usr/bin/env bash
# GPU-box pass for the sharded bench: host-tier tests, then bench.py at N=1
# (cluster-wide watch, the config #4 headline), N=1 with per-namespace
# watches (discover scope, the shard path with one shard) and N=2/N=4
# (torchrun, gloo; one cluster fixture, exactly-once verify sink).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ nproc; lscpu | head -25; free -g; } > gpurun_out/host.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest -m gpu failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --json-out gpurun_out/bench_n1.json > gpurun_out/bench_n1.log 2>&1 || { echo "bench n1 failed"; tail -30 gpurun_out/bench_n1.log; exit 1; }
cat gpurun_out/bench_n1.json
timeout -k 10 300 python bench.py --watch-scope discover --ref-events 0 --json-out gpurun_out/bench_n1_discover.json > gpurun_out/bench_n1_discover.log 2>&1 || { echo "bench n1 discover failed"; tail -30 gpurun_out/bench_n1_discover.log; exit 1; }
cat gpurun_out/bench_n1_discover.json
for n in ${SHARD_NS:-2 4}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29400 + n)) bench.py --gpus $n --ref-events 0 --json-out gpurun_out/bench_n$n.json > gpurun_out/bench_n$n.log 2>&1 || { echo "bench n$n failed"; tail -30 gpurun_out/bench_n$n.log; exit 1; }
  cat gpurun_out/bench_n$n.json
done
echo done
