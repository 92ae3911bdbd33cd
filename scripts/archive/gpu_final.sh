#!/usr/bin/env bash
# GPU-box pass on the final tree: smoke, host-tier tests, headline bench x3
# (default flags, as the driver runs it), N=2 and N=4 shard rehearsals, and
# the five-config suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { echo "pytest -m gpu failed"; tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --json-out gpurun_out/final/bench_n1_$i.json > gpurun_out/final/bench_n1_$i.log 2>&1 || { echo "bench $i failed"; tail -30 gpurun_out/final/bench_n1_$i.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/final/bench_n1_$i.json')); print('n1', d['value'], d['vs_baseline'], d['p50_latency_ms'], d['latency_high_rate']['p50_ms'], d['verify']['exactly_once'], d['cpu_util_rank0'])"
done
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29400 + n)) bench.py --gpus $n --ref-events 0 --json-out gpurun_out/final/bench_n$n.json > gpurun_out/final/bench_n$n.log 2>&1 || { echo "bench n$n failed"; tail -30 gpurun_out/final/bench_n$n.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/final/bench_n$n.json')); print('n$n', d['value'], d['p50_latency_ms'], d['verify']['exactly_once'], [p['elapsed'] for p in d['per_rank']])"
done
timeout -k 10 900 python -m benchmarks.suite --out gpurun_out/final/suite.json > gpurun_out/final/suite.md 2> gpurun_out/final/suite.err || { echo "suite failed"; tail -30 gpurun_out/final/suite.err; exit 1; }
cat gpurun_out/final/suite.md
echo done
