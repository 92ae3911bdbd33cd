#!/usr/bin/env bash
# GPU-box pass on the final tree: https API server through the native reader
# (bench.py --api-tls), https clusterapi (--tls), then N=1/2/4 repeated for the
# scaling picture (streamed steps, per-rank front-ends).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/extra
mkdir -p $out
common="--ref-events 0 --latency-seconds 2 --latency-seconds-high 2"
for v in api-tls tls; do
  timeout -k 10 300 python bench.py $common --$v --json-out $out/$v.json > $out/$v.log 2>&1 || { echo "$v failed"; tail -20 $out/$v.log; exit 1; }
  python -c "import json; d=json.load(open('$out/$v.json')); print('$v', round(d['value']), d['config']['api_server'], d['config']['clusterapi'], d['p50_latency_ms'], d['verify']['exactly_once'], d['cpu_util_rank0'])"
done
for rep in 1 2; do
  for n in 1 2 4; do
    if [ $n = 1 ]; then
      timeout -k 10 300 python bench.py $common --json-out $out/n1_r$rep.json > $out/n1_r$rep.log 2>&1 || { echo "n1 failed"; tail -20 $out/n1_r$rep.log; exit 1; }
    else
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29400 + n)) bench.py --gpus $n $common --json-out $out/n${n}_r$rep.json > $out/n${n}_r$rep.log 2>&1 || { echo "n$n failed"; tail -20 $out/n${n}_r$rep.log; exit 1; }
    fi
    python -c "import json; d=json.load(open('$out/n${n}_r$rep.json')); print('n$n r$rep', round(d['value']), round(d['value']/d['n_gpus']), d['verify']['exactly_once'], d['cpu_util_rank0'])"
  done
done
echo done
