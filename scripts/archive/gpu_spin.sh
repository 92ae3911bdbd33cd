#!/usr/bin/env bash
# GPU-box A/B of bench.py variants, interleaved, at N=1 (cluster watch) and
# N>1 (sharded, torchrun+gloo). Used for the decode-worker idle spin
# (watcher.decode_spin_us) and the stub sink's request loop (--sink-engine):
# the box's cgroup grants 16 CPUs of quota, so at N=4 the job is CPU-bound and
# cycles spent spinning or serving the mock clusterapi come out of the
# watchers' throughput.
#   VARIANTS="name=args;name=args"  REPS="1 2 3"  SHARD_NS="2 4"  REPS_N="1 2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-ab}
mkdir -p $out
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
dp = d.get("decode_pool_rank0") or {}
w = dp.get("workers") or []
print(f"{sys.argv[2]:22s} {d['value']:>12,.0f} ev/s  ms/step {d['ms_per_step']:7.2f}  cpu {d['cpu_util_rank0']}  "
      f"spin {[x['spin_frac'] for x in w]} sleep {[x['sleep_frac'] for x in w]} "
      f"exactly_once {(d.get('verify') or {}).get('exactly_once')}", flush=True)
p = d.get("loop_probe_rank0")
if p:
    n = max(1, p.get("lines", 1))
    print(f"{'':22s} probe ns/line: " + " ".join(f"{k[:-3]} {p[k] / n:.0f}" for k in ("split_ns", "wait_ns", "apply_ns", "run_ns") if k in p)
          + f" notifier_io {p.get('notifier_io_ns', 0) / n:.0f} loop_cpu {p.get('loop_cpu_ns', 0) / n:.0f} lines/call {n / max(1, p.get('calls', 1)):.0f}", flush=True)
PY
}
common="--ref-events 0 --latency-seconds 2 --latency-seconds-high 2"
IFS=';' read -ra VS <<< "${VARIANTS:-old=--decode-spin-us 60 --sink-engine python;new=}"
for rep in ${REPS-1 2 3}; do
  for v in "${VS[@]}"; do
    name=${v%%=*}; args=${v#*=}
    # "SO:<path> rest": this variant loads another build of the extension ($K8S_WATCHER_KWCORE_SO)
    if [[ $args == SO:* ]]; then so=${args%% *}; export K8S_WATCHER_KWCORE_SO=${so#SO:}; args=${args#"$so"}; else unset K8S_WATCHER_KWCORE_SO; fi
    tag=n1_${name}_r$rep
    timeout -k 10 240 python bench.py $common $args --json-out $out/$tag.json > $out/$tag.log 2>&1 || { echo "$tag failed"; tail -20 $out/$tag.log; exit 1; }
    summ $out/$tag.json $tag
  done
done
for rep in ${REPS_N-1 2}; do
  for n in ${SHARD_NS-2 4}; do
    for v in "${VS[@]}"; do
      name=${v%%=*}; args=${v#*=}
      tag=n${n}_${name}_r$rep
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29400 + n)) bench.py --gpus $n $common $args --json-out $out/$tag.json > $out/$tag.log 2>&1 || { echo "$tag failed"; tail -20 $out/$tag.log; exit 1; }
      summ $out/$tag.json $tag
    done
  done
done
echo done
