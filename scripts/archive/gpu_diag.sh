#!/usr/bin/env bash
# GPU-box pass: what bounds the config #4 headline. bench.py N=1 with its
# per-step phase breakdown (fixture send done / first event / last event /
# last acknowledgement) under variants that each remove one suspect.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/diag
common="--ref-events 0 --latency-seconds 2 --latency-seconds-high 2 --steps 10 --warmup 2"
run() {
  name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/diag/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/diag/$name.log; exit 1; }
  python - "$name" <<'EOF'
import json, sys
name = sys.argv[1]
line = [l for l in open(f"gpurun_out/diag/{name}.log") if l.startswith("{")][-1]
d = json.loads(line)
open(f"gpurun_out/diag/{name}.json", "w").write(line)
print(f"{name:14s} {d['value']:>12,.0f} ev/s  phases {d.get('step_phases_ms_rank0')}  cpu {d['cpu_util_rank0']}  other {d['cpu_other_threads_rank0'][:4]}", flush=True)
EOF
}
for rep in 1 2; do
  run base_$rep python bench.py $common
  run nonotify_$rep BENCH_NO_NOTIFY=1 python bench.py $common
  run noverify_$rep python bench.py $common --no-verify
  run dt5_$rep python bench.py $common --decode-threads 5
  run fw4_$rep python bench.py $common --fixture-workers 4 --sink-workers 8
done
echo done
