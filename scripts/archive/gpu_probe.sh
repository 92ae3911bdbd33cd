#!/usr/bin/env bash
# GPU-box pass: bench.py N=1 with the event-loop probe (native time split /
# decode wait / apply / notifier I/O) and the step phase breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
for v in ${PROBE_VARIANTS:-base}; do
  case $v in
    base) extra="" ;;
    dt0) extra="--decode-threads 0" ;;
    dt5) extra="--decode-threads 5" ;;
    nonotify) extra=""; export BENCH_NO_NOTIFY=1 ;;
    *) extra="$v" ;;
  esac
  timeout -k 10 300 python bench.py --ref-events 0 --latency-seconds 2 --latency-seconds-high 2 --probe $extra --json-out gpurun_out/probe/$v.json > gpurun_out/probe/$v.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/probe/$v.log; exit 1; }
  unset BENCH_NO_NOTIFY
  python - gpurun_out/probe/$v.json "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); p = d.get("loop_probe_rank0") or {}
n = max(1, p.get("lines", 1))
per = {k: round(p[k] / n, 1) for k in ("split_ns", "wait_ns", "apply_ns", "run_ns") if k in p}
print(f"{sys.argv[2]:10s} {d['value']:>12,.0f} ev/s phases {d['step_phases_ms_rank0']} cpu {d['cpu_util_rank0']} "
      f"per-line ns {per} notifier_io {p.get('notifier_io_ns', 0) / n:.1f} ns/line over {p.get('notifier_io_calls')} calls, "
      f"loop cpu {p.get('loop_cpu_ns', 0) / n:.1f} ns/line, lines/call {n / max(1, p.get('calls', 1)):.0f}", flush=True)
PY
done
echo done
