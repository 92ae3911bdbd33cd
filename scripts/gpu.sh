#!/usr/bin/env bash
# GPU-box runner (through `gpurun`): scripts/gpu.sh <out-dir> <step>...
#
# Steps run in order, each under its own time limit; the first failure ends
# the run (no GPU step runs after a failed or timed-out one).
#   smoke                       __graft_entry__.smoke()
#   tests                       pytest -m gpu (host tier)
#   bench:<label>[:<args>]      bench.py, extra args comma-separated (bench:apart:--fixture-placement,apart)
#   benchso:<label>:<so>[,<args>]  bench.py with another build of the extension (A/B of native changes)
#   shards:<N>[:<args>]         bench.py --gpus N under torch.distributed.run (gloo barrier)
#   storm:<label>[:<args>]      benchmarks/relist_storm.py
#   suite                       benchmarks/suite.py (the five BASELINE configs)
#   module:<label>:<module>[:<args>]   python -m <module> <args> (any benchmark)
#   rocprof                     rocprofv3 kernel trace + stats of a short bench (expected: no kernels)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:?out dir}
shift
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
{ date; nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; git rev-parse HEAD 2>/dev/null;
  echo "thp $(cat /sys/kernel/mm/transparent_hugepage/enabled) defrag $(cat /sys/kernel/mm/transparent_hugepage/defrag)"; } > "$OUT/host.txt" 2>&1

fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }

for step in "$@"; do
  IFS=':' read -r kind label rest <<< "$step"
  args=()
  if [ -n "$rest" ]; then IFS=',' read -r -a args <<< "$rest"; fi
  case "$kind" in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail smoke "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > "$OUT/pytest_gpu.log" 2>&1 || fail tests "$OUT/pytest_gpu.log"
      tail -1 "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 900 python bench.py --json-out "$OUT/bench_$label.json" "${args[@]}" > "$OUT/bench_$label.log" 2>&1 \
        || fail "bench $label" "$OUT/bench_$label.log"
      python - "$OUT/bench_$label.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rs = d.get("rate_series") or {}
st = d.get("staging") or {}
print(sys.argv[1], d["value"], "ms/step", d["ms_per_step"], "timed_s", round(d["ms_per_step"] * d["steps"] / 1e3, 2),
      "p50", d["p50_latency_ms"], "hi", {k: (d.get("latency_high_rate") or {}).get(k) for k in ("p50_ms", "p99_ms")},
      "exactly_once", (d.get("verify") or {}).get("exactly_once"),
      "rate min/med", rs.get("min_over_median"), "notified/s", d.get("notified_per_s"),
      "cpu", d.get("cpu_util_rank0"), "cgroup", d.get("cgroup_cpu_timed"),
      "staging", {k: st.get(k) for k in ("every_event_notified_per_s", "p50_latency_ms", "p99_latency_ms",
                                         "exactly_once", "cgroup_latency")} if st else None)
PY
      ;;
    benchso)
      so=${args[0]}
      K8S_WATCHER_KWCORE_SO=$so timeout -k 10 900 python bench.py --json-out "$OUT/bench_$label.json" "${args[@]:1}" \
        > "$OUT/bench_$label.log" 2>&1 || fail "bench $label" "$OUT/bench_$label.log"
      python -c "import json; d=json.load(open('$OUT/bench_$label.json')); print('$label', d['value'], d['verify']['exactly_once'])" ;;
    shards)
      n=$label
      tag=n$n
      k=2
      while [ -e "$OUT/bench_$tag.json" ]; do tag=n${n}_$k; k=$((k + 1)); done  # repeats of one N keep their files
      timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
        --master-port $((29400 + n)) bench.py --gpus "$n" --ref-events 0 --json-out "$OUT/bench_$tag.json" "${args[@]}" \
        > "$OUT/bench_$tag.log" 2>&1 || fail "shards $n" "$OUT/bench_$tag.log"
      python -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', d['value'], d['verify']['exactly_once'], d.get('cgroup_cpu_timed'), [p['elapsed'] for p in d['per_rank']])" ;;
    storm)
      timeout -k 10 900 python benchmarks/relist_storm.py --json-out "$OUT/storm_$label.json" "${args[@]}" \
        > "$OUT/storm_$label.log" 2>&1 || fail "storm $label" "$OUT/storm_$label.log"
      python -c "import json; d=json.load(open('$OUT/storm_$label.json')); print('storm $label', json.dumps({k: d[k] for k in ('initial', 'storm')}))" ;;
    module)
      mod=${args[0]}
      timeout -k 10 1200 python -m "$mod" "${args[@]:1}" > "$OUT/$label.log" 2>&1 || fail "$label" "$OUT/$label.log"
      tail -5 "$OUT/$label.log" ;;
    suite)
      timeout -k 10 900 python -m benchmarks.suite --out "$OUT/suite.json" > "$OUT/suite.md" 2> "$OUT/suite.err" \
        || fail suite "$OUT/suite.err"
      cat "$OUT/suite.md" ;;
    rocprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/rocprof" \
        -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --ref-events 0 --latency-seconds 2 \
        --latency-seconds-high 2) > "$OUT/rocprof.log" 2>&1 || fail rocprof "$OUT/rocprof.log"
      find "$OUT/rocprof" -name "*stats*" | head ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
