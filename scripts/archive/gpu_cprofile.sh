#!/usr/bin/env bash
# GPU-box pass: cProfile of the event-loop thread over the timed steps of the
# headline bench (BENCH_PROFILE), summarised by cumulative and own time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cprof
for scope in ${SCOPES:-cluster discover}; do
  BENCH_PROFILE=gpurun_out/cprof/$scope.prof timeout -k 10 300 python bench.py --ref-events 0 --latency-seconds 2 --latency-seconds-high 2 \
    --watch-scope $scope --json-out gpurun_out/cprof/$scope.json > gpurun_out/cprof/$scope.log 2>&1 || { echo "$scope failed"; tail -20 gpurun_out/cprof/$scope.log; exit 1; }
  python - gpurun_out/cprof/$scope.prof gpurun_out/cprof/$scope.json <<'PY' | tee gpurun_out/cprof/$scope.txt
import io, json, pstats, sys
d = json.load(open(sys.argv[2]))
print(f"{d['value']:,.0f} ev/s (under cProfile), events {d['per_rank'][0]['events']}")
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(sys.argv[1], stream=s).sort_stats(key).print_stats(22)
    print(s.getvalue())
PY
done
echo done
