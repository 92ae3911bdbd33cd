# the five BASELINE configurations (benchmarks.suite) and the latency-vs-load curves on the current tree
set -o pipefail
O=gpurun_out/${SUITE_OUT:-suite_latency}
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 420 python3 -m benchmarks.suite --out $O/suite.json > $O/suite.md 2> $O/suite.err &&
timeout -k 10 300 python3 -m benchmarks.latency_curve --profile staging --out $O/lat_staging.json > $O/lat_staging.md 2> $O/lat_staging.err &&
timeout -k 10 300 python3 -m benchmarks.latency_curve --profile production --out $O/lat_production.json > $O/lat_production.md 2> $O/lat_production.err
