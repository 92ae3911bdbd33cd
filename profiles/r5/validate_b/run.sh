# the driver's own commands on the current tree: bench (exact driver shape, twice), host-tier tests, smoke, rocprof
set -o pipefail
O=gpurun_out/${VALIDATE_OUT:-validate}
mkdir -p $O
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench_detail.json > $O/bench.out 2> $O/bench.err &&
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench_detail_2.json > $O/bench_2.out 2> $O/bench_2.err &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rocprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --apart off --staging off --ref-events 0 --latency-seconds 2 --latency-seconds-high 2 > $GRAFT_REPO_ROOT/$O/rocprof.log 2>&1)
