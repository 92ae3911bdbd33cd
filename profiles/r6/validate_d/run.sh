# The round-end tiers on one box: the host-tier tests (pytest -m gpu), smoke(), the driver's
# bench command (twice), and a rocprofv3 kernel trace of a short bench.
# usage: bash scripts/boxruns/validate.sh TAG
set -o pipefail
T=${1:-x}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench_detail.json > $O/bench.out 2> $O/bench.err &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench_detail_2.json > $O/bench_2.out 2> $O/bench_2.err &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --apart off --staging off --ref-events 0 --latency-seconds 2 --latency-seconds-high 2 > $O/rocprof.log 2>&1
