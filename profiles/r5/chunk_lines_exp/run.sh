# A/B: the current tree vs exp_ff (chunks taken whole as lines), interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r5ck
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
run() {  # tree tag extra-args
  (cd $GRAFT_REPO_ROOT/$1 && timeout -k 10 240 $B $3 --json-out $O/$2.json > $O/$2.out 2> $O/$2.err)
}
run . cl_main_a "" && run exp_ff cl_exp_a "" &&
run . ns64_main_a "--watch-scope discover --namespaces 64" && run exp_ff ns64_exp_a "--watch-scope discover --namespaces 64" &&
run exp_ff cl_exp_b "" && run . cl_main_b "" &&
run exp_ff ns64_exp_b "--watch-scope discover --namespaces 64" && run . ns64_main_b "--watch-scope discover --namespaces 64"
