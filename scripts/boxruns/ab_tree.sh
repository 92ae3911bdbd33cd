# A/B of two trees, interleaved: the current tree (main) against the tree in abtree/ (old), each
# with its own in-tree build. usage: bash scripts/boxruns/ab_tree.sh TAG PAIRS [extra bench args...]
set -o pipefail
T=${1:-x}; P=${2:-2}; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/abt_$T
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
for i in $(seq 1 $P); do
  if [ $((i % 2)) = 1 ]; then order="main old"; else order="old main"; fi
  for v in $order; do
    if [ $v = old ]; then d=$GRAFT_REPO_ROOT/abtree; else d=$GRAFT_REPO_ROOT; fi
    (cd $d && timeout -k 10 300 $B "$@" --json-out $O/${v}_$i.json > $O/${v}_$i.out 2> $O/${v}_$i.err) || exit $?
  done
done
