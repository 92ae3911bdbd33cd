# A/B of two builds of _kwcore on the same tree, interleaved: the in-tree .so (main) against
# abexp/_kwcore*.so (exp), loaded through $K8S_WATCHER_KWCORE_SO.
# usage: bash scripts/boxruns/ab_so.sh TAG PAIRS [extra bench args...]
set -o pipefail
T=${1:-x}; P=${2:-2}; shift 2
O=gpurun_out/ab_$T
mkdir -p $O
EXP=$(ls $PWD/abexp/_kwcore*.so)
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
for i in $(seq 1 $P); do
  if [ $((i % 2)) = 1 ]; then order="main exp"; else order="exp main"; fi
  for v in $order; do
    if [ $v = exp ]; then export K8S_WATCHER_KWCORE_SO=$EXP; else unset K8S_WATCHER_KWCORE_SO; fi
    timeout -k 10 300 $B "$@" --json-out $O/${v}_$i.json > $O/${v}_$i.out 2> $O/${v}_$i.err || exit $?
  done
done
