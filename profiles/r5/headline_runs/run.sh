# round 5: the driver's exact command six times in one call (run-to-run spread on one box)
set -o pipefail
O=gpurun_out/r5runs
mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/run$i.json > $O/run$i.out 2> $O/run$i.err || exit $?
done
