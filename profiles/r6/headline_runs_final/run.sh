# the driver's exact command N times in one call (the round's headline spread on one box)
set -o pipefail
O=gpurun_out/${1:-r6hl}; N=${2:-4}
mkdir -p $O
for i in $(seq 1 $N); do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/run$i.json > $O/run$i.out 2> $O/run$i.err || exit $?
done
