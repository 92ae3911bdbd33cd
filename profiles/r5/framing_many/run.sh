# round 5: hub framing on/off with many watches (64 and 1,000 namespaces), interleaved
set -o pipefail
mkdir -p gpurun_out/r5j
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --watch-scope discover"
for r in a b; do
  timeout -k 10 240 $B --namespaces 64 --json-out gpurun_out/r5j/ns64_on_$r.json > gpurun_out/r5j/ns64_on_$r.out 2> gpurun_out/r5j/ns64_on_$r.err || exit 1
  timeout -k 10 240 $B --namespaces 64 --hub-framing off --json-out gpurun_out/r5j/ns64_off_$r.json > gpurun_out/r5j/ns64_off_$r.out 2> gpurun_out/r5j/ns64_off_$r.err || exit 1
done
timeout -k 10 300 $B --namespaces 1000 --json-out gpurun_out/r5j/ns1000_on.json > gpurun_out/r5j/ns1000_on.out 2> gpurun_out/r5j/ns1000_on.err &&
timeout -k 10 300 $B --namespaces 1000 --hub-framing off --json-out gpurun_out/r5j/ns1000_off.json > gpurun_out/r5j/ns1000_off.out 2> gpurun_out/r5j/ns1000_off.err
