# round 5: ring-based TLS reader; hub framing on/off A/B on the cluster watch (loop has headroom since the concurrent tail)
set -o pipefail
mkdir -p gpurun_out/r5i
for args in "--client-threads 3 --server-threads 3" "--client-threads 5 --server-threads 5"; do
  timeout -k 10 120 python3 -m benchmarks.tls_throughput --gb 8 $args >> gpurun_out/r5i/tp.jsonl 2>> gpurun_out/r5i/tp.err || exit 1
done
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
timeout -k 10 240 $B --api-tls --json-out gpurun_out/r5i/tls.json > gpurun_out/r5i/tls.out 2> gpurun_out/r5i/tls.err &&
timeout -k 10 240 $B --json-out gpurun_out/r5i/fr_on_a.json > gpurun_out/r5i/fr_on_a.out 2> gpurun_out/r5i/fr_on_a.err &&
timeout -k 10 240 $B --hub-framing off --json-out gpurun_out/r5i/fr_off_a.json > gpurun_out/r5i/fr_off_a.out 2> gpurun_out/r5i/fr_off_a.err &&
timeout -k 10 240 $B --json-out gpurun_out/r5i/fr_on_b.json > gpurun_out/r5i/fr_on_b.out 2> gpurun_out/r5i/fr_on_b.err &&
timeout -k 10 240 $B --hub-framing off --json-out gpurun_out/r5i/fr_off_b.json > gpurun_out/r5i/fr_off_b.out 2> gpurun_out/r5i/fr_off_b.err
