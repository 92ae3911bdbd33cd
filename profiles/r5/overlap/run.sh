# round 5: TLS reader with recv/decrypt overlap — raw record throughput, then the https bench
set -o pipefail
mkdir -p gpurun_out/r5h
for args in "--client-threads 3 --server-threads 3" "--client-threads 5 --server-threads 5"; do
  timeout -k 10 120 python3 -m benchmarks.tls_throughput --gb 8 $args >> gpurun_out/r5h/tp.jsonl 2>> gpurun_out/r5h/tp.err || exit 1
done
B="python3 bench.py --api-tls --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
timeout -k 10 240 $B --json-out gpurun_out/r5h/tls.json > gpurun_out/r5h/tls.out 2> gpurun_out/r5h/tls.err &&
timeout -k 10 240 $B --watch-scope discover --namespaces 64 --json-out gpurun_out/r5h/tls_ns64.json > gpurun_out/r5h/tls_ns64.out 2> gpurun_out/r5h/tls_ns64.err &&
P="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
timeout -k 10 300 $P --watch-scope discover --namespaces 1000 --json-out gpurun_out/r5h/ns1000.json > gpurun_out/r5h/ns1000.out 2> gpurun_out/r5h/ns1000.err &&
timeout -k 10 240 $P --watch-scope discover --namespaces 64 --json-out gpurun_out/r5h/ns64.json > gpurun_out/r5h/ns64.out 2> gpurun_out/r5h/ns64.err
