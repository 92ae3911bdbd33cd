# round 5: https API server after the fixture's pipelined TLS writer
set -o pipefail
mkdir -p gpurun_out/r5e
B="python3 bench.py --api-tls --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
timeout -k 10 240 $B --json-out gpurun_out/r5e/tls_native.json > gpurun_out/r5e/tls_native.out 2> gpurun_out/r5e/tls_native.err &&
timeout -k 10 240 $B --tls-threads 5 --fixture-tls-threads 5 --json-out gpurun_out/r5e/tls_native_t5.json > gpurun_out/r5e/tls_native_t5.out 2> gpurun_out/r5e/tls_native_t5.err &&
timeout -k 10 240 $B --watch-scope discover --namespaces 64 --json-out gpurun_out/r5e/tls_ns64.json > gpurun_out/r5e/tls_ns64.out 2> gpurun_out/r5e/tls_ns64.err
