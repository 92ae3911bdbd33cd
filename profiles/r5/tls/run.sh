set -o pipefail
mkdir -p gpurun_out/r5c
B="python3 bench.py --api-tls --steps 20 --warmup 5 --apart off --staging off --ref-events 0"
timeout -k 10 240 $B --json-out gpurun_out/r5c/tls_native.json > gpurun_out/r5c/tls_native.out 2> gpurun_out/r5c/tls_native.err &&
timeout -k 10 240 $B --tls-records openssl --json-out gpurun_out/r5c/tls_openssl.json > gpurun_out/r5c/tls_openssl.out 2> gpurun_out/r5c/tls_openssl.err &&
timeout -k 10 240 $B --watch-scope discover --namespaces 64 --json-out gpurun_out/r5c/tls_ns64.json > gpurun_out/r5c/tls_ns64.out 2> gpurun_out/r5c/tls_ns64.err &&
timeout -k 10 240 $B --fixture-tls python --tls-records openssl --json-out gpurun_out/r5c/tls_r4path.json > gpurun_out/r5c/tls_r4path.out 2> gpurun_out/r5c/tls_r4path.err
