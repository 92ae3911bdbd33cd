# round 5: TLS record-layer throughput alone (benchmarks/tls_throughput.py) + OpenSSL's AES-GCM speed
set -o pipefail
mkdir -p gpurun_out/r5g
( timeout -k 5 60 openssl speed -seconds 2 -bytes 16384 -evp aes-128-gcm > gpurun_out/r5g/openssl_speed.txt 2>&1 || true )
for args in "--records openssl" "--client-threads 0 --server-threads 0" "--client-threads 3 --server-threads 3" "--client-threads 5 --server-threads 5" "--client-threads 3 --server-threads 3 --buf-mb 1"; do
  timeout -k 10 120 python3 -m benchmarks.tls_throughput --gb 8 $args >> gpurun_out/r5g/tp.jsonl 2>> gpurun_out/r5g/tp.err || exit 1
done
