# round 5: one vs two reader-hub threads with one pod watch per namespace (interleaved)
set -o pipefail
O=gpurun_out/r5rt
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --watch-scope discover"
timeout -k 10 240 $B --namespaces 64 --reader-threads 1 --json-out $O/ns64_r1_a.json > $O/ns64_r1_a.out 2> $O/ns64_r1_a.err &&
timeout -k 10 240 $B --namespaces 64 --reader-threads 2 --json-out $O/ns64_r2_a.json > $O/ns64_r2_a.out 2> $O/ns64_r2_a.err &&
timeout -k 10 240 $B --namespaces 64 --reader-threads 1 --json-out $O/ns64_r1_b.json > $O/ns64_r1_b.out 2> $O/ns64_r1_b.err &&
timeout -k 10 240 $B --namespaces 64 --reader-threads 2 --json-out $O/ns64_r2_b.json > $O/ns64_r2_b.out 2> $O/ns64_r2_b.err &&
timeout -k 10 300 $B --namespaces 1000 --reader-threads 1 --json-out $O/ns1000_r1.json > $O/ns1000_r1.out 2> $O/ns1000_r1.err &&
timeout -k 10 300 $B --namespaces 1000 --reader-threads 2 --json-out $O/ns1000_r2.json > $O/ns1000_r2.out 2> $O/ns1000_r2.err &&
timeout -k 10 240 $B --namespaces 64 --api-tls --reader-threads 2 --json-out $O/tls_ns64_r2.json > $O/tls_ns64_r2.out 2> $O/tls_ns64_r2.err
