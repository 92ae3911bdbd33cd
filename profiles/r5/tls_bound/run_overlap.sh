# round 5: the fixture's https sends with patching overlapped with sealing (interleaved with the previous fixture)
set -o pipefail
O=gpurun_out/r5to
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --api-tls"
timeout -k 10 240 $B --json-out $O/new_a.json > $O/new_a.out 2> $O/new_a.err &&
timeout -k 10 240 $B --fixture-tls-threads 1 --json-out $O/new_fx1.json > $O/new_fx1.out 2> $O/new_fx1.err &&
timeout -k 10 240 $B --json-out $O/new_b.json > $O/new_b.out 2> $O/new_b.err
