# round 5: where one https cluster watch is bound — the fixture's sealing threads vs the watcher's opening threads
set -o pipefail
O=gpurun_out/r5tb
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --api-tls"
timeout -k 10 240 $B --json-out $O/base.json > $O/base.out 2> $O/base.err &&
timeout -k 10 240 $B --fixture-tls-threads 6 --json-out $O/fx6.json > $O/fx6.out 2> $O/fx6.err &&
timeout -k 10 240 $B --tls-threads 5 --json-out $O/w5.json > $O/w5.out 2> $O/w5.err &&
timeout -k 10 240 $B --fixture-tls-threads 6 --tls-threads 5 --json-out $O/fx6w5.json > $O/fx6w5.out 2> $O/fx6w5.err &&
timeout -k 10 240 $B --fixture-tls-threads 1 --json-out $O/fx1.json > $O/fx1.out 2> $O/fx1.err
