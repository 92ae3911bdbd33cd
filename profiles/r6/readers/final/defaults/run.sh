# round 6: the multi-scope hub defaults (two readers on a 12+ CPU share, 8 MiB read-ahead) against
# the old ones (one reader, the whole pool) at 64 and 1,000 namespace watches, and torchrun N=4
set -o pipefail
O=gpurun_out/${1:-r6md}
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
OLD="--set watcher.watch_reader_max_bytes=268435456"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 $B --watch-scope discover --namespaces 64 --json-out $O/1_ns64_new.json > $O/1_ns64_new.out 2> $O/1_ns64_new.err &&
BENCH_HUB_READERS=1 timeout -k 10 300 $B --watch-scope discover --namespaces 64 $OLD --json-out $O/2_ns64_old.json > $O/2_ns64_old.out 2> $O/2_ns64_old.err &&
BENCH_HUB_READERS=1 timeout -k 10 300 $B --watch-scope discover --namespaces 1000 $OLD --json-out $O/3_ns1000_old.json > $O/3_ns1000_old.out 2> $O/3_ns1000_old.err &&
timeout -k 10 300 $B --watch-scope discover --namespaces 1000 --json-out $O/4_ns1000_new.json > $O/4_ns1000_new.out 2> $O/4_ns1000_new.err &&
timeout -k 10 300 $B --watch-scope discover --namespaces 64 --json-out $O/5_ns64_new.json > $O/5_ns64_new.out 2> $O/5_ns64_new.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out $O/6_n4_new.json > $O/6_n4_new.out 2> $O/6_n4_new.err
