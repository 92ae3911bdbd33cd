# The sharded shape on one box: discover mode at 64 namespaces (one rank), then torchrun N=2 and
# N=4 (gloo, CPU ranks; the GPU is not used), per-rank stage CPU in the record.
set -o pipefail
O=gpurun_out/${1:-r6sh}
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 $B --watch-scope discover --namespaces 64 --json-out $O/ns64.json > $O/ns64.out 2> $O/ns64.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out $O/n2.json > $O/n2.out 2> $O/n2.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out $O/n4.json > $O/n4.out 2> $O/n4.err
