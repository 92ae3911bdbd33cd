# torchrun N=2 on one box with the current defaults (gloo, CPU ranks; the GPU is not used)
set -o pipefail
O=gpurun_out/${1:-r6n2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out $O/n2.json > $O/n2.out 2> $O/n2.err
