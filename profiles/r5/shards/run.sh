# round 5: the sharded shape with the fixture's namespace rings — discover mode
# at 64 and 1,000 namespaces (one rank), then torchrun N=2 and N=4 (gloo, CPU
# ranks; the GPU is not used) with per-rank stage CPU in the record
set -o pipefail
mkdir -p gpurun_out/r5d
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 $B --watch-scope discover --namespaces 64 --json-out gpurun_out/r5d/ns64.json > gpurun_out/r5d/ns64.out 2> gpurun_out/r5d/ns64.err &&
timeout -k 10 300 $B --watch-scope discover --namespaces 1000 --json-out gpurun_out/r5d/ns1000.json > gpurun_out/r5d/ns1000.out 2> gpurun_out/r5d/ns1000.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out gpurun_out/r5d/n2.json > gpurun_out/r5d/n2.out 2> gpurun_out/r5d/n2.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out gpurun_out/r5d/n4.json > gpurun_out/r5d/n4.out 2> gpurun_out/r5d/n4.err
