# round 5: current tree — https cluster watch (framing on the loop), torchrun N=2 and N=4, 1,000 namespaces
set -o pipefail
mkdir -p gpurun_out/r5l
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5"
timeout -k 10 240 $B --api-tls --json-out gpurun_out/r5l/tls.json > gpurun_out/r5l/tls.out 2> gpurun_out/r5l/tls.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out gpurun_out/r5l/n2.json > gpurun_out/r5l/n2.out 2> gpurun_out/r5l/n2.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 4 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out gpurun_out/r5l/n4.json > gpurun_out/r5l/n4.out 2> gpurun_out/r5l/n4.err &&
timeout -k 10 300 $B --watch-scope discover --namespaces 1000 --json-out gpurun_out/r5l/ns1000.json > gpurun_out/r5l/ns1000.out 2> gpurun_out/r5l/ns1000.err
