# round 5: concurrent tail (loop-bound shapes) + TLS fixture batching
set -o pipefail
mkdir -p gpurun_out/r5f
B="python3 bench.py --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --probe"
timeout -k 10 240 $B --watch-scope discover --namespaces 64 --json-out gpurun_out/r5f/ns64.json > gpurun_out/r5f/ns64.out 2> gpurun_out/r5f/ns64.err &&
timeout -k 10 240 $B --json-out gpurun_out/r5f/cluster.json > gpurun_out/r5f/cluster.out 2> gpurun_out/r5f/cluster.err &&
timeout -k 10 240 $B --api-tls --json-out gpurun_out/r5f/tls.json > gpurun_out/r5f/tls.out 2> gpurun_out/r5f/tls.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 --apart off --staging off --ref-events 0 --latency-seconds 5 --latency-seconds-high 5 --json-out gpurun_out/r5f/n2.json > gpurun_out/r5f/n2.out 2> gpurun_out/r5f/n2.err
