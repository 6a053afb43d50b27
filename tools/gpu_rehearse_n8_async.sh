# Rehearse N=8 with the asynchronous node search (DPOW_NODE_ASYNC=1): 8 gloo ranks on device 0.
set -o pipefail
mkdir -p gpurun_out
DPOW_NODE_ASYNC=1 timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 8 --steps 2 --warmup 1 --backend gloo --same-device --no-probe > gpurun_out/r02_bench_n8_async_rehearsal.json 2> gpurun_out/r02_bench_n8_async_rehearsal.err
