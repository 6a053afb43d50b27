set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_node.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "node or bound" > gpurun_out/r02_gpu_tests_i.log 2>&1 && \
DPOW_NODE_ASYNC=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --same-device --no-probe > gpurun_out/r02_bench_n2_async.json 2> gpurun_out/r02_bench_n2_async.err && \
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --same-device --no-probe > gpurun_out/r02_bench_n2_sync.json 2> gpurun_out/r02_bench_n2_sync.err
