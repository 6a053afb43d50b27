# Node-search check on a one-GPU box: the two-rank GPU node test, then 2- and 8-rank gloo
# rehearsals of the driver's N>1 bench path (all ranks on device 0).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_node.py -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_node.log 2>&1 && \
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --same-device --no-probe > gpurun_out/${TAG}_bench_n2_rehearsal.json 2> gpurun_out/${TAG}_bench_n2_rehearsal.err && \
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 2 --warmup 1 --backend gloo --same-device --no-probe > gpurun_out/${TAG}_bench_n8_rehearsal.json 2> gpurun_out/${TAG}_bench_n8_rehearsal.err
