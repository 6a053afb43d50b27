# Rehearse the driver's N>1 bench path on a one-GPU box: N gloo ranks on device 0 (the
# node board and its vote are shared memory, as on an 8-GPU node; the sweep's per-step
# all-reduce runs on gloo here instead of RCCL).
#   gpurun --timeout 900 -- bash tools/gpu_rehearse_n8.sh <tag> [N]
set -o pipefail
tag=${1:-rehearse}; n=${2:-8}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus $n --steps 2 --warmup 1 --backend gloo --same-device --no-probe > gpurun_out/$tag/bench_n$n.json 2> gpurun_out/$tag/bench_n$n.err
