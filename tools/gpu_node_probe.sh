# Emulated G-GPU node time-to-secret (tools/node_probe.py) on one GPU, through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_node_probe.sh
set -o pipefail
mkdir -p gpurun_out/r03np
timeout -k 10 600 python3 -u tools/node_probe.py 3 ${1:-2,4,8} > gpurun_out/r03np/node_probe.json 2> gpurun_out/r03np/node_probe.err
