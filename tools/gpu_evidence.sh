set -o pipefail
bash tools/profile_gpu.sh r03 pmc > gpurun_out/prof_r03.list 2>&1 &&
bash tools/gpu_node_probe.sh r03probe
