# Final-build evidence, part B, through gpurun: the layout check and sweep
# (tools/gpu_layouts.sh), a 3-minute parity soak (tests/soak/parity_soak.py) and an 8-rank
# rehearsal of the N > 1 bench path on one GPU (tools/gpu_rehearse_n8.sh), the emulated
# 2/4/8-GPU node (tools/node_probe.py).
#   gpurun --timeout 1200 -- bash tools/gpu_final_b.sh <tag>
set -o pipefail
tag=${1:-finalb}
out=gpurun_out/$tag
bash tools/gpu_layouts.sh $tag 34 2 &&
timeout -k 10 240 python3 -u tests/soak/parity_soak.py 180 7 > $out/parity_soak.json 2> $out/parity_soak.err &&
bash tools/gpu_rehearse_n8.sh $tag 8 &&
timeout -k 10 600 python3 -u tools/node_probe.py 3 > $out/node_probe.json 2> $out/node_probe.err
