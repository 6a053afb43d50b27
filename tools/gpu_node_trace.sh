# Emulated 8-GPU node (tools/node_probe.py, G8 only) on the current build, then the per-wave
# timelines of its ranks on the diagnostic build (tools/wave_trace_node.py), through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_node_trace.sh <tag>
set -o pipefail
tag=${1:-nodetrace}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u tools/node_probe.py 3 8 > $out/node_probe.json 2> $out/node_probe.err &&
DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so timeout -k 10 300 \
    python3 -u tools/wave_trace_node.py > $out/wave_trace_node.json 2> $out/wave_trace_node.err
