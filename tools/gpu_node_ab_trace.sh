# tools/gpu_node_ab.sh, then the node wave traces of the diagnostic build (tools/wave_trace_node.py):
#   gpurun --timeout 1500 -- bash tools/gpu_node_ab_trace.sh <tag> <runs> name=lib.so[,VAR=value...] ...
set -o pipefail
tag=$1
bash tools/gpu_node_ab.sh "$@" &&
DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so timeout -k 10 300 \
    python3 -u tools/wave_trace_node.py > gpurun_out/$tag/wave_trace_node.json 2> gpurun_out/$tag/wave_trace_node.err
