# tools/gpu_node_ab.sh, then the node wave traces of diagnostic builds (tools/wave_trace_node.py;
# TRACE_LIBS: space-separated libraries, default distpow/libdpow_trace.so):
#   gpurun --timeout 1500 -- bash tools/gpu_node_ab_trace.sh <tag> <runs> name=lib.so[,VAR=value...] ...
set -o pipefail
tag=$1
bash tools/gpu_node_ab.sh "$@" || exit $?
for lib in ${TRACE_LIBS:-distributed-proof-of-work_amd/distpow/libdpow_trace.so}; do
    DPOW_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/wave_trace_node.py \
        > gpurun_out/$tag/wave_trace_node_$(basename $lib .so).json 2> gpurun_out/$tag/wave_trace_node_$(basename $lib .so).err || exit $?
done
