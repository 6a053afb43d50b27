# GPU check plus the node emulation (tools/gpu_check.sh, then tools/node_probe.py) and,
# with extra arguments, the short-search knob probe (tools/small_search_probe.py), through gpurun:
#   gpurun --timeout 1200 -- bash tools/gpu_evidence.sh <tag> [bpc,min_chunk,poll_wb,cpw ...]
set -o pipefail
tag=${1:-ev}; shift
bash tools/gpu_check.sh $tag &&
timeout -k 10 600 python3 -u tools/node_probe.py 3 > gpurun_out/$tag/node_probe.json 2> gpurun_out/$tag/node_probe.err &&
if [ $# -gt 0 ]; then
    timeout -k 10 300 python3 -u tools/small_search_probe.py "$@" > gpurun_out/$tag/small.json 2> gpurun_out/$tag/small.err
fi
