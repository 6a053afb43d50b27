# Short-search launch knobs over fresh nonces (tools/small_search_probe.py --random), through gpurun:
#   gpurun --timeout 600 -- bash tools/gpu_r04_small.sh <tag> bpc,min_chunk,poll_wb,cpw ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 500 python3 -u tools/small_search_probe.py --random "$@" > gpurun_out/$tag/small.json 2> gpurun_out/$tag/small.err
