# Short-search launch knobs on the BASELINE cases and over fresh nonces (tools/small_search_probe.py):
#   gpurun --timeout 600 -- bash tools/gpu_small_knobs.sh <tag> bpc,min_chunk,poll_wb,cpw ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u tools/small_search_probe.py "$@" > gpurun_out/$tag/cases.json 2> gpurun_out/$tag/cases.err &&
timeout -k 10 400 python3 -u tools/small_search_probe.py --random "$@" > gpurun_out/$tag/random.json 2> gpurun_out/$tag/random.err
