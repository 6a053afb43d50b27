# The short-search launch knobs (tools/small_search_probe.py: the BASELINE cases, fresh
# nonces, or the stop latency of a rank) through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_small_probe.sh <tag> <mode: cases|random|stop> [bpc,min_chunk,poll_wb,cpw ...]
set -o pipefail
tag=$1; mode=$2; shift 2
mkdir -p gpurun_out/$tag
case $mode in
    cases) flag="" ;;
    *) flag="--$mode" ;;
esac
timeout -k 10 500 python3 -u tools/small_search_probe.py $flag "$@" > gpurun_out/$tag/$mode.json 2> gpurun_out/$tag/$mode.err
