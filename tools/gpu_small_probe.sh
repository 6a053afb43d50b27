# GPU tests, then the short-search launch knobs (tools/small_search_probe.py: the BASELINE
# cases, then fresh nonces), through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_small_probe.sh <tag> [bpc,min_chunk,poll_wb ...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -1 gpurun_out/$tag/pytest.log
timeout -k 10 300 python3 -u tools/small_search_probe.py "$@" > gpurun_out/$tag/small.json 2> gpurun_out/$tag/small.err &&
timeout -k 10 500 python3 -u tools/small_search_probe.py --random "$@" > gpurun_out/$tag/random.json 2> gpurun_out/$tag/random.err
