# Launch knobs for the mid-size searches of an 8-GPU rank (N = 7): the owner's search
# (tools/small_search_probe.py cases) and a stopped rank's drain (--stop), through gpurun.
set -o pipefail
tag=${1:-mid}; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 -u tools/small_search_probe.py "$@" > $out/cases.json 2> $out/cases.err &&
timeout -k 10 300 python3 -u tools/small_search_probe.py --stop "$@" > $out/stop.json 2> $out/stop.err
