# The emulated 8-GPU node (tools/node_probe.py) and the stop latency of a rank
# (tools/small_search_probe.py --stop) on this build and, if present, A/B builds abx/*.so:
#   gpurun --timeout 900 -- bash tools/gpu_node_stop.sh <tag>
set -o pipefail
tag=${1:-nodestop}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u tools/node_probe.py 3 8 > $out/node_probe.json 2> $out/node_probe.err &&
timeout -k 10 200 python3 -u tools/small_search_probe.py --stop > $out/stop.json 2> $out/stop.err || exit $?
for lib in abx/libdpow_ws*.so; do
    [ -f "$lib" ] || continue
    b=$(basename $lib .so)
    DPOW_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/small_search_probe.py --stop > $out/stop_$b.json 2> $out/stop_$b.err || exit $?
done
