# Node-path check through gpurun: GPU tests, stop-signal latency breakdown under rocprofv3
# (tools/stop_latency.py) and the emulated G-GPU node (tools/node_probe.py).
#   gpurun --timeout 900 -- bash tools/gpu_node_check.sh <tag>
set -o pipefail
tag=${1:-node}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 tools/stop_latency.py > $out/stop.json 2> $out/stop.err &&
timeout -k 10 600 python3 -u tools/node_probe.py 3 > $out/node_probe.json 2> $out/node_probe.err
