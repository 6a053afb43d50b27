# Stop-signal latency breakdown (tools/stop_latency.py) under rocprofv3, through gpurun.
set -o pipefail
tag=${1:-stop}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 tools/stop_latency.py > $out/stop.json 2> $out/stop.err &&
DPOW_DIAG_POLL_WB=4 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/trace4 -o run -- python3 tools/stop_latency.py > $out/stop4.json 2> $out/stop4.err
