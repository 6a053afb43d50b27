# Final-build evidence, part C: parity soaks (random, span, long) of the final build.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02i}
timeout -k 10 360 python3 tests/soak/parity_soak.py 300 53 > gpurun_out/${TAG}_parity_soak.json 2> gpurun_out/${TAG}_parity_soak.err && \
timeout -k 10 180 python3 tests/soak/parity_soak.py 120 59 span > gpurun_out/${TAG}_parity_soak_span.json 2> gpurun_out/${TAG}_parity_soak_span.err && \
timeout -k 10 180 python3 tests/soak/parity_soak.py 120 61 long > gpurun_out/${TAG}_parity_soak_long.json 2> gpurun_out/${TAG}_parity_soak_long.err && \
DPOW_NODE_PROBE=1 timeout -k 10 500 python3 tools/node_probe.py 3 > gpurun_out/${TAG}_node_probe.json 2> gpurun_out/${TAG}_node_probe.err
