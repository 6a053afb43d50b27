# Final-build evidence, part B: layout sweep and the parity soaks (random, span, long).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02f}
timeout -k 10 420 python3 tools/layout_sweep.py 34 3 > gpurun_out/${TAG}_layout_sweep.log 2>&1 && \
timeout -k 10 240 python3 tests/soak/parity_soak.py 180 29 > gpurun_out/${TAG}_parity_soak.json 2> gpurun_out/${TAG}_parity_soak.err && \
timeout -k 10 120 python3 tests/soak/parity_soak.py 75 31 span > gpurun_out/${TAG}_parity_soak_span.json 2> gpurun_out/${TAG}_parity_soak_span.err && \
timeout -k 10 120 python3 tests/soak/parity_soak.py 75 37 long > gpurun_out/${TAG}_parity_soak_long.json 2> gpurun_out/${TAG}_parity_soak_long.err
