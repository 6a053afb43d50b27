# Long parity soaks on one GPU box (random, segment-spanning, long-chunk modes).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02s}
timeout -k 10 480 python3 tests/soak/parity_soak.py 420 41 > gpurun_out/${TAG}_soak.json 2> gpurun_out/${TAG}_soak.err && \
timeout -k 10 240 python3 tests/soak/parity_soak.py 180 43 span > gpurun_out/${TAG}_soak_span.json 2> gpurun_out/${TAG}_soak_span.err && \
timeout -k 10 240 python3 tests/soak/parity_soak.py 180 47 long > gpurun_out/${TAG}_soak_long.json 2> gpurun_out/${TAG}_soak_long.err
