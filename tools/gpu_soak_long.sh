# Long parity soaks on one GPU box (random, segment-spanning, long-chunk modes).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02s}
SEED=${2:-41}
timeout -k 10 660 python3 tests/soak/parity_soak.py 600 $SEED > gpurun_out/${TAG}_soak.json 2> gpurun_out/${TAG}_soak.err && \
timeout -k 10 210 python3 tests/soak/parity_soak.py 150 $((SEED + 2)) span > gpurun_out/${TAG}_soak_span.json 2> gpurun_out/${TAG}_soak_span.err && \
timeout -k 10 210 python3 tests/soak/parity_soak.py 150 $((SEED + 6)) long > gpurun_out/${TAG}_soak_long.json 2> gpurun_out/${TAG}_soak_long.err
