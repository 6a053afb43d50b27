# 6- and 7-byte chunks (k up to DPOW_K_LIMIT = 2^55 - 1): GPU tests, then a long-chunk soak.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02_long}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 tests/soak/parity_soak.py 120 55 long > gpurun_out/${TAG}_parity_soak.json 2> gpurun_out/${TAG}_parity_soak.err && \
timeout -k 10 300 python3 tests/soak/parity_soak.py 60 56 > gpurun_out/${TAG}_parity_soak_mixed.json 2> gpurun_out/${TAG}_parity_soak_mixed.err
