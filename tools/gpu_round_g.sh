set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_g.log 2>&1 && \
timeout -k 10 400 python3 tools/layout_sweep.py 34 3 > gpurun_out/r02_layout_sweep_g.log 2>&1
