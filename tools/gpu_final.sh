# Round-end evidence on one GPU box: parity tests, bench, profile, sweeps, soak.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 300 python3 tools/partition_sweep.py > gpurun_out/${TAG}_partition_sweep.json 2> gpurun_out/${TAG}_partition_sweep.err && \
timeout -k 10 400 python3 tools/layout_sweep.py 34 3 > gpurun_out/${TAG}_layout_sweep.log 2>&1 && \
timeout -k 10 300 python3 tests/soak/parity_soak.py 150 23 > gpurun_out/${TAG}_parity_soak.json 2> gpurun_out/${TAG}_parity_soak.err && \
bash tools/profile_gpu.sh $TAG pmc > gpurun_out/${TAG}_prof.out 2>&1
