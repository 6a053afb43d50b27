# Final-build evidence, part A: GPU tests, the driver's default bench, a 20-step bench,
# the rocprofv3 profile (kernel trace + PMC passes) and the partition sweep.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02f}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_driver_bench.json 2> gpurun_out/${TAG}_driver_bench.err && \
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
bash tools/profile_gpu.sh $TAG pmc > gpurun_out/${TAG}_prof.out 2>&1 && \
timeout -k 10 300 python3 tools/partition_sweep.py > gpurun_out/${TAG}_partition_sweep.json 2> gpurun_out/${TAG}_partition_sweep.err
