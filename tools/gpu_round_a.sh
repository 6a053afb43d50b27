set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not n10" > gpurun_out/r02_gpu_tests_a.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python3 tools/partition_sweep.py > gpurun_out/r02_partition_a.json 2> gpurun_out/r02_partition_a.err && \
timeout -k 10 600 python3 bench.py --steps 5 --warmup 1 > gpurun_out/r02_bench_a.json 2> gpurun_out/r02_bench_a.err
