set -o pipefail
mkdir -p gpurun_out
{
echo "nproc=$(nproc)"; python3 -c 'import os; print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))'
cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"
lscpu | grep -E "Model name|Socket|Core|Thread|^CPU\(s\)"
grep -o -w -E "avx2|avx512f" /proc/cpuinfo | sort | uniq -c
} > gpurun_out/box_probe.txt 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_start.log 2>&1
