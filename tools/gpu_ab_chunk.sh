set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ab_variants.py abt/chunk32.so abt/chunk64.so > gpurun_out/r02_ab_chunk.log 2>&1
