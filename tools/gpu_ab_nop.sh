set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 tools/ab_variants.py abt/nopbase.so abt/nopA1.so abt/nopA3.so abt/nopR1.so abt/nopB0.so > gpurun_out/r02_ab_nop.log 2>&1
