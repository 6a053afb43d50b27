# A/B: chunk cap for launches with an expected early hit (DPOW_HIT_CLAIMS 0 = off / 16 / 32 / 64).
set -o pipefail
mkdir -p gpurun_out/abhit
timeout -k 10 600 python3 tools/ab_variants.py abt/hit0.so abt/hit16.so abt/hit32.so abt/hit64.so > gpurun_out/abhit/ab.log 2>&1 && \
for v in hit0 hit32; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 300 python3 tools/node_probe.py 3 > gpurun_out/abhit/node_$v.json 2> gpurun_out/abhit/node_$v.err || exit 1
done
