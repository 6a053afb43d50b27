# A/B: workgroups per CU (6 default) for small launches / time-to-secret.
set -o pipefail
mkdir -p gpurun_out/abblocks
timeout -k 10 600 python3 tools/ab_variants.py abt/b6.so abt/b4.so abt/b3.so > gpurun_out/abblocks/ab.log 2>&1 && \
for v in b6 b4 b3; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/node_probe.py 5 > gpurun_out/abblocks/node_$v.json 2> gpurun_out/abblocks/node_$v.err || exit 1
done
