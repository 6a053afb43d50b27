# A/B: claim-ahead atomic waited at once (head) vs read after the chunk (defer), chunk 32 vs 16.
set -o pipefail
mkdir -p gpurun_out/abdefer
timeout -k 10 600 python3 tools/ab_variants.py abt/head.so abt/defer.so abt/defer_c16.so > gpurun_out/abdefer/ab.log 2>&1 && \
for v in head defer; do
  DPOW_LIB_PATH=abx/tr_$v.so timeout -k 10 120 python3 tools/wave_trace_small.py > gpurun_out/abdefer/trace_$v.json 2> gpurun_out/abdefer/trace_$v.err || exit 1
done && \
for v in head defer defer_c16; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/node_probe.py 5 > gpurun_out/abdefer/node_$v.json 2> gpurun_out/abdefer/node_$v.err || exit 1
done
