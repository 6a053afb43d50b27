# A/B of the launch tail: tail claims without a claim ahead, smaller / more tail claims.
set -o pipefail
mkdir -p gpurun_out/abtail
timeout -k 10 600 python3 tools/ab_variants.py abt/base.so abt/t0.so abt/t0c2.so abt/t0c2x4.so abt/c2.so > gpurun_out/abtail/ab.log 2>&1 && \
for v in base t0 t0c2 t0c2x4 c2; do
  DPOW_LIB_PATH=abx/tr_$v.so timeout -k 10 120 python3 tools/wave_trace_small.py > gpurun_out/abtail/trace_$v.json 2> gpurun_out/abtail/trace_$v.err || exit 1
done && \
for v in base t0c2 t0c2x4; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/node_probe.py 5 > gpurun_out/abtail/node_$v.json 2> gpurun_out/abtail/node_$v.err || exit 1
done
