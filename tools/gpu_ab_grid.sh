# A/B: fixed 6-per-CU grids (head) vs the short-launch grid policy + timer slack (new); then GPU tests.
set -o pipefail
mkdir -p gpurun_out/abgrid
timeout -k 10 600 python3 tools/ab_variants.py abt/head.so abt/new.so > gpurun_out/abgrid/ab.log 2>&1 && \
for v in head new; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/node_probe.py 5 > gpurun_out/abgrid/node_$v.json 2> gpurun_out/abgrid/node_$v.err || exit 1
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/launch_size_probe.py > gpurun_out/abgrid/size_$v.json 2> gpurun_out/abgrid/size_$v.err || exit 1
done && \
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/abgrid/gpu_tests.log 2>&1
