set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ab_variants.py abx/lead4.so abx/lead2.so abx/lead3.so > gpurun_out/r02_ab_lead.log 2>&1 && \
for v in lead4 lead2 lead3; do DPOW_LIB_PATH=abx/$v.so timeout -k 10 300 python3 tools/layout_sweep.py 33 2 > gpurun_out/r02_ab_lead_layout_$v.log 2>&1 || exit 1; done
