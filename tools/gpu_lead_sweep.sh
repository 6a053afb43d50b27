set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 tools/lead_sweep.py abx/lead1.so abx/lead2.so abx/lead3.so abx/lead4.so abx/lead5.so abx/lead6.so > gpurun_out/r02_lead_sweep.json 2> gpurun_out/r02_lead_sweep.err
