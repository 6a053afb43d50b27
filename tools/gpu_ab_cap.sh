# Per-layout A/B of the VGPR-K cap (DPOW_VGPR_K_MAX) builds in ab/ (tools/lead_sweep.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 tools/lead_sweep.py ab/cap20.so ab/cap12.so ab/cap14.so ab/cap16.so > gpurun_out/r02_ab_cap.json 2> gpurun_out/r02_ab_cap.err
