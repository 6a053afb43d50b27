# Per-layout A/B of the s_nop padding builds in ab/ (tools/lead_sweep.py over all 64 nonce lengths).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 tools/lead_sweep.py ab/nop_def.so ab/nop_a1.so ab/nop_a3.so ab/nop_r1.so ab/nop_d0.so > gpurun_out/r02_ab_nop_layouts.json 2> gpurun_out/r02_ab_nop_layouts.err
