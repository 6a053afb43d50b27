# Per-layout A/B of the layout-tuning builds (tools/lead_sweep.py) through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_r04_leads.sh <tag>
set -o pipefail
tag=${1:-leads}
D=distributed-proof-of-work_amd/distpow
mkdir -p gpurun_out/$tag
timeout -k 10 800 python3 -u tools/lead_sweep.py $D/libdpow.so $D/ab/libdpow_lead1.so $D/ab/libdpow_lead2.so \
    $D/ab/libdpow_lead3.so $D/ab/libdpow_lead4.so $D/ab/libdpow_lead5.so $D/ab/libdpow_lead6.so \
    $D/ab/libdpow_sgpr100.so $D/ab/libdpow_cap16.so $D/ab/libdpow_cap24.so \
    > gpurun_out/$tag/lead_sweep.json 2> gpurun_out/$tag/lead_sweep.err
