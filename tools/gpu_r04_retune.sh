# The per-layout retune: GPU tests, the layout check, and the per-layout sweep of the new build
# against the previous one (tools/lead_sweep.py), through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_r04_retune.sh <tag>
set -o pipefail
tag=${1:-retune}
D=distributed-proof-of-work_amd/distpow
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python3 -u tests/soak/layout_check.py > $out/layout_check.json 2> $out/layout_check.err &&
timeout -k 10 600 python3 -u tools/lead_sweep.py $D/libdpow.so $D/ab/libdpow_old.so > $out/lead_sweep.json 2> $out/lead_sweep.err
