# Shared-device policy check: BASELINE configs 3 / 4 over fresh nonces and the aggregate rate of
# 8 / 4 concurrent searches on one GPU (plan.h grid_share, cap_shared_launch).
#   gpurun -- bash tools/gpu_coord_probe.sh <tag>
set -o pipefail
d=gpurun_out/${1:-share}; mkdir -p $d
timeout -k 10 200 python3 -u tools/coord_fresh.py 16 > $d/fresh.json 2> $d/fresh.err &&
timeout -k 10 120 python3 -u tools/concurrent_rate.py 8 26 3 > $d/w8.json 2> $d/w8.err &&
timeout -k 10 120 python3 -u tools/concurrent_rate.py 4 26 3 > $d/w4.json 2> $d/w4.err &&
timeout -k 10 200 python3 -u tools/coord_probe.py 5 > $d/coord.json 2> $d/coord.err
