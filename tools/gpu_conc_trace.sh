# Kernel trace of 4 and 8 concurrent searches on one GPU (tools/concurrent_rate.py): the grids
# each search's launches get and their lengths (plan.h grid_share, cap_shared_launch).
#   gpurun -- bash tools/gpu_conc_trace.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/${1:-conc_trace}; mkdir -p $d
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d/w4 -o kt -- python3 -u tools/concurrent_rate.py 4 26 1 > $d/w4.json 2> $d/w4.err &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d/w8 -o kt -- python3 -u tools/concurrent_rate.py 8 26 1 > $d/w8.json 2> $d/w8.err
