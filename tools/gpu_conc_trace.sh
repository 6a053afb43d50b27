# Kernel trace of 4 concurrent searches with share-sized grids (1 workgroup per CU each):
# do the searches' kernels overlap on the device, and on which hardware queues?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/r04conc_trace; mkdir -p $d
DPOW_DIAG_BPC=4 DPOW_DIAG_POLL_WB=4 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d/w4 -o kt -- python3 -u tools/concurrent_rate.py 4 26 1 > $d/w4.json 2> $d/w4.err &&
DPOW_DIAG_BPC=4 DPOW_DIAG_POLL_WB=4 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 -u tools/concurrent_rate.py 4 26 2 > $d/w4_q8.json 2> $d/w4_q8.err &&
DPOW_DIAG_BPC=2 DPOW_DIAG_POLL_WB=4 timeout -k 10 120 python3 -u tools/concurrent_rate.py 2 26 2 > $d/w2_bpc2.json 2> $d/w2_bpc2.err &&
find $d -name '*.csv' > $d/files.txt
