# Launch length on a shared device (DPOW_DIAG_SHARE_LAUNCH_US): aggregate rate of 8 / 4
# concurrent searches and config 4 over fresh nonces.
set -o pipefail
d=gpurun_out/r04capab; mkdir -p $d
run() { tag=$1; w=$2; shift 2; env "$@" timeout -k 10 120 python3 -u tools/concurrent_rate.py $w 26 3 > $d/$tag.json 2> $d/$tag.err; }
run w8_c2 8 DPOW_DIAG_SHARE_LAUNCH_US=2000 &&
run w8_c4 8 DPOW_DIAG_SHARE_LAUNCH_US=4000 &&
run w8_c8 8 DPOW_DIAG_SHARE_LAUNCH_US=8000 &&
run w8_c16 8 DPOW_DIAG_SHARE_LAUNCH_US=16000 &&
run w4_c2 4 DPOW_DIAG_SHARE_LAUNCH_US=2000 &&
run w4_c8 4 DPOW_DIAG_SHARE_LAUNCH_US=8000 &&
run w8_c2b 8 DPOW_DIAG_SHARE_LAUNCH_US=2000 &&
run w8_c8b 8 DPOW_DIAG_SHARE_LAUNCH_US=8000 &&
DPOW_DIAG_SHARE_LAUNCH_US=2000 timeout -k 10 200 python3 -u tools/coord_fresh.py 16 > $d/fresh_c2.json 2> $d/fresh_c2.err &&
DPOW_DIAG_SHARE_LAUNCH_US=8000 timeout -k 10 200 python3 -u tools/coord_fresh.py 16 > $d/fresh_c8.json 2> $d/fresh_c8.err
