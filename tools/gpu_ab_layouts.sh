# Layout A/B of the one-block layouts: session-start build (head0) vs current (new3).
set -o pipefail
mkdir -p gpurun_out/ablay4
for rnd in 1 2 3; do for v in head0 new3; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/layout_sweep.py 33 1 0,1,2,3,4,5,6,7,8,12,16,24,32,40,48,50,64,68,100,56,61 > gpurun_out/ablay4/${v}_$rnd.log 2>&1 || exit 1
done; done
