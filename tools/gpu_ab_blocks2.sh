set -o pipefail
mkdir -p gpurun_out/abblocks
for v in b6 b4 b3; do
  DPOW_LIB_PATH=abt/$v.so timeout -k 10 200 python3 tools/launch_size_probe.py > gpurun_out/abblocks/size_$v.json 2> gpurun_out/abblocks/size_$v.err || exit 1
done
