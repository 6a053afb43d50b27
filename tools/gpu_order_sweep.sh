set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 tools/lead_sweep.py abt/order2.so abt/order1.so > gpurun_out/r02_order_sweep.json 2> gpurun_out/r02_order_sweep.err
