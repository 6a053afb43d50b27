# A/B: claim-ahead (next claim requested while hashing) vs one claim in flight per wave.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ab_variants.py abt/ahead1.so abt/ahead0.so abt/ahead0p8.so > gpurun_out/r02_ab_ahead.log 2>&1 && \
DPOW_LIB_PATH=abt/ahead1.so timeout -k 10 200 python3 tools/node_probe.py 5 > gpurun_out/r02_ab_ahead_node1.json 2> gpurun_out/r02_ab_ahead_node1.err && \
DPOW_LIB_PATH=abt/ahead0.so timeout -k 10 200 python3 tools/node_probe.py 5 > gpurun_out/r02_ab_ahead_node0.json 2> gpurun_out/r02_ab_ahead_node0.err
