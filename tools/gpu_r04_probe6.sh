set -o pipefail
D=distributed-proof-of-work_amd/distpow
mkdir -p gpurun_out/r04ot3
timeout -k 10 200 python3 -u tools/owner_timeline.py > gpurun_out/r04ot3/base.json 2> gpurun_out/r04ot3/base.err &&
bash tools/gpu_node_ab.sh r04ab6 5 base=$D/libdpow.so early=$D/libdpow_early.so bpc6=$D/libdpow.so,DPOW_DIAG_BPC=6 bpc5=$D/libdpow.so,DPOW_DIAG_BPC=5 cpw32=$D/libdpow.so,DPOW_DIAG_CPW=32 mc8=$D/libdpow.so,DPOW_DIAG_MIN_CHUNK=8 poll8=$D/libdpow.so,DPOW_DIAG_POLL_WB=8 &&
DPOW_LIB_PATH=$D/libdpow_trace.so timeout -k 10 300 python3 -u tools/wave_trace_node.py > gpurun_out/r04ab6/wave_trace_node.json 2> gpurun_out/r04ab6/wave_trace_node.err
