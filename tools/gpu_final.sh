# Final-build evidence through gpurun: GPU tests, the driver's default bench line, the
# time-to-secret timeline, the per-wave trace, the emulated node (tools/gpu_evidence.sh),
# smoke(), then the rocprofv3 kernel-trace + PMC passes of the bench (tools/profile_gpu.sh).
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-final}
bash tools/gpu_evidence.sh $tag &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 &&
bash tools/profile_gpu.sh $tag pmc > gpurun_out/$tag/profile.list 2>&1
