# Round-4 final-build evidence through gpurun: GPU tests, the driver's default bench line, the
# 2-rank bench through bench.py's own launcher, the time-to-secret timeline (tools/gpu_check.sh),
# the emulated 2/4/8-GPU node, the layout check, smoke(), an 8-rank rehearsal of
# `bench.py --gpus 8` on one GPU (gloo, --same-device), then the rocprofv3 kernel-trace and PMC
# passes of the bench (tools/profile_gpu.sh).
#   gpurun --timeout 1500 -- bash tools/gpu_final_r04.sh <tag>
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag
bash tools/gpu_check.sh $tag &&
timeout -k 10 400 python3 -u tools/node_probe.py 3 > $out/node_probe.json 2> $out/node_probe.err &&
timeout -k 10 300 python3 -u tests/soak/layout_check.py > $out/layout_check.json 2> $out/layout_check.err &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 600 python3 bench.py --gpus 8 --backend gloo --same-device --steps 2 --warmup 1 --no-probe \
    > $out/bench_n8.json 2> $out/bench_n8.err &&
bash tools/profile_gpu.sh $tag pmc > $out/profile.list 2>&1
