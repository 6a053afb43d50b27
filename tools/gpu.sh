#!/bin/bash
# The GPU runs of this repo, one task per call, through gpurun (every step under its own time
# limit, chained with &&: a failed step ends the call).  Results go to gpurun_out/<tag>/.
#
#   gpurun --timeout 1500 -- bash tools/gpu.sh <task> <tag> [args]
#
#   tests            the GPU test suite (pytest -m gpu)
#   check            GPU tests, the driver's default bench line, the 2-rank bench through
#                    bench.py's own launcher (gloo, both ranks on the one GPU), the time-to-secret
#                    launch timeline under rocprofv3
#   final            the final-build evidence: check, the emulated 2/4/8-GPU node
#                    (tools/node_probe.py), the layout check, smoke(), an 8-rank rehearsal of
#                    `bench.py --gpus 8` (gloo, --same-device), the rocprofv3 kernel-trace and
#                    PMC passes of the bench (tools/profile_gpu.sh)
#   node [runs] [G,..] [small]   the emulated node alone
#   node-small-ab name=lib.so[,VAR=value...] ...   the emulated node's small cases per library (A/B;
#                    NODE_RUNS runs per case, default 3)
#   timeline [G,..]  host timelines of one GPU's and the node ranks' searches (tools/owner_timeline.py)
#   stl [G,..] [cases]   host + device timeline of small searches on one clock (tools/search_timeline.py)
#   trace [G,..] [cases]   per-wave traces (diag build distpow/libdpow_trace.so, tools/wave_trace_node.py)
#   layouts [log2 rounds lengths]   GPU tests, the layout check, the layout sweep (tools/layout_sweep.py)
#   rehearse [N]     N gloo ranks of bench.py on device 0 (the driver's N > 1 path, one GPU)
#   coord            searches sharing one GPU: configs 3 / 4 over fresh nonces, 8 / 4 concurrent
#                    searches (tools/coord_fresh.py, concurrent_rate.py, coord_probe.py)
#   small <cases|random|stop> [knobs]   short-search launch knobs (tools/small_search_probe.py)
#   ab lib.so ...    sweep-rate A/B of prebuilt libraries (tools/ab_variants.py)
#   node-ab runs name=lib.so[,VAR=value...] ...   the emulated 8-GPU node per library, then ab
set -o pipefail
task=${1:?task}; tag=${2:?tag}; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
# The in-tree libdpow.so must be the sources' build: it is built here, not on the box.
DPOW_NO_AUTOBUILD=1 python3 -c 'import sys; sys.path.insert(0, "distributed-proof-of-work_amd"); import distpow; distpow.lib()' \
    || { echo "tools/gpu.sh: libdpow.so does not match the sources (build it before the call)" >&2; exit 3; }

tests() {
    timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
    local rc=$?
    tail -3 $out/pytest.log
    return $rc
}

check() {
    mkdir -p $out/tts
    tests &&
    timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err &&
    timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --same-device --steps 2 --warmup 1 --no-probe \
        --no-cpu-baseline > $out/bench_n2.json 2> $out/bench_n2.err &&
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/tts/trace -o run -- \
        python3 tools/tts_trace.py > $out/tts/tts.json 2> $out/tts/tts.err
}

rehearse() {
    local n=${1:-8}
    timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port 29513 bench.py --gpus $n --steps 2 --warmup 1 --backend gloo --same-device --no-probe \
        > $out/bench_n$n.json 2> $out/bench_n$n.err
}

case $task in
tests) tests ;;
check) check ;;
final)
    check &&
    timeout -k 10 400 python3 -u tools/node_probe.py 3 > $out/node_probe.json 2> $out/node_probe.err &&
    timeout -k 10 300 python3 -u tests/soak/layout_check.py > $out/layout_check.json 2> $out/layout_check.err &&
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
    timeout -k 10 600 python3 bench.py --gpus 8 --backend gloo --same-device --steps 2 --warmup 1 --no-probe \
        > $out/bench_n8.json 2> $out/bench_n8.err &&
    bash tools/profile_gpu.sh $tag pmc > $out/profile.list 2>&1 ;;
node) timeout -k 10 600 python3 -u tools/node_probe.py "${1:-3}" "${2:-2,4,8}" $3 > $out/node_probe.json 2> $out/node_probe.err ;;
node-small-ab)  # the emulated 2/4/8-GPU node's small cases per library, twice, interleaved
    for rnd in 1 2; do
        for spec in "$@"; do
            name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=()
            [ "$rest" != "$lib" ] && IFS=, read -ra envs <<< "${rest#*,}"
            env "${envs[@]}" DPOW_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/node_probe.py ${NODE_RUNS:-3} 2,4,8 small \
                > $out/node_${name}_$rnd.json 2> $out/node_${name}_$rnd.err || exit $?
        done
    done ;;
stl)  # the timeline with the product library, then with the diag build's per-wave records
    timeout -k 10 300 python3 -u tools/search_timeline.py "$@" > $out/search_timeline.json 2> $out/search_timeline.err &&
    DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so timeout -k 10 300 \
        python3 -u tools/search_timeline.py "$@" > $out/search_timeline_trace.json 2> $out/search_timeline_trace.err ;;
timeline) timeout -k 10 300 python3 -u tools/owner_timeline.py "${1:-2,4,8}" > $out/owner_timeline.json 2> $out/owner_timeline.err ;;
trace)
    DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so timeout -k 10 300 \
        python3 -u tools/wave_trace_node.py "$@" > $out/wave_trace.json 2> $out/wave_trace.err ;;
layouts)
    tests &&
    timeout -k 10 300 python3 -u tests/soak/layout_check.py > $out/layout_check.json 2> $out/layout_check.err &&
    timeout -k 10 600 python3 -u tools/layout_sweep.py "$@" > $out/layout_sweep.log 2> $out/layout_sweep.err ;;
rehearse) rehearse "$@" ;;
coord)
    timeout -k 10 200 python3 -u tools/coord_fresh.py 16 > $out/fresh.json 2> $out/fresh.err &&
    timeout -k 10 120 python3 -u tools/concurrent_rate.py 8 26 3 > $out/w8.json 2> $out/w8.err &&
    timeout -k 10 120 python3 -u tools/concurrent_rate.py 4 26 3 > $out/w4.json 2> $out/w4.err &&
    timeout -k 10 200 python3 -u tools/coord_probe.py 5 > $out/coord.json 2> $out/coord.err ;;
small)
    mode=${1:-cases}; shift
    flag=""; [ "$mode" != cases ] && flag="--$mode"
    timeout -k 10 500 python3 -u tools/small_search_probe.py $flag "$@" > $out/$mode.json 2> $out/$mode.err ;;
ab) timeout -k 10 800 python3 -u tools/ab_variants.py "$@" > $out/ab.log 2>&1 ;;
node-ab)
    runs=$1; shift
    libs=()
    for rnd in 1 2; do
        for spec in "$@"; do
            name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=()
            [ "$rest" != "$lib" ] && IFS=, read -ra envs <<< "${rest#*,}"
            [ $rnd = 1 ] && [[ ! " ${libs[*]} " =~ " $lib " ]] && libs+=("$lib")
            env "${envs[@]}" DPOW_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/node_probe.py $runs 8 \
                > $out/node_${name}_$rnd.json 2> $out/node_${name}_$rnd.err || exit $?
        done
    done
    timeout -k 10 600 python3 -u tools/ab_variants.py "${libs[@]}" > $out/ab.log 2>&1 ;;
*) echo "tools/gpu.sh: unknown task $task" >&2; exit 2 ;;
esac
