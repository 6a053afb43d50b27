# GPU check of the current tree (run through gpurun): the GPU test suite, the driver's
# default bench line, the 2-rank bench through bench.py's own launcher (gloo, both ranks on
# the one GPU), and the time-to-secret launch timeline under rocprofv3.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh <tag>
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out/tts
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --same-device --steps 2 --warmup 1 --no-probe \
    --no-cpu-baseline > $out/bench_n2.json 2> $out/bench_n2.err &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/tts/trace -o run -- python3 tools/tts_trace.py > $out/tts/tts.json 2> $out/tts/tts.err
rc=$?
tail -3 $out/pytest.log
exit $rc
