set -o pipefail
mkdir -p gpurun_out/tts
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tts/trace -o run -- python3 tools/tts_trace.py > gpurun_out/tts/tts.json 2> gpurun_out/tts/tts.err
