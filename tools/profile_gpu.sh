#!/bin/bash
# Profile bench.py on the GPU box (run via gpurun).  Usage: tools/profile_gpu.sh <tag> [pmc]
#  1. rocprofv3 --kernel-trace --stats (CSV) of the bench command      -> gpurun_out/prof_<tag>/trace
#  2. with "pmc": separate counter passes (SQ/GRBM; FETCH_SIZE; WRITE_SIZE) on a 1-step bench
set -euo pipefail
TAG=${1:?tag}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $BENCH > "$OUT/bench.json" 2> "$OUT/trace.err"
if [ "${2:-}" = "pmc" ]; then
    ONE="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-probe --no-tts"
    timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_sq" -o run -- \
        python3 $ONE > "$OUT/pmc_sq.json" 2> "$OUT/pmc_sq.err"
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
        python3 $ONE > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
        python3 $ONE > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
fi
find "$OUT" -type f | sort
