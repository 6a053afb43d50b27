set -o pipefail
mkdir -p gpurun_out/clock
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/clock/pmc -o run -- python3 tools/clock_probe.py > gpurun_out/clock/probe.json 2> gpurun_out/clock/probe.err
