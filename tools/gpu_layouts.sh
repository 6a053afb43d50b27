# GPU tests, the layout check against the oracle (tests/soak/layout_check.py) and a layout
# sweep (tools/layout_sweep.py) through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_layouts.sh <tag> [log2 rounds lengths]
set -o pipefail
tag=${1:-layouts}; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python3 -u tests/soak/layout_check.py > $out/layout_check.json 2> $out/layout_check.err &&
timeout -k 10 600 python3 -u tools/layout_sweep.py "$@" > $out/layout_sweep.log 2> $out/layout_sweep.err
