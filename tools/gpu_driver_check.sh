# The round-end driver's own sequence on one GPU box: GPU tests, smoke(), default bench.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02_driver}
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
