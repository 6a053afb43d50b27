# The driver's round-end sequence on the current tree, through gpurun: GPU tests, smoke(), the
# default bench line.
set -o pipefail
tag=${1:-driver}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err
rc=$?
tail -1 $out/pytest.log; tail -1 $out/smoke.log
exit $rc
