# GPU tests then an A/B of prebuilt libraries (tools/ab_variants.py) through gpurun
set -o pipefail
mkdir -p gpurun_out/r03i
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i/pytest.log 2>&1 || { tail -30 gpurun_out/r03i/pytest.log; exit 1; }
tail -1 gpurun_out/r03i/pytest.log
timeout -k 10 600 python3 -u tools/ab_variants.py ab/ed13f8e.so ab/head2.so ab/nolspan.so > gpurun_out/r03i/ab.log 2>&1
tail -4 gpurun_out/r03i/ab.log
