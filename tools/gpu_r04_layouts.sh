set -o pipefail
out=gpurun_out/r04lay
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "early_found or two_contexts or bound_beyond" --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 600 python3 -u tools/layout_sweep.py 34 3 0,3,4,7,8,48,51,52,55,56,57,58,59,60,63 > $out/layout_sweep.log 2> $out/layout_sweep.err
