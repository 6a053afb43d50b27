# GPU tests, the short-search probe and the 8-rank one-GPU rehearsal of the N > 1 bench path
# (8 processes sharing the card: the device-queue load of each process matters), through gpurun.
set -o pipefail
tag=${1:-reh}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 200 python3 -u tools/small_search_probe.py > $out/small.json 2> $out/small.err &&
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 2 --warmup 1 --backend gloo --same-device --no-probe > $out/bench_n8.json 2> $out/bench_n8.err
