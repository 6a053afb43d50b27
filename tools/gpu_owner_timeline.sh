set -o pipefail
mkdir -p gpurun_out/${1:-ot}
timeout -k 10 200 python3 -u tools/owner_timeline.py > gpurun_out/${1:-ot}/base.json 2> gpurun_out/${1:-ot}/base.err
