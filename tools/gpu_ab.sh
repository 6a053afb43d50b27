# A/B of prebuilt libraries (tools/ab_variants.py) through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_ab.sh <tag> lib1.so lib2.so ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 800 python3 -u tools/ab_variants.py "$@" > gpurun_out/$tag/ab.log 2>&1
