# A/B of libdpow builds (tools/ab_variants.py) through gpurun:
#   gpurun --timeout 900 -- bash tools/gpu_ab.sh <tag> ab/a.so ab/b.so ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 800 python3 -u tools/ab_variants.py "$@" > gpurun_out/$tag/ab.log 2>&1
rc=$?
tail -8 gpurun_out/$tag/ab.log
exit $rc
