# Launch-policy A/B of two builds on the BASELINE short cases, fresh nonces (tools/small_search_probe.py)
# and the emulated 8-GPU node (tools/node_probe.py G8), through gpurun:
#   gpurun --timeout 1200 -- bash tools/gpu_r04_policy_ab.sh <tag> new.so old.so
set -o pipefail
tag=$1; new=$2; old=$3
out=gpurun_out/$tag
mkdir -p $out
for rnd in 1 2; do
  for lib in $new $old; do
    n=$(basename $lib .so)
    DPOW_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/small_search_probe.py > $out/cases_${n}_$rnd.json 2> $out/cases_${n}_$rnd.err || exit $?
    DPOW_LIB_PATH=$lib timeout -k 10 400 python3 -u tools/small_search_probe.py --random > $out/random_${n}_$rnd.json 2> $out/random_${n}_$rnd.err || exit $?
  done
done
bash tools/gpu_node_ab.sh $tag 3 new=$new old=$old
