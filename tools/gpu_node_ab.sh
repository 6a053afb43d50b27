# A/B of prebuilt libraries on the emulated 8-GPU node (tools/node_probe.py, G8) and on the
# sweep rate (tools/ab_variants.py), through gpurun:
#   gpurun --timeout 1200 -- bash tools/gpu_node_ab.sh <tag> <runs> name=lib.so[,VAR=value...] ...
# (VAR=value: environment of that variant's node probe, e.g. DPOW_DIAG_POLL_WB=2)
set -o pipefail
tag=$1; runs=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
libs=()
for rnd in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=()
    [ "$rest" != "$lib" ] && IFS=, read -ra envs <<< "${rest#*,}"
    [ $rnd = 1 ] && [[ ! " ${libs[*]} " =~ " $lib " ]] && libs+=("$lib")
    env "${envs[@]}" DPOW_LIB_PATH=$lib timeout -k 10 300 python3 -u tools/node_probe.py $runs 8 > $out/node_${name}_$rnd.json 2> $out/node_${name}_$rnd.err || exit $?
  done
done
timeout -k 10 600 python3 -u tools/ab_variants.py "${libs[@]}" > $out/ab.log 2>&1
