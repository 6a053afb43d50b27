# A/B of the k = 0 kernel's stream (DPOW_DIAG_K0_STREAM: 1 = the context's second stream,
# beside the first md5 launch; 0 = the search stream, ahead of it): short searches on one
# GPU (tools/small_search_probe.py) and the 8-rank one-GPU rehearsal, through gpurun.
set -o pipefail
tag=${1:-k0ab}
out=gpurun_out/$tag
mkdir -p $out
for v in 1 0; do
    DPOW_DIAG_K0_STREAM=$v timeout -k 10 200 python3 -u tools/small_search_probe.py > $out/small_k0s$v.json 2> $out/small_k0s$v.err || exit $?
done
DPOW_DIAG_K0_STREAM=0 bash tools/gpu_rehearse_n8.sh $tag 8
