# The round-3 evidence run: the node emulation and a 2-rank rehearsal of the N>1 bench path,
# then tools/gpu_evidence.sh (GPU tests, bench, time-to-secret timeline, wave trace, node probe).
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag>
set -o pipefail
tag=${1:-round}
mkdir -p gpurun_out/$tag
bash tools/gpu_rehearse_n8.sh $tag 2 && bash tools/gpu_evidence.sh $tag
