#!/bin/bash
# Round 5: host timelines of one GPU and of 2-, 4- and 8-GPU node ranks at small N.
set -e -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u tools/owner_timeline.py 2,4,8 > $O/owner_timeline.json 2> $O/owner_timeline.err
