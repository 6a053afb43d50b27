#!/bin/bash
# Round 5, first GPU call: the Option A state machine on the GPU, host timelines of an
# 8-GPU node's owner / non-owner ranks, and the emulated node's small-N cases.
set -e -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_option_a.py -m gpu > $O/opta.log 2>&1
timeout -k 10 300 python -u tools/owner_timeline.py > $O/owner_timeline.json 2> $O/owner_timeline.err
timeout -k 10 500 python -u tools/node_probe.py 3 2,4,8 small > $O/node_probe.json 2> $O/node_probe.err
