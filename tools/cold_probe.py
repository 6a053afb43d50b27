#!/usr/bin/env python3
"""The first long search after the GPU idled: config 4's BASELINE nonce ([1,2,3,4]/8, ~19 ms of
hashing) through Miner.mine, back to back and after idle gaps of 0.1 / 1 s, in one context.
GPU box only.
    python3 tools/cold_probe.py > gpurun_out/<tag>/cold.json"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-proof-of-work_amd"))
import distpow  # noqa: E402

out = []
with distpow.Miner(0) as m:
    for gap in (0, 0, 0, 0.1, 0, 1.0, 0, 0.1, 1.0):
        time.sleep(gap)
        t = time.perf_counter()
        r = m.mine([1, 2, 3, 4], 8)
        out.append({"idle_s_before": gap, "ms": round((time.perf_counter() - t) * 1e3, 3), "global_idx": r.global_idx})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
print(json.dumps(out))
