#!/usr/bin/env python3
"""Aggregate rate of W concurrent searches sharing one GPU (the coordinator mirror's
logical workers, BASELINE configs 4-5): W threads, one Miner each, worker w of
workerBits log2(W) over the same k window with no hit (N = 14), started together.
Reports the wall time to drain all W, the aggregate GH/s and each search's finish
time (fairness).  The first hit among W workers is the minimum of W geometric waits,
so its expected time follows the aggregate rate, not how it is split.  GPU box only.
    python3 tools/concurrent_rate.py [W] [log2 k-span] [reps]"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import distpow  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
SPAN = int(sys.argv[2]) if len(sys.argv) > 2 else 26
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
bits = W.bit_length() - 1
assert 1 << bits == W
K0 = 1 << 24
miners = [distpow.Miner(0) for _ in range(W)]
for m in miners:
    m.search([1, 2, 3, 4], 14, 0, bits, K0, K0 + (1 << 16))  # warm
cands = W * (1 << SPAN) << (8 - bits)
out = {"build_id": distpow.build_id(), "W": W, "candidates": cands,
       "env": {k: v for k, v in os.environ.items() if k.startswith("DPOW_DIAG_") or k == "GPU_MAX_HW_QUEUES"},
       "runs": []}
for _ in range(REPS):
    go = threading.Barrier(W + 1)
    ends = [0.0] * W

    def run(w):
        go.wait()
        r = miners[w].search([1, 2, 3, 4], 14, w, bits, K0, K0 + (1 << SPAN))
        assert r.status != distpow.FOUND
        ends[w] = time.perf_counter()
    th = [threading.Thread(target=run, args=(w,)) for w in range(W)]
    for t in th:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    wall = max(ends) - t0
    out["runs"].append({"wall_ms": round(wall * 1e3, 2), "ghs": round(cands / wall / 1e9, 1),
                        "finish_ms": sorted(round((e - t0) * 1e3, 1) for e in ends)})
    print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
for m in miners:
    m.close()
print(json.dumps(out))
