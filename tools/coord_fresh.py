#!/usr/bin/env python3
"""BASELINE configs 3 and 4 over fresh nonces: the coordinator mirror's first-arrived answer
with W logical workers sharing one GPU, one request per nonce (no cache hits).  A single nonce
times one draw: which worker holds the first hit and what share of the device its search got;
the mean over nonces follows the device's aggregate rate.  GPU box only.
    python3 tools/coord_fresh.py [n_nonces] > gpurun_out/<tag>/fresh.json"""
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import distpow  # noqa: E402
from distpow.coordinator import Coordinator  # noqa: E402

n_nonces = int(sys.argv[1]) if len(sys.argv) > 1 else 12
rng = random.Random(20261017)
out = {"build_id": distpow.build_id(), "cases": {}}
for workers, ntz in ((4, 7), (8, 8)):
    nonces = [[rng.randrange(256) for _ in range(4)] for _ in range(n_nonces)]
    ms = []
    with Coordinator(workers) as c:
        c.mine([9, 9, 9, 9], 5)  # warm
        for nonce in nonces:
            t = time.perf_counter()
            s = c.mine(nonce, ntz)
            ms.append((time.perf_counter() - t) * 1e3)
            assert distpow.verify(nonce, s, ntz)
    key = f"{workers}workers_n{ntz}"
    out["cases"][key] = {"mean_ms": round(statistics.mean(ms), 3), "median_ms": round(statistics.median(ms), 3),
                         "ms": [round(x, 3) for x in ms]}
    print(key, json.dumps(out["cases"][key]), file=sys.stderr, flush=True)
print(json.dumps(out))
