#!/usr/bin/env python3
"""BASELINE configs 3 and 4 over fresh nonces, W logical workers sharing one GPU, one request
per nonce (no cache hits), in both coordinator modes on the same nonces:
  - node: the workers share a node board (csrc/board.cpp), the answer is the node's first hit;
  - first: node=False, the reference's first-arrived race (coordinator.go:202);
next to one Miner.mine of the same nonce (the workerBits = 0 search alone on the GPU).  Every
node answer must equal Miner.mine's (the deterministic first hit); the first-arrived ones only
verify.  A single nonce times one draw; the mean over nonces follows the device's aggregate
rate.  Each mode's first request of a fresh coordinator is timed separately (`cold_ms`).
GPU box only.
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
with distpow.Miner(0) as m:
    for workers, ntz in ((4, 7), (8, 8)):
        nonces = [[rng.randrange(256) for _ in range(4)] for _ in range(n_nonces)]
        key = f"{workers}workers_n{ntz}"
        case = {}
        single, want = [], []
        for nonce in nonces:
            t = time.perf_counter()
            r = m.mine(nonce, ntz)
            single.append((time.perf_counter() - t) * 1e3)
            want.append(r.secret)
        case["miner_mine"] = {"mean_ms": round(statistics.mean(single), 3),
                              "median_ms": round(statistics.median(single), 3)}
        for mode in ("node", "first"):
            ms, cold, exact = [], [], 0
            for rep in range(3):  # the first request of a fresh coordinator (board pages, pools)
                with Coordinator(workers, node=(mode == "node")) as c:
                    t = time.perf_counter()
                    s = c.mine([rep, 7, 7, 7], ntz)
                    cold.append((time.perf_counter() - t) * 1e3)
            with Coordinator(workers, node=(mode == "node")) as c:
                c.mine([9, 9, 9, 9], 5)  # warm
                for nonce, w in zip(nonces, want):
                    t = time.perf_counter()
                    s = c.mine(nonce, ntz)
                    ms.append((time.perf_counter() - t) * 1e3)
                    assert distpow.verify(nonce, s, ntz)
                    exact += s == w
            if mode == "node" and exact != len(nonces):
                raise SystemExit(f"{key}: node mode returned {len(nonces) - exact} non-deterministic answers")
            case[mode] = {"mean_ms": round(statistics.mean(ms), 3), "median_ms": round(statistics.median(ms), 3),
                          "cold_ms": [round(x, 3) for x in cold], "deterministic": exact,
                          "ms": [round(x, 3) for x in ms]}
        out["cases"][key] = case
        print(key, json.dumps({k: {x: y for x, y in v.items() if x != "ms"} for k, v in case.items()}),
              file=sys.stderr, flush=True)
print(json.dumps(out))
