#!/usr/bin/env python3
"""Kernel time of one search window against its size (L = 3 segment, nonce [1,2,3,4],
N = 32, workerBits 0 and 3), median of 5: the fixed cost of a launch and the rate
beyond it, for the grid-size A/B of small launches.  GPU box only."""
import json, sys, time
sys.path.insert(0, "distributed-proof-of-work_amd")
import torch  # noqa: F401
import distpow
m = distpow.Miner(0)
m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
out = {}
for wbits, wb in ((0, 0), (3, 5)):
    R = 1 << (8 - wbits)
    for lg in (18, 20, 22, 24, 25, 26, 28):
        nk = (1 << lg) // R
        ts, ws = [], []
        for rep in range(5):
            k0 = (1 << 20) + rep * nk
            m.reset_stats()
            t0 = time.perf_counter()
            m.search([1, 2, 3, 4], 32, wb, wbits, k0, k0 + nk)
            ws.append((time.perf_counter() - t0) * 1e6)
            ts.append(m.stats().kernel_ms * 1e3)
        out[f"wbits{wbits}/2^{lg}"] = {"kernel_us": round(sorted(ts)[2], 1), "wall_us": round(sorted(ws)[2], 1)}
print(json.dumps(out))
