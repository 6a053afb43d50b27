#!/usr/bin/env python3
"""Sweep throughput per message layout (nonce length -> kernel variant <NBLK, W0, SH>).

    python tools/layout_sweep.py [log2_candidates] [rounds] [nonce lengths, comma-separated]

For each nonce length, hashes 2^n candidates (default 2^34) of an all-0x5a nonce at
N = 32 (unreachable) in the L = 4 chunk segment and prints the kernel GH/s (HIP-event
time) of its layout, so that no variant is left pathologically slow.  GPU box only.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-proof-of-work_amd"))
import torch  # noqa: F401,E402  (one HIP runtime with torch)
import distpow  # noqa: E402

LOG2 = int(sys.argv[1]) if len(sys.argv) > 1 else 34
K0 = 1 << 24
NK = (1 << LOG2) >> 8
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
LENGTHS = (0, 1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 24, 32, 40, 48, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60,
           61, 62, 63, 64, 68, 100, 120)
if len(sys.argv) > 3:
    LENGTHS = tuple(int(x) for x in sys.argv[3].split(","))
out = {}
with distpow.Miner(0) as m:
    m.search([1, 2, 3, 4], 32, 0, 0, K0, K0 + NK)  # warm the clocks on a full-size run first
    for rnd in range(ROUNDS):  # interleaved rounds: the spread is the run-to-run noise
        for n in LENGTHS:
            nonce = [0x5A] * n
            p = distpow.plan_window(nonce, 0, 0, K0, K0 + 1)[0]
            m.reset_stats()
            r = m.search(nonce, 32, 0, 0, K0 + rnd * NK, K0 + (rnd + 1) * NK)
            st = m.stats()
            assert r.status == distpow.EXHAUSTED
            e = out.setdefault(n, {"layout": f"<{p.nblk},{p.w0},{p.sh}>", "kernel_ghs": []})
            e["kernel_ghs"].append(round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2))
            print(rnd, n, e, flush=True)
print(json.dumps(out))
