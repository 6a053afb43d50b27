#!/usr/bin/env python3
"""Kernel GH/s of the bench sweep (nonce [1,2,3,4], N = 32, 2^36 candidates in the L = 4
segment) for the partitions a rank searches at 1/2/4/8 GPUs (workerBits 0..3).  GPU box only."""
import os, sys, json
sys.path.insert(0, "distributed-proof-of-work_amd")
import torch, distpow
m = distpow.Miner(0)
m.search([1,2,3,4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 24))
out = {}
for wbits, wb in ((0, 0), (1, 1), (2, 3), (3, 5), (3, 0)):
    R = 1 << (8 - wbits)
    nk = (1 << 36) // R
    m.reset_stats()
    r = m.search([1,2,3,4], 32, wb, wbits, 1 << 24, (1 << 24) + nk)
    st = m.stats()
    out[f"wbits{wbits}/wb{wb}"] = round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2)
print(json.dumps(out))
