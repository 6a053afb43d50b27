#!/usr/bin/env python3
"""Kernel GH/s against launch size (2^26 / 2^29 / 2^32 candidates per launch) for
workerBits 0 and 3 (bench sweep nonce, N = 32, L = 4 segment).  GPU box only."""
import sys, json
sys.path.insert(0, "distributed-proof-of-work_amd")
import torch, distpow
m = distpow.Miner(0)
m.search([1,2,3,4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 24))
out = {}
for wbits, wb in ((0, 0), (3, 5)):
    R = 1 << (8 - wbits)
    for log2c in (26, 29, 32):
        nk = (1 << log2c) // R
        if nk > (1 << 24):
            continue
        m.reset_stats()
        k0 = 1 << 25
        for t in range(8):
            m.search([1,2,3,4], 32, wb, wbits, k0 + t * nk, k0 + (t + 1) * nk)
        st = m.stats()
        out[f"wbits{wbits}/2^{log2c}"] = [round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2), st.launches,
                                          round(st.kernel_ms / st.launches, 3)]
print(json.dumps(out))
