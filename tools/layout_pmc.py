#!/usr/bin/env python3
"""One layout's sweep window for a PMC pass (rocprofv3 --pmc ...): nonce of the given
length (all 0x5a), N = 32, 2^33 candidates in the L = 4 segment, after a warm-up window.
    python tools/layout_pmc.py <nonce_len>      (GPU box only; DPOW_LIB_PATH selects a build)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-proof-of-work_amd"))
import torch  # noqa: F401
import distpow
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K0, NK = 1 << 24, (1 << 33) >> 8
with distpow.Miner(0) as m:
    m.search([0x5A] * n, 32, 0, 0, K0, K0 + NK)
    m.reset_stats()
    m.search([0x5A] * n, 32, 0, 0, K0 + NK, K0 + 2 * NK)
    st = m.stats()
    print(n, round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2))
