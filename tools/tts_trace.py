#!/usr/bin/env python3
"""Launch timeline of single-GPU time-to-secret (Miner.mine): run under
rocprofv3 --kernel-trace, it brackets each search with host timestamps (printed as
JSON) so tools/tts_timeline.py can line the kernel trace up with them."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import torch  # noqa: E402,F401

import distpow  # noqa: E402

cases = [([1, 2, 3, 4], 3), ([1, 2, 3, 4], 6), ([1, 2, 3, 4], 7), ([2, 2, 2, 2], 8), ([1, 2, 3, 4], 8)]
out = []
with distpow.Miner(0) as m:
    m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
    for nonce, n in cases:
        for rep in range(3):
            torch.cuda.synchronize()
            m.reset_stats()
            t0 = time.perf_counter_ns()
            r = m.mine(nonce, n)
            t1 = time.perf_counter_ns()
            st = m.stats()
            out.append({"case": f"{bytes(nonce).hex()}/{n}", "rep": rep, "ms": (t1 - t0) / 1e6,
                        "t0_ns": t0, "t1_ns": t1,
                        "g": r.global_idx, "launches": st.launches, "kernel_ms": st.kernel_ms,
                        "candidates": st.candidates})
            time.sleep(0.01)
print(json.dumps(out, indent=1))
