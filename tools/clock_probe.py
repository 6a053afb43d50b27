#!/usr/bin/env python3
"""Small launches after idle gaps (run under rocprofv3 --pmc GRBM_GUI_ACTIVE ...): the L = 2
segment window (16.7 M candidates, N = 32) after 0 / 1 / 10 / 100 ms of idle, and right
after a long launch, to see whether a short launch runs at a lower clock."""
import json, os, sys, time
sys.path.insert(0, "distributed-proof-of-work_amd")
import torch  # noqa: F401
import distpow
m = distpow.Miner(0)
out = []
m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
for gap in (0.0, 0.001, 0.01, 0.1, 0.0, 0.001, 0.01, 0.1):
    time.sleep(gap)
    m.reset_stats()
    m.search([1, 2, 3, 4], 32, 0, 0, 256, 65536)
    st = m.stats()
    out.append({"gap_ms": gap * 1e3, "kernel_us": round(st.kernel_ms * 1e3, 1)})
print(json.dumps(out))
