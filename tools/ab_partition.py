#!/usr/bin/env python3
"""A/B of libdpow builds on the multi-GPU ranks' partitions: tools/ab_partition.py lib1.so lib2.so ...
Each library in its own process, two interleaved rounds; kernel GH/s of a 2^35-candidate window
of the bench sweep (nonce [1,2,3,4], N = 32, L = 4 segment) at workerBits 0 and 3, whose launches
are 2^32 and 2^29 candidates (the host splits windows at every 2^24 k)."""
import json, os, subprocess, sys

CHILD = r"""
import os, sys, json
sys.path.insert(0, os.path.join(os.environ["ROOT"], "distributed-proof-of-work_amd"))
import distpow
m = distpow.Miner(0)
m.search([1,2,3,4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 24))   # warm the clock
out = {}
for wbits, wb in ((3, 5), (0, 0), (3, 0)):
    nk = (1 << 35) >> (8 - wbits)
    m.reset_stats()
    m.search([1,2,3,4], 32, wb, wbits, 1 << 25, (1 << 25) + nk)
    st = m.stats()
    out[f"wbits{wbits}/wb{wb}"] = round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2)
print(json.dumps(out))
"""

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {l: [] for l in sys.argv[1:]}
for rnd in range(2):
    for l in sys.argv[1:]:
        env = dict(os.environ, DPOW_LIB_PATH=os.path.abspath(l), ROOT=root)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            print(l, "FAILED", r.stderr[-1500:], flush=True)
            sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        res[l].append(d)
        print(rnd, l, json.dumps(d), flush=True)
