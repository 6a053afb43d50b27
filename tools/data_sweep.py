#!/usr/bin/env python3
"""Does the sweep rate of one kernel layout depend on the data hashed?  (GPU box only.)

    python tools/data_sweep.py [log2_candidates]

Hashes 2^n candidates (default 2^34) at N = 32 in the L = 4 segment for several nonces
of the same length (so the same kernel <NBLK, W0, SH>), interleaved over 3 rounds, and
prints kernel GH/s per nonce and round.  A spread between nonces of one layout is a
property of the data (switching activity -> power -> clock), not of the code, and bounds
how finely layouts can be compared.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "distributed-proof-of-work_amd"))
import torch  # noqa: F401,E402
import distpow  # noqa: E402

LOG2 = int(sys.argv[1]) if len(sys.argv) > 1 else 34
K0 = 1 << 24
NK = (1 << LOG2) >> 8
NONCES = {
    "len0": [], "len64_5a": [0x5A] * 64, "len64_00": [0] * 64, "len64_ff": [0xFF] * 64,
    "len4_01020304": [1, 2, 3, 4], "len4_5a": [0x5A] * 4, "len4_00": [0] * 4, "len4_ff": [0xFF] * 4,
    "len4_810396a1": [129, 3, 150, 161],
    "len1_5a": [0x5A], "len1_00": [0], "len5_5a": [0x5A] * 5, "len5_00": [0] * 5,
}
out = {k: [] for k in NONCES}
with distpow.Miner(0) as m:
    m.search([1, 2, 3, 4], 32, 0, 0, K0, K0 + NK)  # warm
    for rnd in range(3):
        for name, nonce in NONCES.items():
            m.reset_stats()
            r = m.search(nonce, 32, 0, 0, K0 + rnd * NK, K0 + (rnd + 1) * NK)
            assert r.status == distpow.EXHAUSTED
            st = m.stats()
            out[name].append(round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2))
        print(rnd, json.dumps(out), flush=True)
lay = {name: "<{0.nblk},{0.w0},{0.sh}>".format(distpow.plan_window(n, 0, 0, K0, K0 + 1)[0])
       for name, n in NONCES.items()}
print(json.dumps({name: {"layout": lay[name], "ghs": v} for name, v in out.items()}))
