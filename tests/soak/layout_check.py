#!/usr/bin/env python3
"""Correctness sweep over every message layout (GPU box only; test infrastructure under
tests/ because it loads the oracle, not collected by pytest): for nonce lengths
0..130 (every (NBLK, W0, SH) layout, midstate and two-block cases), search windows in
every chunk-length segment at N = 1..3 and compare with the byte-wise oracle; prints
the failing (length, layout, window) cases, exit 1 if any.  Quicker to localise a
layout bug than the parity suite, which stops at the first mismatch."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import distpow  # noqa: E402
from _oracle import Oracle  # noqa: E402

o = Oracle()
bad = []
rnd = random.Random(5)
with distpow.Miner(0) as m:
    for n in list(range(0, 72)) + [100, 119, 120, 127, 128, 130]:
        nonce = [rnd.randrange(256) for _ in range(n)]
        for k0, nk in ((0, 300), (300, 200), (70000, 64), ((1 << 24) - 5, 40), ((1 << 24) + 999, 40),
                       ((1 << 32) - 3, 30), ((1 << 32) + 77, 30)):
            for ntz in (1, 2, 3):
                wbits = rnd.choice([0, 0, 3, 8])
                wb = rnd.randrange(1 << wbits) if wbits else 0
                exp = o.mine_window(nonce, ntz, wb, wbits, k0, k0 + nk)
                try:
                    r = m.search(nonce, ntz, wb, wbits, k0, k0 + nk)
                    got = None if r.status != distpow.FOUND else (list(r.secret), r.global_idx)
                except distpow.DpowError as e:
                    got = f"error {e.code}"
                want = None if exp is None else (exp[0], exp[1])
                if got != want:
                    p = distpow.plan_window(nonce, wb, wbits, k0, k0 + 1)[0]
                    bad.append({"len": n, "layout": [p.nblk, p.w0, p.sh], "k0": k0, "ntz": ntz, "wbits": wbits,
                                "got": str(got), "want": str(want)})
print(json.dumps({"bad": bad[:60], "n_bad": len(bad)}))
sys.exit(1 if bad else 0)
