#!/usr/bin/env python3
"""Randomised parity soak of the GPU search against the C oracle (test infrastructure:
lives under tests/ because it loads the oracle; not collected by pytest).

    python tests/soak/parity_soak.py [seconds] [seed] [span|long]

Random nonce lengths (0..130, every kernel layout), partitions (workerBits 0..10),
windows (every chunk-length segment, straddling segment / 2^24 boundaries) and
trailing-zero counts (1..5); every GPU answer must equal the oracle's first hit
(or "no hit").  Prints one JSON line with the case count (progress on stderr every
30 s).  GPU box only.

With "span" every case is a window across one or more 2^24-k segment boundaries
(the segment-word path of launches that span segments): workerBits 5..8 (8..1
thread bytes per k), up to ~2^20 candidates, L = 4 and 5.  With "long" every window
has 6- or 7-byte chunks (k from 2^40 to DPOW_K_LIMIT), at and across the launch splits
there (2^24-k segments, word W0+2's period for SH 1-2, 2^48).
"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import distpow  # noqa: E402
from _oracle import Oracle  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
span = len(sys.argv) > 3 and sys.argv[3] == "span"
long_k = len(sys.argv) > 3 and sys.argv[3] == "long"  # 6- and 7-byte chunks only (k >= 2^40)
rnd = random.Random(seed)
o = Oracle()
n_cases = hits = 0
t_end = time.time() + secs
t_log = time.time() + 30
with distpow.Miner(0) as m:
    while time.time() < t_end:
        nlen = rnd.randrange(131)
        nonce = [rnd.randrange(256) for _ in range(nlen)]
        wbits = rnd.choice([0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
        wb = rnd.randrange(1 << (wbits % 9)) if wbits % 9 else rnd.randrange(256)
        rb = 8 - wbits % 9
        ntz = rnd.choice([1, 2, 3, 3, 4, 4, 5])
        seg = rnd.choice([0, 1, 2, 3, 4, 5])
        k0 = rnd.randrange(1 << (8 * seg)) if seg else 0
        if seg >= 2 and rnd.random() < 0.3:
            k0 = max(0, (1 << (8 * seg)) - rnd.randrange(1, 64))
        if seg >= 4 and rnd.random() < 0.3:
            k0 = max(0, ((k0 >> 24) + 1 << 24) - rnd.randrange(1, 64))
        nk = max(1, rnd.randrange(1, 1 + (1 << 17) // (1 << rb)))
        if span:  # straddle 1..3 segment boundaries of L = 4 or 5
            wbits = rnd.choice([5, 6, 7, 8])
            wb = rnd.randrange(1 << wbits)
            rb = 8 - wbits
            edge = rnd.choice([rnd.randrange(2, 255), rnd.randrange(257, 1 << 16)]) << 24
            nk = rnd.randrange(2, (1 << 20) >> rb)
            k0 = edge - rnd.randrange(1, nk)
            if rnd.random() < 0.3:  # a window over whole segments
                nk += rnd.randrange(1, 3) << 24 if rb == 0 else 0
            ntz = rnd.choice([3, 4, 4, 5, 5])
        if long_k:  # L = 6 / 7, at and across 2^24-k segments, word W0+2's splits (SH 1-2) and 2^48
            top = distpow.DPOW_K_LIMIT
            edge = rnd.choice([1 << 40, 1 << 48, rnd.randrange(2, 256) << 40, rnd.randrange(2, 128) << 48,
                               rnd.randrange(1 << 16, 1 << 31) << 24, rnd.randrange(1 << 40, top)])
            k0 = min(top - 1, max(1 << 40, edge - rnd.randrange(0, nk + 1)))
        k1 = min(k0 + nk, distpow.DPOW_K_LIMIT)
        exp = o.mine_window(nonce, ntz, wb, wbits, k0, k1)
        r = m.search(nonce, ntz, wb, wbits, k0, k1)
        case = (nlen, nonce[:8], ntz, wb, wbits, k0, k1)
        if exp is None:
            assert r.status == distpow.EXHAUSTED, (case, r)
        else:
            assert r.status == distpow.FOUND and (list(r.secret), r.global_idx) == (exp[0], exp[1]), (case, r, exp)
            hits += 1
        n_cases += 1
        if time.time() >= t_log:  # progress line: a silent run looks hung to the GPU harness
            print(f"... {n_cases} cases, {hits} hits", file=sys.stderr, flush=True)
            t_log += 30
print(json.dumps({"cases": n_cases, "hits": hits, "seed": seed, "seconds": secs, "span": span, "long": long_k}))
