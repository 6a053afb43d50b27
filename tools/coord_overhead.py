#!/usr/bin/env python3
"""Where a coordinator request's time goes when the search itself is tiny (N = 5 on fresh
nonces, ~25 us of hashing): the coordinator mirror's phases (coordinator.go:139-298) timed from
the request's start -- the Mine fan-out to the W workers returned, the first result received,
the Found fan-out returned, the 2W-th message received -- next to one Miner.mine of the same
nonce.  Node mode (the workers on a board) and the first-arrived race.  GPU box only.
    python3 tools/coord_overhead.py [W] [n_nonces] > gpurun_out/<tag>/overhead.json"""
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import distpow  # noqa: E402
from distpow import coordinator as C  # noqa: E402


class Timed(C.Coordinator):
    """The mirror with phase stamps (the protocol unchanged)."""

    def mine(self, nonce, num_trailing_zeros, token=None):
        self.stamps = {"t0": time.perf_counter()}
        return super().mine(nonce, num_trailing_zeros, token)

    def _get(self, q, ack_phase=False):
        r = super()._get(q, ack_phase)
        key = "acks_done" if ack_phase else "first_result"
        self.stamps[key] = time.perf_counter()
        return r

    def _record(self, token, action, **fields):
        super()._record(token, action, **fields)
        if action == "CoordinatorWorkerMine" and fields.get("WorkerByte") == len(self.workers) - 1:
            self.stamps["last_mine_call"] = time.perf_counter()
        if action == "CoordinatorWorkerCancel" and fields.get("WorkerByte") == 0:
            self.stamps.setdefault("found_fanout_start", time.perf_counter())
        if action == "CoordinatorSuccess":
            self.stamps["success"] = time.perf_counter()


W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
rng = random.Random(7)
nonces = [[rng.randrange(256) for _ in range(4)] for _ in range(n)]
out = {"build_id": distpow.build_id(), "W": W, "ntz": 5}
with distpow.Miner(0) as m:
    ms = []
    for nonce in nonces:
        t = time.perf_counter()
        m.mine(nonce, 5)
        ms.append((time.perf_counter() - t) * 1e3)
    out["miner_mine_ms"] = round(statistics.median(ms), 3)
for mode in ("node", "first"):
    phases = {}
    with Timed(W, node=(mode == "node")) as c:
        c.mine([9, 9, 9, 9], 5)  # warm
        for nonce in nonces:
            c.mine(nonce, 5)
            t0 = c.stamps["t0"]
            for k, v in c.stamps.items():
                if k != "t0":
                    phases.setdefault(k, []).append((v - t0) * 1e3)
    out[mode] = {k: round(statistics.median(v), 3) for k, v in phases.items()}
    print(mode, json.dumps(out[mode]), file=sys.stderr, flush=True)
print(json.dumps(out))
