#!/usr/bin/env python3
"""Randomised soak of the coordinator protocol in node mode (test infrastructure: not collected
by pytest).  GPU box only.

    python tests/soak/coordinator_soak.py [seconds] [seed]

Rounds of random requests -- nonce lengths 1..70 (one- and two-block layouts), N = 1..5 (6 on
one request in ten: the oracle's scalar search bounds the rate),
W = 2, 4, 8 workers, the shared-GPU role (rank 0 searches for the node) and the per-rank role
(DPOW_DIAG_BOARD_SPLIT=1), and two clients at once -- through `Coordinator` (the reference's
coordinator.go:139-298 over native workers on a node board).  Every answer must equal the
oracle's workerBits = 0 first hit (worker.go:301-400, oracle/dpow_oracle.c) for the same nonce
and N, be reported by the owner of its index alone, and leave no task on the board.  Prints one
JSON line (progress on stderr every 30 s).
"""
import json
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402
import distpow  # noqa: E402
from _oracle import Oracle  # noqa: E402
from distpow.coordinator import Coordinator  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rnd = random.Random(seed)
o = Oracle()
cases = bad = tok = 0
failures = []
by = {}
t_end = time.time() + secs
t_log = time.time() + 30
while time.time() < t_end:
    W = rnd.choice((2, 4, 8))
    split = rnd.random() < 0.5
    if split:
        os.environ["DPOW_DIAG_BOARD_SPLIT"] = "1"
    else:
        os.environ.pop("DPOW_DIAG_BOARD_SPLIT", None)
    seen = set()  # fresh nonces per coordinator: no cache hit stands in for a search
    with Coordinator(W) as c:
        for _ in range(8):  # 8 rounds per coordinator, two clients each
            reqs = []
            while len(reqs) < 2:
                nonce = [rnd.randrange(256) for _ in range(rnd.randrange(1, 71))]
                if bytes(nonce) in seen:
                    continue
                seen.add(bytes(nonce))
                reqs.append((nonce, 6 if rnd.random() < 0.1 else rnd.randrange(1, 6)))
            out = {}

            def client(i, nonce, n, token):
                try:
                    out[i] = c.mine(nonce, n, token=token)
                except Exception as e:  # recorded as a failure below
                    out[i] = e

            th = []
            for i, (nonce, n) in enumerate(reqs):
                tok += 1
                th.append(threading.Thread(target=client, args=(i, nonce, n, tok)))
                reqs[i] = (nonce, n, tok)
            for t in th:
                t.start()
            for t in th:
                t.join(120)
            trace = c.trace()
            for i, (nonce, n, token) in enumerate(reqs):
                cases += 1
                key = f"W{W}_{'split' if split else 'shared'}"
                by[key] = by.get(key, 0) + 1
                want = o.mine_window(nonce, n, 0, 0, 0, 1 << 20)
                got = out.get(i)
                ok = isinstance(got, bytes) and want is not None and list(got) == want[0]
                # node mode: the owner of the minimum index alone sends a WorkerResult
                res = [t["WorkerByte"] for t in trace
                       if t["trace"] == token and t["action"] == "CoordinatorWorkerResult"]
                wbits = W.bit_length() - 1
                owner = (want[1] & 255) >> (8 - wbits) if want is not None else None
                if not ok or res != [owner]:
                    bad += 1
                    if len(failures) < 20:
                        failures.append({"W": W, "split": split, "nonce": nonce, "ntz": n,
                                         "got": repr(got), "want": want, "results_from": res})
            if c.board.tasks() != 0:
                bad += 1
                failures.append({"W": W, "split": split, "board_tasks_left": c.board.tasks()})
            dropped = [t for t in trace if t["action"] == "CoordinatorDroppedResult"]
            if dropped:
                bad += 1
                failures.append({"W": W, "split": split, "dropped": len(dropped)})
                break
    if time.time() > t_log:
        print(json.dumps({"cases": cases, "bad": bad}), file=sys.stderr, flush=True)
        t_log = time.time() + 30
print(json.dumps({"build_id": distpow.build_id(), "seconds": secs, "seed": seed, "cases": cases, "bad": bad,
                  "by_mode": by, "failures": failures}))
