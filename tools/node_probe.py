#!/usr/bin/env python3
"""Time-to-secret of node_mine's batch schedules, one rank emulated on one GPU.

    python tools/node_probe.py [runs]

For a node of G GPUs the time to the answer is the time the rank owning the answer
(owner = (g & 255) >> (8 - log2 G)) takes to reach it: its own first hit is the node's
answer (the min rule), and the other ranks only have to finish the same batches.  This
runs that rank alone (world = G, no process group: no all-reduce, but the per-batch
host <-> device copies of the all-reduce buffer do run) for the bench's time-to-secret
configs, with the growing schedule (2^8 k, x4, cap 2^29 candidates; round 2's first) and
the expected-time schedule (node.auto_batch_candidates).  It also measures the fixed
per-batch cost c of this loop (tiny batches at N = 32).  An 8-GPU node adds one RCCL
all-reduce of 16 bytes per batch on top.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))

import torch  # noqa: E402

import distpow  # noqa: E402
from distpow.node import auto_batch_candidates, node_mine, owner_rank  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")))
    want = [([1, 2, 3, 4], 3), ([1, 2, 3, 4], 6), ([1, 2, 3, 4], 7), ([1, 2, 3, 4], 8), ([2, 2, 2, 2], 8),
            ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5)]
    exp = {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in gold["first_hits"] + gold["deep_hits"]}
    want += [(list(n), 9) for (n, z) in exp if z == 9 and n not in ((1, 2, 3, 4), (5, 6, 7, 8), (2, 2, 2, 2))]
    dev = torch.device("cuda", 0)
    out = {"per_batch_cost_ms": {}, "tts_ms": {}}
    with distpow.Miner(0) as m:
        search = lambda *a: m.search(*a[:6], bound=a[6])  # noqa: E731
        m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        for G in (1, 8):
            nb = 200
            t = time.perf_counter()
            r = node_mine(search, [1, 2, 3, 4], 32, 0, G, batch_k=1 << 6, growth=1, k_start=1 << 24,
                          k_limit=(1 << 24) + nb * (1 << 6), device=dev)
            assert r.status == distpow.EXHAUSTED and r.batches == nb
            out["per_batch_cost_ms"][f"G{G}"] = round((time.perf_counter() - t) * 1e3 / nb, 4)
        for G in (1, 2, 4, 8):
            for nonce, n in want:
                g = exp[(tuple(nonce), n)]
                o = owner_rank(g, G)
                row = {"global_idx": g, "owner": o,
                       "auto_batch_candidates": auto_batch_candidates(n, G)}
                for name, kw in (("grow", {"batch_k": 1 << 8}), ("auto", {})):
                    ts, nb = [], 0
                    for _ in range(runs):
                        torch.cuda.synchronize()
                        t = time.perf_counter()
                        r = node_mine(search, nonce, n, o, G, device=dev, **kw)
                        ts.append((time.perf_counter() - t) * 1e3)
                        assert r.status == distpow.FOUND and r.global_idx == g, (nonce, n, G, name, r)
                        nb = r.batches
                    row[name] = {"ms": round(sorted(ts)[len(ts) // 2], 3), "batches": nb}
                out["tts_ms"][f"G{G} {bytes(nonce).hex()}/{n}"] = row
                print(f"G{G} {bytes(nonce).hex()}/{n}: grow {row['grow']['ms']} ms ({row['grow']['batches']} b), "
                      f"auto {row['auto']['ms']} ms ({row['auto']['batches']} b)", file=sys.stderr, flush=True)
        # Every rank of the node (sync schedule): a rank hashes its batches up to and
        # including the one that holds the answer, or stops at its own first hit in it;
        # the node's time is the slowest rank's (plus one all-reduce per batch).
        out["node_ms"] = {}
        for G in (2, 8):
            for nonce, n in want:
                g = exp[(tuple(nonce), n)]
                rb = 8 - (G.bit_length() - 1)
                bk = max(1, auto_batch_candidates(n, G) >> rb)
                k_lim = ((g >> 8) // bk + 1) * bk
                per_rank = []
                for r in range(G):
                    ts = []
                    for _ in range(runs):
                        torch.cuda.synchronize()
                        t = time.perf_counter()
                        res = node_mine(search, nonce, n, r, G, device=dev, k_limit=k_lim)
                        ts.append((time.perf_counter() - t) * 1e3)
                        assert res.status in (distpow.FOUND, distpow.EXHAUSTED)
                        assert res.status != distpow.FOUND or res.global_idx >= g
                    per_rank.append(round(sorted(ts)[len(ts) // 2], 3))
                key = f"G{G} {bytes(nonce).hex()}/{n}"
                out["node_ms"][key] = {"max_rank_ms": max(per_rank), "owner_ms": per_rank[owner_rank(g, G)],
                                       "per_rank_ms": per_rank}
                print(f"node {key}: slowest rank {max(per_rank)} ms, owner {per_rank[owner_rank(g, G)]} ms",
                      file=sys.stderr, flush=True)
    out["build_id"] = distpow.build_id()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
