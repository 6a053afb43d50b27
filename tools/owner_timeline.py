#!/usr/bin/env python3
"""Host timeline of an 8-GPU node rank's search (tools/node_probe.py's owner, one GPU):
where node_mine's time goes beyond the kernels.

    python3 tools/owner_timeline.py [G,...] > gpurun_out/<tag>/owner_timeline.json

Per case (median of 7): node_mine's wall time; inside it, the time to the search call, the
search call (Miner.search -> dpow_search), and after it; dpow_search's own timeline
(dpow_diag_search_times: first launch planned, k = 0 kernel queued, first md5 launch
queued, first completion record seen, done); the launches' kernel time from their records;
and one plain Miner.search over the same window for comparison.  GPU box only."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import torch  # noqa: E402

import distpow  # noqa: E402
from distpow.node import BOARD_BATCH_CANDIDATES, NodeBoard, node_mine, owner_rank  # noqa: E402

CASES = [([1, 2, 3, 4], 6, 2532284), ([1, 2, 3, 4], 7, 231910082), ([2, 2, 2, 2], 8, 293615578),
         ([1, 2, 3, 4], 3, 97), ([5, 6, 7, 8], 5, None), ([2, 2, 2, 2], 5, None)]
RUNS = 7


def med(v):
    return round(sorted(v)[len(v) // 2], 4)


def main():
    lib = distpow.lib()
    board = NodeBoard.local()
    warm = NodeBoard.local()
    out = {"build_id": distpow.build_id(), "cases": {}}
    gs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [8]
    with distpow.Miner(0) as m:
        m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        tl = (ctypes.c_int64 * 8)()
        gold = json.load(open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")))
        exp = {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in gold["first_hits"]}
        # one GPU (Miner.mine, as bench.py's N = 1 time-to-secret) with its dpow_search timeline
        for nonce, n, g in CASES:
            ms, tls = [], []
            for _ in range(RUNS):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = m.mine(nonce, n)
                ms.append((time.perf_counter() - t0) * 1e3)
                lib.dpow_diag_search_times(m._ctx, tl)
                tls.append([round(x / 1e3, 1) for x in tl])
            key = f"G1 {bytes(nonce).hex()}/{n}"
            out["cases"][key] = {"mine_ms": med(ms), "dpow_timeline_us": tls[len(tls) // 2]}
            print(key, json.dumps(out["cases"][key]), file=sys.stderr, flush=True)
        for G, (nonce, n, g) in [(G, c) for G in gs for c in CASES]:
            g = exp[(tuple(nonce), n)] if g is None else g
            o = owner_rank(g, G)
            rec = {"node_mine_ms": [], "to_search_ms": [], "search_ms": [], "after_ms": [], "kernel_ms": [],
                   "launches": [], "dpow_timeline_us": [], "plain_search_ms": [], "plain_kernel_ms": []}
            for _ in range(RUNS):
                stamps = {}

                def search(*a):
                    stamps["s0"] = time.perf_counter()
                    r = m.search(*a[:6], bound=a[6])
                    stamps["s1"] = time.perf_counter()
                    return r
                torch.cuda.synchronize()
                m.reset_stats()
                t0 = time.perf_counter()
                r = node_mine(search, nonce, n, o, G, board=board, attach_fn=m.attach_node)
                t1 = time.perf_counter()
                assert r.global_idx == g
                st = m.stats()
                lib.dpow_diag_search_times(m._ctx, tl)
                rec["node_mine_ms"].append((t1 - t0) * 1e3)
                rec["to_search_ms"].append((stamps["s0"] - t0) * 1e3)
                rec["search_ms"].append((stamps["s1"] - stamps["s0"]) * 1e3)
                rec["after_ms"].append((t1 - stamps["s1"]) * 1e3)
                rec["kernel_ms"].append(st.kernel_ms)
                rec["launches"].append(st.launches)
                rec["dpow_timeline_us"].append([round(x / 1e3, 1) for x in tl])
                # the same window as one plain search (no node_mine, no board)
                rbits = 8 - (G.bit_length() - 1)
                torch.cuda.synchronize()
                m.reset_stats()
                t0 = time.perf_counter()
                r2 = m.search(nonce, n, o, G.bit_length() - 1, 0, BOARD_BATCH_CANDIDATES >> rbits)
                rec["plain_search_ms"].append((time.perf_counter() - t0) * 1e3)
                rec["plain_kernel_ms"].append(m.stats().kernel_ms)
                assert r2.global_idx == g
            key = f"G{G} owner {bytes(nonce).hex()}/{n}"
            out["cases"][key] = {k: (med(v) if k != "dpow_timeline_us" else v[len(v) // 2]) if k != "launches" else v[0]
                                 for k, v in rec.items()}
            print(key, json.dumps(out["cases"][key]), file=sys.stderr, flush=True)
            # a non-owner, the owner's hit posted to its slot when the owner posted it (node_probe.py)
            t_post = med([a + b / 1e3 for a, b in zip(rec["to_search_ms"],
                                                      [tl_[7] if tl_[7] >= 0 else 1e9 for tl_ in rec["dpow_timeline_us"]])])
            non = (o + 1) % G
            nrec = {"node_mine_ms": [], "to_search_ms": [], "search_ms": [], "after_ms": [], "kernel_ms": [],
                    "launches": [], "dpow_timeline_us": []}
            for _ in range(RUNS):
                stamps = {}

                def search2(*a):
                    stamps["s0"] = time.perf_counter()
                    r = m.search(*a[:6], bound=a[6])
                    stamps["s1"] = time.perf_counter()
                    return r
                slot = board.begin()
                lib.dpow_diag_node_post_at(warm.slot(0), 0, 0)  # the poster thread running before the clock
                torch.cuda.synchronize()
                m.reset_stats()
                t0 = time.perf_counter()
                lib.dpow_diag_node_post_at(slot, g, time.perf_counter_ns() + int(t_post * 1e6))
                t0b = time.perf_counter()
                r = node_mine(search2, nonce, n, non, G, board=board, attach_fn=m.attach_node)
                t1 = time.perf_counter()
                assert r.global_idx == g
                st = m.stats()
                lib.dpow_diag_search_times(m._ctx, tl)
                nrec["node_mine_ms"].append((t1 - t0) * 1e3)
                nrec["to_search_ms"].append((stamps["s0"] - t0) * 1e3)
                nrec["search_ms"].append((stamps["s1"] - stamps["s0"]) * 1e3)
                nrec["after_ms"].append((t1 - stamps["s1"]) * 1e3)
                nrec["kernel_ms"].append(st.kernel_ms)
                nrec["launches"].append(st.launches)
                nrec["dpow_timeline_us"].append([round(x / 1e3, 1) for x in tl] + [round((t0b - t0) * 1e6, 1)])
            key = f"G{G} non-owner {bytes(nonce).hex()}/{n}"
            out["cases"][key] = {k: (med(v) if k != "dpow_timeline_us" else v[len(v) // 2]) if k != "launches" else v[0]
                                 for k, v in nrec.items()}
            out["cases"][key]["post_ms"] = round(t_post, 4)
            print(key, json.dumps(out["cases"][key]), file=sys.stderr, flush=True)
    out["note"] = ("dpow_timeline_us: [0] k0 queued, [1] first md5 queued, [2] first record seen, [3] done, "
                   "[4] first launch planned, [5] k0 slot retired, [6] md5 slot retired, [7] early hit posted "
                   "(us from dpow_search's start); non-owner: [8] the poster thread's creation (us); post_ms: "
                   "the owner's post, from its node_mine start")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
