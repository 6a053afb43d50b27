#!/usr/bin/env python3
"""Time-to-secret of a G-GPU node, emulated rank by rank on one GPU.

    python tools/node_probe.py [runs] [G,...] [small] > profiles/<round>_node_probe.json

node_mine with the node board (NodeBoard: the shared-memory Found fan-out,
dpow_node_slot): every rank searches its partition of the same window; the rank that
owns the answer (owner = (g & 255) >> (8 - log2 G)) posts it to the board the moment
its search returns, and every other rank's running search takes it as its bound and
stops.  The node's time is therefore the slowest rank's: the owner's time to its own
hit, or a non-owner's time to notice the posted hit and drain.  This runs

  1. the owner alone (world = G, no process group): t_owner;
  2. every other rank alone, with a native thread (dpow_diag_node_post_at) that posts the
     owner's hit to the board slot when the owner's search posted it (its dpow_search
     returning FOUND, measured in step 1), counted from the rank's own start, as the
     owner's process would;

and reports max over ranks, next to one GPU's Miner.mine (G1).  node_mine runs here
without a process group or a shared board, so its batch boundary is a no-op on the host
(no tensors, no collective): the real node adds one node vote per batch on a shared board
(NodeBoard), measured on this host by dpow_diag_vote_latency -- G threads on CPUs spread over
the process's affinity set, the last rank voting after the others wait in the vote: the time
until every rank holds the result (round 4 added a constant 3.5 us, the 2-rank rehearsal's
median of a Python-level vote after a gloo barrier).  Across hosts it is one RCCL all-reduce
(33 us at world 1).  The ranks run one after another, each with the whole GPU; the 8-GPU
number itself is the driver's (bench.py --gpus 8).
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))

import torch  # noqa: E402

import distpow  # noqa: E402
from distpow.node import NodeBoard, node_mine, owner_rank  # noqa: E402


# DPOW_NODE_VOTE_US: a fixed node-vote cost instead of the measured one (round 4: 3.5)
VOTE_US_FIXED = os.environ.get("DPOW_NODE_VOTE_US")
# The rank's search through the native loop (dpow_node_mine, as bench.py runs it) unless
# DPOW_NODE_PY=1 (round 4's Python loop over Miner.search).
NATIVE = os.environ.get("DPOW_NODE_PY") != "1"


def med(v):
    return round(sorted(v)[len(v) // 2], 3)


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    gs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2, 4, 8]
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")))
    want = [([1, 2, 3, 4], 3), ([1, 2, 3, 4], 6), ([1, 2, 3, 4], 7), ([1, 2, 3, 4], 8), ([2, 2, 2, 2], 8),
            ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5)]
    exp = {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in gold["first_hits"] + gold["deep_hits"]}
    if not (len(sys.argv) > 3 and sys.argv[3] == "small"):  # "small": the cases up to N = 8 only
        want += [(list(n), 9) for (n, z) in exp if z == 9 and n not in ((1, 2, 3, 4), (5, 6, 7, 8), (2, 2, 2, 2))]
    out = {"note": __doc__.strip().splitlines()[0], "g1_ms": {}, "node_ms": {}}
    board = NodeBoard.local()
    lib = distpow.lib()
    # the node vote's cost per G on this host (the slowest rank's time + it = the node's)
    vote_ms = {}
    for G in gs:
        if VOTE_US_FIXED:
            vote_ms[G] = float(VOTE_US_FIXED) / 1e3
            continue
        last, all_ = ctypes.c_double(), ctypes.c_double()
        assert lib.dpow_diag_vote_latency(G, 400, ctypes.byref(last), ctypes.byref(all_)) == 0, \
            lib.dpow_last_error().decode()
        vote_ms[G] = all_.value / 1e3
    out["vote_us"] = {str(G): round(v * 1e3, 3) for G, v in vote_ms.items()}
    with distpow.Miner(0) as m:
        search = lambda *a: m.search(*a[:6], bound=a[6])  # noqa: E731
        m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        for nonce, n in want:
            ts = []
            for _ in range(runs):
                torch.cuda.synchronize()
                t = time.perf_counter()
                r = m.mine(nonce, n)
                ts.append((time.perf_counter() - t) * 1e3)
                assert r.global_idx == exp[(tuple(nonce), n)]
            out["g1_ms"][f"{bytes(nonce).hex()}/{n}"] = med(ts)

        found_at = {}
        tl = (ctypes.c_int64 * 8)()

        def search_timed(*a):
            t_call = time.perf_counter_ns() / 1e9
            r = search(*a)
            if r.status == distpow.FOUND:
                # when the owner's hit reached the node slot: the early Found fan-out (its
                # watcher relays the hit, the host verifies and posts it while the launch
                # drains: dpow_diag_search_times[7], ns from dpow_search's start, which follows
                # t_call by the ctypes call -- so this errs early by ~1-2 us), else dpow_search's
                # own post just before it returned
                lib.dpow_diag_search_times(m._ctx, tl)
                found_at["t"] = t_call + tl[7] / 1e9 if tl[7] >= 0 else time.perf_counter_ns() / 1e9
            return r

        warm = NodeBoard.local()

        def run_rank(nonce, n, rank, G, post_after_s=None, g=None):
            slot = board.begin()
            lib.dpow_diag_node_post_at(warm.slot(0), 0, 0)  # the poster thread running before the clock
            torch.cuda.synchronize()
            found_at.clear()
            t0 = time.perf_counter_ns()  # CLOCK_MONOTONIC
            if post_after_s is not None:
                # the owner's process posts its hit at t0 + post_after_s: a native thread, off
                # this interpreter (a Python poster thread took the GIL and its start alone
                # cost the rank 50-100 us; round 3 created a native thread per post, on the
                # clock; now one queues a request for a poster already running)
                lib.dpow_diag_node_post_at(slot, g, t0 + int(post_after_s * 1e9))
            if NATIVE:  # the native loop (dpow_node_mine): one call; the post from the last search's timeline
                res = node_mine(None, nonce, n, rank, G, board=board, miner=m)
                dt = (time.perf_counter_ns() - t0) / 1e9
                if res.status == distpow.FOUND and res.global_idx != distpow.DPOW_NO_HIT:
                    lib.dpow_diag_search_times(m._ctx, tl)
                    if tl[7] >= 0:  # errs early by the call's entry (~1 us), as search_timed's t_call
                        found_at["t"] = t0 / 1e9 + tl[7] / 1e9
            else:
                res = node_mine(search_timed, nonce, n, rank, G, board=board, attach_fn=m.attach_node)
                dt = (time.perf_counter_ns() - t0) / 1e9
            t_post = found_at.get("t", t0 / 1e9 + dt) - t0 / 1e9
            return res, dt, t_post

        for G in gs:
            for nonce, n in want:
                g = exp[(tuple(nonce), n)]
                o = owner_rank(g, G)
                t_own, t_posts = [], []
                for _ in range(runs):
                    res, dt, tp = run_rank(nonce, n, o, G)
                    assert res.status == distpow.FOUND and res.global_idx == g, (nonce, n, G, res)
                    t_own.append(dt)
                    t_posts.append(tp)
                t_o = sorted(t_own)[len(t_own) // 2]
                t_p = sorted(t_posts)[len(t_posts) // 2]  # when the owner's search posted its hit
                per_rank = []
                for r in range(G):
                    if r == o:
                        per_rank.append(round(t_o * 1e3, 3))
                        continue
                    ts = []
                    for _ in range(runs):
                        res, dt, _ = run_rank(nonce, n, r, G, post_after_s=t_p, g=g)
                        # bounded by the posted hit (EXHAUSTED of this rank's batch -> no
                        # process group: node_mine reports the rank's own status), never a
                        # hit above it
                        assert res.status in (distpow.FOUND, distpow.EXHAUSTED), res
                        # (its own first hit, above g, when it found one before the post
                        # arrived: the node's vote then takes g, the owner's)
                        assert res.status != distpow.FOUND or res.global_idx >= g
                        ts.append(dt * 1e3)
                    per_rank.append(med(ts))
                key = f"G{G} {bytes(nonce).hex()}/{n}"
                g1 = out["g1_ms"][f"{bytes(nonce).hex()}/{n}"]
                node = max(per_rank) + vote_ms[G]  # the slowest rank plus the node's one vote
                out["node_ms"][key] = {"global_idx": g, "owner": o, "owner_ms": per_rank[o],
                                       "max_rank_ms": max(per_rank), "per_rank_ms": per_rank,
                                       "node_ms": round(node, 3), "speedup_vs_g1": round(g1 / node, 2)}
                print(f"{key}: node {round(node, 3)} ms (slowest rank {max(per_rank)}, owner {per_rank[o]}), G1 {g1} ms",
                      file=sys.stderr, flush=True)
    out["build_id"] = distpow.build_id()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
