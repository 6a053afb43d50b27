#!/usr/bin/env python3
"""Per-wave timelines of an emulated 8-GPU node's ranks (diagnostic build, -DDPOW_WAVE_TRACE=1):
where the owner of a small-N answer spends its time beyond hashing, and how a non-owner
drains after the owner's posted hit (tools/node_probe.py emulates the node the same way).

    make -C distributed-proof-of-work_amd/csrc BUILD=build_trace OUT=../distpow/libdpow_trace.so \
        EXTRA=-DDPOW_WAVE_TRACE=1 ../distpow/libdpow_trace.so
    DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so python3 tools/wave_trace_node.py [G,...] [nonce/N,...]

G = 1 traces one GPU's Miner.mine (bench.py's N = 1 time-to-secret) instead of a node rank.

For every case it runs the owner alone (node_mine over a local board, as node_probe.py), then
one non-owner with the owner's hit posted at the owner's post time, and reads the per-wave
record of the launch that held the end of the search (times in us from the launch's first
wave start): wave starts, first claims, the first own hit, the exits (percentiles), the waves
that exit last (their last chunk, its start, wave-blocks hashed, exit reason: 1 drained,
2 chunk at/above the best, 3 stop), and the host's view (search ms)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import torch  # noqa: E402

import distpow  # noqa: E402
from distpow import _lib  # noqa: E402
from distpow.node import NodeBoard, node_mine, owner_rank  # noqa: E402

W, F = 8192, 8
CASES = [([2, 2, 2, 2], 8, 293615578), ([1, 2, 3, 4], 7, 231910082), ([1, 2, 3, 4], 6, 2532284),
         ([5, 6, 7, 8], 5, 167625), ([2, 2, 2, 2], 5, None)]


def read(fn):
    buf = (ctypes.c_ulonglong * (F * W))()
    assert fn(buf, F * W) == 0
    return [tuple(buf[F * i:F * i + F]) for i in range(W)]


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def summarize(before, after):
    """Waves whose record changed in this run (both trace buffers: the "_ls" kernels and the
    others); the launch whose waves exited last."""
    launches = []
    for b, a in zip(before, after):
        t = [x for x, y in zip(a[:-1], b[:-1]) if x != y and x[0]]
        if t:
            launches.append((t, a[-1] if a[-1] != b[-1] else None))
    if not launches:
        return None
    t, wt = max(launches, key=lambda ws: max(x[2] for x in ws[0]))
    t0 = min(x[0] for x in t)
    us = lambda v: round(v / 100.0, 2)  # noqa: E731  (100 MHz ticks -> us)
    watcher = None
    if wt is not None:  # the watcher's record (last slot): start, node best relayed, early relay, exit
        watcher = {"start_us": us(wt[0] - t0), "node_best_us": us(wt[1] - t0) if wt[1] else None,
                   "early_us": us(wt[2] - t0) if wt[2] else None, "exit_us": us(wt[3] - t0) if wt[3] else None}
    ends = [x[2] - t0 for x in t]
    hits = [x[7] - t0 for x in t if x[7]]
    last = sorted(t, key=lambda x: x[2])[-8:]
    reasons = {}
    for x in t:
        reasons[str(x[6])] = reasons.get(str(x[6]), 0) + 1
    return {
        "watcher": watcher,
        "waves": len(t),
        "start_us_p50_max": [us(pct([x[0] - t0 for x in t], .5)), us(max(x[0] - t0 for x in t))],
        "first_claim_us_p50_p99_max": [us(pct([x[1] - x[0] for x in t], .5)), us(pct([x[1] - x[0] for x in t], .99)),
                                       us(max(x[1] - x[0] for x in t))],
        "first_own_hit_us": us(min(hits)) if hits else None,
        "own_hits": len(hits),
        "exit_us_min_p10_p50_p90_p99_max": [us(min(ends)), us(pct(ends, .1)), us(pct(ends, .5)), us(pct(ends, .9)),
                                            us(pct(ends, .99)), us(max(ends))],
        "exit_reasons": reasons,
        "wblocks_mean_max": [round(sum(x[3] for x in t) / len(t), 1), max(x[3] for x in t)],
        "last_exits": [{"exit_us": us(x[2] - t0), "start_us": us(x[0] - t0), "last_chunk": x[5],
                        "last_chunk_start_us": us(x[4] - t0) if x[4] else None, "wblocks": x[3], "reason": x[6]}
                       for x in last],
        "chunk_of_first_hit": min((x for x in t if x[7]), key=lambda x: x[7])[5] if hits else None,
        # the wave that found the first hit: when it started the hit's chunk, its wave-blocks,
        # and where it stood among all waves (its wave-blocks' rank, 0 = fewest)
        "hit_wave": (lambda x: {"start_us": us(x[0] - t0), "hit_chunk_start_us": us(x[4] - t0),
                                "hit_us": us(x[7] - t0), "wblocks": x[3],
                                "wblocks_rank": sum(1 for y in t if y[3] < x[3]) / len(t)})(
            min((x for x in t if x[7]), key=lambda x: x[7])) if hits else None,
        "wblocks_p0_p10_p50": [min(x[3] for x in t), pct([x[3] for x in t], .1), pct([x[3] for x in t], .5)],
    }


def main():
    L = ctypes.CDLL(_lib.LIB_PATH)
    fns = [L.dpow_diag_wave_trace, L.dpow_diag_wave_trace_ls]
    lib = distpow.lib()
    board = NodeBoard.local()
    out = {"build_id": distpow.build_id(), "cases": {}}
    gs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [8]
    want = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")))
    exp = {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in gold["first_hits"]}
    cases = [(nc, n, exp[(tuple(nc), n)]) for nc, n, _ in CASES
             if want is None or f"{bytes(nc).hex()}/{n}" in want]
    with distpow.Miner(0) as m:
        m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        found_at = {}

        tl = (ctypes.c_int64 * 8)()

        def search(*a):
            t_call = time.perf_counter_ns()
            r = m.search(*a[:6], bound=a[6])
            if r.status == distpow.FOUND:  # when the hit reached the slot (tools/node_probe.py)
                lib.dpow_diag_search_times(m._ctx, tl)
                found_at["t"] = t_call + tl[7] if tl[7] >= 0 else time.perf_counter_ns()
            return r

        warm = NodeBoard.local()

        def run(nonce, n, rank, post_ns=None, g=None, G=8):
            slot = board.begin()
            lib.dpow_diag_node_post_at(warm.slot(0), 0, 0)  # the poster thread running before the clock
            torch.cuda.synchronize()
            before = [read(f) for f in fns]
            found_at.clear()
            t0 = time.perf_counter_ns()
            if post_ns is not None:
                lib.dpow_diag_node_post_at(slot, g, t0 + post_ns)
            if G == 1:
                res = m.mine(nonce, n)
            else:
                res = node_mine(search, nonce, n, rank, G, board=board, attach_fn=m.attach_node)
            dt = time.perf_counter_ns() - t0
            torch.cuda.synchronize()
            after = [read(f) for f in fns]
            return res, dt, found_at.get("t", t0 + dt) - t0, summarize(before, after)

        for G, (nonce, n, g) in [(G, c) for G in gs for c in cases]:
            o = owner_rank(g, G) if G > 1 else 0
            non = (o + 1) % G
            key = f"G{G} {bytes(nonce).hex()}/{n}"
            for rep in range(3):
                res, dt, tp, tr = run(nonce, n, o, G=G)
                assert res.global_idx == g
                out["cases"].setdefault(key, []).append({"role": "owner", "rank": o, "ms": round(dt / 1e6, 3),
                                                         "post_ms": round(tp / 1e6, 3), "trace": tr})
                if G == 1:
                    print(f"{key} rep {rep}: {dt / 1e6:.3f} ms", file=sys.stderr, flush=True)
                    continue
                res2, dt2, _, tr2 = run(nonce, n, non, post_ns=tp, g=g, G=G)
                out["cases"][key].append({"role": "non-owner", "rank": non, "ms": round(dt2 / 1e6, 3),
                                          "post_ms": round(tp / 1e6, 3), "trace": tr2})
                print(f"{key} rep {rep}: owner {dt / 1e6:.3f} ms (post {tp / 1e6:.3f}), non-owner {dt2 / 1e6:.3f} ms",
                      file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
