#!/usr/bin/env python3
"""Host and device timeline of one GPU's and an emulated node rank's small searches, on one
host clock: where a time-to-secret of tens of microseconds goes.

    python3 tools/search_timeline.py [G,...] [nonce/N,...] > gpurun_out/<tag>/search_timeline.json

Per run, the device's s_memrealtime stamps (the k = 0 kernel's start and end, each md5
launch's start as its watcher stamps it and its end as its last workgroup publishes the
record) are mapped to the host's CLOCK_MONOTONIC by dpow_diag_clock_sync, taken right
before the run (late by the stamp's write latency to host memory, ~1 us), and shown in us
from the search's start next to the host's own events (dpow_diag_search_launches: each
launch queued, each record consumed; the search's return; for a non-owner the owner's
post).  G1: Miner.mine on one GPU (bench.py's time-to-secret).  G > 1: the owner of the
answer, then one non-owner with the owner's hit posted at the owner's post moment, through
the native node loop (dpow_node_mine), as tools/node_probe.py emulates the node.  With the diag
build (DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so, -DDPOW_WAVE_TRACE=1)
also the last md5 launch's watcher events and its waves' starts and exits."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import torch  # noqa: E402

import distpow  # noqa: E402
from distpow._lib import LaunchTime  # noqa: E402
from distpow.node import NodeBoard, node_mine, owner_rank  # noqa: E402

W, F = 8192, 8  # the diag build's per-wave trace (md5_search_kernel.h DPOW_WAVE_TRACE)
CASES = [([1, 2, 3, 4], 3), ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5), ([1, 2, 3, 4], 6)]
RUNS = 5


def timeline(lib, ctx, off_ns, t_call_ns, t_ret_ns, post_ns=None):
    t0 = ctypes.c_int64()
    buf = (LaunchTime * 32)()
    n = lib.dpow_diag_search_launches(ctx, ctypes.byref(t0), buf, 32)
    assert n >= 0
    base = t0.value
    us = lambda ns: round((ns - base) / 1e3, 2)  # noqa: E731
    dev = lambda tick: us(tick * 10 + off_ns) if tick else None  # noqa: E731
    out = {"call_us": us(t_call_ns), "return_us": us(t_ret_ns), "launches": [], "t0_ns": base}
    if post_ns is not None:
        out["post_us"] = us(post_ns)
    for x in buf[:min(n, 32)]:
        out["launches"].append({
            "kind": "k0" if x.kind == 0 else "md5", "queued_us": us(x.queued_ns),
            "dev_start_us": dev(x.t_start_tick), "dev_end_us": dev(x.t_end_tick),
            "seen_us": us(x.seen_ns) if x.seen_ns >= 0 else None, "candidates": x.candidates,
            "best": x.best if x.best != distpow.DPOW_NO_HIT else None})
    return out


def read_traces(fns):
    if not fns:
        return None
    out = []
    for fn in fns:
        buf = (ctypes.c_ulonglong * (F * W))()
        assert fn(buf, F * W) == 0
        out.append([tuple(buf[F * i:F * i + F]) for i in range(W)])
    return out


def trace_events(before, after, off_ns, base_ns):
    """The diag build's records of the run's last md5 launch, on the host clock (us from the
    search's start): its watcher's start, first node best relayed, first early-hit relay and
    exit; its worker waves' starts and exits (percentiles), its first own hit; the publishing
    workgroup's retirement steps (trace slot W - 2)."""
    if before is None:
        return None
    us = lambda tick: round((tick * 10 + off_ns - base_ns) / 1e3, 2)  # noqa: E731
    best = None
    for b, a in zip(before, after):
        waves = [x for x, y in zip(a[:-2], b[:-2]) if x != y and x[0]]
        if waves and (best is None or max(x[2] for x in waves) > max(x[2] for x in best[0])):
            best = (waves, a[-1] if a[-1] != b[-1] else None, a[-2] if a[-2] != b[-2] else None)
    if best is None:
        return None
    waves, wt, rt = best
    pct = lambda v, q: sorted(v)[min(len(v) - 1, int(q * len(v)))]  # noqa: E731
    ends = [x[2] for x in waves]
    hits = [x[7] for x in waves if x[7]]
    ev = {"waves": len(waves), "wave_start_us_min_max": [us(min(x[0] for x in waves)), us(max(x[0] for x in waves))],
          "wave_exit_us_min_p50_p90_max": [us(min(ends)), us(pct(ends, .5)), us(pct(ends, .9)), us(max(ends))],
          "first_own_hit_us": us(min(hits)) if hits else None}
    if wt is not None:
        ev["watcher"] = {"start_us": us(wt[0]), "node_best_us": us(wt[1]) if wt[1] else None,
                         "early_us": us(wt[2]) if wt[2] else None, "exit_us": us(wt[3]) if wt[3] else None}
    if rt is not None:  # the publishing workgroup: claims performed, barrier passed, its Ctrl::done
        # increment returned; the record released (after the system-scope release's L2 write-back)
        ev["publisher"] = {"claims_us": us(rt[0]), "barrier_us": us(rt[1]), "done_us": us(rt[2]),
                           "released_us": us(rt[3]) if rt[3] else None}
    return ev


def med_run(runs):
    return sorted(runs, key=lambda r: r["return_us"])[len(runs) // 2]


def main():
    gs = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 8]
    want = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")))
    exp = {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in gold["first_hits"] + gold["deep_hits"]}
    cases = [(nc, n) for nc, n in CASES if want is None or f"{bytes(nc).hex()}/{n}" in want]
    lib = distpow.lib()
    # the diag build (DPOW_LIB_PATH=.../libdpow_trace.so): per-wave records too
    tfns = [lib.dpow_diag_wave_trace, lib.dpow_diag_wave_trace_ls] if hasattr(lib, "dpow_diag_wave_trace") else None
    board = NodeBoard.local()
    warm = NodeBoard.local()
    out = {"build_id": distpow.build_id(), "note": __doc__.strip().splitlines()[0], "cases": {}}
    off = ctypes.c_int64()
    tl = (ctypes.c_int64 * 8)()
    with distpow.Miner(0) as m:
        m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        for G in gs:
            for nonce, n in cases:
                g = exp[(tuple(nonce), n)]
                key = f"G{G} {bytes(nonce).hex()}/{n}"
                if G == 1:
                    runs = []
                    for _ in range(RUNS):
                        before = read_traces(tfns)
                        assert lib.dpow_diag_clock_sync(m._ctx, 20, ctypes.byref(off)) == 0
                        t_call = time.perf_counter_ns()
                        r = m.mine(nonce, n)
                        t_ret = time.perf_counter_ns()
                        assert r.global_idx == g
                        torch.cuda.synchronize()
                        runs.append(timeline(lib, m._ctx, off.value, t_call, t_ret))
                        runs[-1]["trace"] = trace_events(before, read_traces(tfns), off.value, runs[-1]["t0_ns"])
                    out["cases"][key] = {"g1": med_run(runs)}
                    print(key, json.dumps(out["cases"][key]), file=sys.stderr, flush=True)
                    continue
                o = owner_rank(g, G)
                roles = {}
                posts = []
                for role, rank in (("owner", o), ("non-owner", (o + 1) % G)):
                    runs = []
                    for _ in range(RUNS):
                        slot = board.begin()
                        lib.dpow_diag_node_post_at(warm.slot(0), 0, 0)  # the poster running before the clock
                        before = read_traces(tfns)
                        assert lib.dpow_diag_clock_sync(m._ctx, 20, ctypes.byref(off)) == 0
                        t_call = time.perf_counter_ns()
                        post = None
                        if role == "non-owner":
                            post = t_call + sorted(posts)[len(posts) // 2]
                            lib.dpow_diag_node_post_at(slot, g, post)
                        res = node_mine(None, nonce, n, rank, G, board=board, miner=m)
                        t_ret = time.perf_counter_ns()
                        assert res.status in (distpow.FOUND, distpow.EXHAUSTED), res
                        lib.dpow_diag_search_times(m._ctx, tl)
                        if role == "owner":
                            assert res.global_idx == g
                            t0 = ctypes.c_int64()
                            lib.dpow_diag_search_launches(m._ctx, ctypes.byref(t0), None, 0)
                            posts.append(t0.value + tl[7] - t_call if tl[7] >= 0 else t_ret - t_call)
                        torch.cuda.synchronize()
                        time.sleep(2e-4)
                        runs.append(timeline(lib, m._ctx, off.value, t_call, t_ret, post))
                        runs[-1]["trace"] = trace_events(before, read_traces(tfns), off.value, runs[-1]["t0_ns"])
                    roles[role] = med_run(runs)
                    roles[role]["rank"] = rank
                out["cases"][key] = roles
                print(key, json.dumps(roles), file=sys.stderr, flush=True)
    out["clock_offset_note"] = "device stamps mapped with the offset of the run's own dpow_diag_clock_sync"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
