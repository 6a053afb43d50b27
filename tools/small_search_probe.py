#!/usr/bin/env python3
"""Time-to-secret of short searches against the launch knobs (A/B, one GPU):

    python3 tools/small_search_probe.py > gpurun_out/<tag>/small.json

For each setting of the diagnostic overrides read at dpow_open (DPOW_DIAG_BPC worker
workgroups per CU, DPOW_DIAG_MIN_CHUNK wave-blocks per claim, DPOW_DIAG_POLL_WB
wave-blocks per poll group, DPOW_DIAG_CPW claims per wave; 0 = the library's own choice) it opens a context and runs
the BASELINE time-to-secret cases one GPU and one rank of an 8-GPU node meet at small
N: median ms of the search call, the host timeline (dpow_diag_search_times) and the
md5 kernel time."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import torch  # noqa: E402,F401

import distpow  # noqa: E402

RUNS = 7
# (label, nonce, ntz, worker_byte, worker_bits): one GPU (Miner.mine), and the owning rank of
# an 8-GPU node (workerBits 3) searching from k = 0 up to the answer
CASES = [("1234/3", [1, 2, 3, 4], 3, 0, 0), ("2222/5", [2, 2, 2, 2], 5, 0, 0), ("1234/5", [1, 2, 3, 4], 5, 0, 0), ("5678/5", [5, 6, 7, 8], 5, 0, 0), ("1234/6", [1, 2, 3, 4], 6, 0, 0),
         ("1234/7", [1, 2, 3, 4], 7, 0, 0), ("G8 1234/6", [1, 2, 3, 4], 6, 5, 3), ("G8 1234/7", [1, 2, 3, 4], 7, 6, 3),
         ("G8 1234/8", [1, 2, 3, 4], 8, 0, 3), ("G8 2222/8", [2, 2, 2, 2], 8, 6, 3), ("2222/8", [2, 2, 2, 2], 8, 0, 0)]


def random_cases(count=24):
    """Expected time-to-secret: fresh 4-byte nonces (seeded), one GPU at N = 5 / 6 and one
    rank of an 8-GPU node (workerBits 3, a random partition) at N = 6 / 7."""
    import random
    rnd = random.Random(2026)
    out = []
    for label, n, wbits in (("rand/5", 5, 0), ("rand/6", 6, 0), ("G8 rand/6", 6, 3), ("G8 rand/7", 7, 3)):
        for i in range(count):
            nonce = [rnd.randrange(256) for _ in range(4)]
            out.append((f"{label}#{i}", nonce, n, rnd.randrange(1 << wbits) if wbits else 0, wbits))
    return out


def stop_cases(m, lib, runs=7):
    """A rank stopped by another rank's hit: a search over an 8-GPU rank's window (workerBits 3,
    a partition without a hit there) whose node slot receives a hit 300 us in, just behind the
    search's position (a native poster, dpow_diag_node_post_at).  ms = the search's return
    after the post; timeline = dpow_diag_search_times."""
    slot_mem = (ctypes.c_uint64 * 8)()
    slot = ctypes.addressof(slot_mem)
    out = {}
    for label, n, k0 in (("stop N=6", 6, 1 << 24), ("stop N=7", 7, 1 << 24), ("stop N=8", 8, 1 << 24),
                         ("stop N=32", 32, 1 << 24)):
        ms, tls = [], []
        for _ in range(runs):
            lib.dpow_node_slot_reset(slot)
            m.attach_node(slot)
            torch.cuda.synchronize()
            t_post_rel = 300e-6
            g = (k0 + int(2.17e11 * 200e-6 / 32)) << 8  # ~100 us behind the search's position
            t0 = time.perf_counter_ns()
            lib.dpow_diag_node_post_at(slot, g, t0 + int(t_post_rel * 1e9))
            r = m.search([1, 2, 3, 4], n, 0, 3, k0, k0 + (1 << 24))
            t1 = time.perf_counter_ns()
            m.attach_node(None)
            assert r.status in (distpow.EXHAUSTED, distpow.FOUND), r  # (a hit of its own below g: FOUND)
            ms.append((t1 - t0) / 1e6 - t_post_rel * 1e3)
            tl = (ctypes.c_int64 * 8)()
            lib.dpow_diag_search_times(m._ctx, tl)
            tls.append([round(x / 1e3, 1) for x in tl])
        i = sorted(range(runs), key=lambda j: ms[j])[runs // 2]
        out[label] = {"ms": round(ms[i], 4), "timeline_us": tls[i]}
    return out


def main():
    global CASES, RUNS
    args = sys.argv[1:]
    stop_mode = bool(args) and args[0] == "--stop"
    if stop_mode:
        args = args[1:]
    if args and args[0] == "--random":  # mean over fresh nonces instead of the BASELINE cases
        CASES, RUNS, args = random_cases(), 3, args[1:]
    settings = [(0, 0, 0, 0)]
    for arg in args:
        v = [int(x) for x in arg.split(",")]
        settings.append(tuple(v + [0] * (4 - len(v))))
    lib = distpow.lib()
    out = []
    for bpc, mc, pw, cpw in settings:
        os.environ["DPOW_DIAG_BPC"] = str(bpc)
        os.environ["DPOW_DIAG_MIN_CHUNK"] = str(mc)
        os.environ["DPOW_DIAG_POLL_WB"] = str(pw)
        os.environ["DPOW_DIAG_CPW"] = str(cpw)
        row = {"bpc": bpc, "min_chunk": mc, "poll_wb": pw, "cpw": cpw, "cases": {}}
        with distpow.Miner(0) as m:
            m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
            tl = (ctypes.c_int64 * 8)()
            if stop_mode:
                row["cases"] = stop_cases(m, lib)
            for label, nonce, n, wb, wbits in ([] if stop_mode else CASES):
                ms, tls, kus, g = [], [], [], None
                for _ in range(RUNS):
                    torch.cuda.synchronize()
                    m.reset_stats()
                    t = time.perf_counter()
                    r = m.mine(nonce, n, wb, wbits)
                    ms.append((time.perf_counter() - t) * 1e3)
                    lib.dpow_diag_search_times(m._ctx, tl)
                    tls.append([round(x / 1e3, 1) for x in tl])
                    st = m.stats()
                    kus.append(round(st.kernel_ms * 1e3, 1))
                    assert r.status == distpow.FOUND
                    g = r.global_idx
                i = sorted(range(RUNS), key=lambda j: ms[j])[RUNS // 2]
                row["cases"][label] = {"ms": round(ms[i], 4), "timeline_us": tls[i], "kernel_us": kus[i], "g": g}
        groups = {}
        for label, v in row["cases"].items():
            groups.setdefault(label.split("#")[0], []).append(v["ms"])
        row["mean_ms"] = {k: round(sum(v) / len(v), 4) for k, v in groups.items()}
        print(json.dumps({k: row[k] for k in ("bpc", "min_chunk", "poll_wb", "cpw", "mean_ms")}), file=sys.stderr, flush=True)
        out.append(row)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
