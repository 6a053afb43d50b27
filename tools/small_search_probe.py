#!/usr/bin/env python3
"""Time-to-secret of short searches against the launch knobs (A/B, one GPU):

    python3 tools/small_search_probe.py > gpurun_out/<tag>/small.json

For each setting of the diagnostic overrides read at dpow_open (DPOW_DIAG_BPC worker
workgroups per CU, DPOW_DIAG_MIN_CHUNK wave-blocks per claim, DPOW_DIAG_POLL_WB
wave-blocks per poll group; 0 = the library's own choice) it opens a context and runs
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
CASES = [("1234/5", [1, 2, 3, 4], 5, 0, 0), ("5678/5", [5, 6, 7, 8], 5, 0, 0), ("1234/6", [1, 2, 3, 4], 6, 0, 0),
         ("1234/7", [1, 2, 3, 4], 7, 0, 0), ("G8 1234/6", [1, 2, 3, 4], 6, 5, 3), ("G8 1234/7", [1, 2, 3, 4], 7, 6, 3)]


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


def main():
    global CASES, RUNS
    args = sys.argv[1:]
    if args and args[0] == "--random":  # mean over fresh nonces instead of the BASELINE cases
        CASES, RUNS, args = random_cases(), 3, args[1:]
    settings = [(0, 0, 0)]
    for arg in args:
        v = [int(x) for x in arg.split(",")]
        settings.append(tuple(v + [0] * (3 - len(v))))
    lib = distpow.lib()
    out = []
    for bpc, mc, pw in settings:
        os.environ["DPOW_DIAG_BPC"] = str(bpc)
        os.environ["DPOW_DIAG_MIN_CHUNK"] = str(mc)
        os.environ["DPOW_DIAG_POLL_WB"] = str(pw)
        row = {"bpc": bpc, "min_chunk": mc, "poll_wb": pw, "cases": {}}
        with distpow.Miner(0) as m:
            m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
            tl = (ctypes.c_int64 * 8)()
            for label, nonce, n, wb, wbits in CASES:
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
        print(json.dumps({k: row[k] for k in ("bpc", "min_chunk", "poll_wb", "mean_ms")}), file=sys.stderr, flush=True)
        out.append(row)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
