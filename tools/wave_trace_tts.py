#!/usr/bin/env python3
"""Per-wave timeline of the md5 launch of short time-to-secret searches (a diagnostic build
with -DDPOW_WAVE_TRACE=1): where a launch whose hashing takes ~10 us spends the rest --
wave start spread, first-claim delay, the spread of wave exits after the hit.
GPU box only:  DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so python3 tools/wave_trace_tts.py"""
import ctypes, json, sys
sys.path.insert(0, "distributed-proof-of-work_amd")
import distpow
from distpow import _lib

W = 8192
F = 8  # words per wave (md5_search_kernel.h kTraceFields)
lib = ctypes.CDLL(_lib.LIB_PATH)
m = distpow.Miner(0)
m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 24))  # warm the clock


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


cases = {"mine_1234_N6": ([1, 2, 3, 4], 6, 0, 0, 0, 1 << 24), "mine_5678_N5": ([5, 6, 7, 8], 5, 0, 0, 0, 1 << 24),
         "nohit_k1_2p16_N32": ([1, 2, 3, 4], 32, 0, 0, 1, 1 << 16),
         "wb3_1234_N7": ([1, 2, 3, 4], 7, 5, 3, 0, 1 << 24)}
out = {}
for rep in range(2):
    for name, args in cases.items():
        buf = (ctypes.c_ulonglong * (F * W))()
        lib.dpow_diag_wave_trace_ls(buf, F * W)
        m.reset_stats()
        r = m.search(*args)
        st = m.stats()
        assert lib.dpow_diag_wave_trace_ls(buf, F * W) == 0
        t = [tuple(buf[F * i:F * i + 4]) for i in range(W)]
        t = [x for x in t if x[0]]
        t0 = min(x[0] for x in t)
        us = lambda v: round(v / 100.0, 2)  # 100 MHz ticks -> us
        start = [x[0] - t0 for x in t]
        first = [x[1] - x[0] for x in t]
        end = [x[2] - t0 for x in t]
        nwb = [x[3] for x in t]
        out[f"{name}#{rep}"] = {
            "status": r.status, "g": r.global_idx, "launches": st.launches, "kernel_us": round(st.kernel_ms * 1e3, 1),
            "waves": len(t), "wave_span_us": us(max(end)),
            "start_us_p50_p99_max": [us(pct(start, .5)), us(pct(start, .99)), us(max(start))],
            "first_claim_us_p50_p99_max": [us(pct(first, .5)), us(pct(first, .99)), us(max(first))],
            "end_us_min_p10_p50_p90_max": [us(min(end)), us(pct(end, .1)), us(pct(end, .5)), us(pct(end, .9)),
                                           us(max(end))],
            "wblocks_min_mean_max": [min(nwb), round(sum(nwb) / len(t), 1), max(nwb)],
            "wblocks_hist": {str(k): nwb.count(k) for k in sorted(set(nwb))},
        }
print(json.dumps(out, indent=1))
