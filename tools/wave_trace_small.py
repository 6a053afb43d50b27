#!/usr/bin/env python3
"""Per-wave timeline of the small launches on the time-to-secret path (a diagnostic build
with -DDPOW_WAVE_TRACE=1): the L = 2 chunk segment (k in [256, 65536), 16.7 M candidates)
without a hit and with an early one (N = 6), and an L = 3 window of the same size.
GPU box only:  DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so python3 tools/wave_trace_small.py"""
import ctypes, json, os, sys
sys.path.insert(0, "distributed-proof-of-work_amd")
import distpow
from distpow import _lib

W = 6144
F = 8  # words per wave (md5_search_kernel.h kTraceFields)
lib = ctypes.CDLL(_lib.LIB_PATH)
m = distpow.Miner(0)
m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 24))  # warm the clock


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


out = {}
for name, (ntz, k0, k1) in {"L2_N32": (32, 256, 65536), "L2_N6_hit": (6, 256, 65536),
                            "L3_N32_same_size": (32, 1 << 20, (1 << 20) + 65280),
                            "L2_N32_again": (32, 256, 65536)}.items():
    buf = (ctypes.c_ulonglong * (F * W))()
    lib.dpow_diag_wave_trace(buf, F * W)  # clear: read the previous launch's record
    m.reset_stats()
    r = m.search([1, 2, 3, 4], ntz, 0, 0, k0, k1)
    st = m.stats()
    assert lib.dpow_diag_wave_trace(buf, F * W) == 0
    t = [tuple(buf[F * i:F * i + 4]) for i in range(W)]
    t = [x for x in t if x[0]]
    t0 = min(x[0] for x in t)
    us = lambda v: round(v / 100.0, 2)  # 100 MHz ticks -> us
    start = [x[0] - t0 for x in t]
    first = [x[1] - x[0] for x in t]
    end = [x[2] - t0 for x in t]
    nwb = [x[3] for x in t]
    out[name] = {
        "status": r.status, "kernel_us": round(st.kernel_ms * 1e3, 1), "waves": len(t),
        "wave_span_us": us(max(end)),
        "start_us_p50_p99_max": [us(pct(start, .5)), us(pct(start, .99)), us(max(start))],
        "first_claim_us_p50_p99_max": [us(pct(first, .5)), us(pct(first, .99)), us(max(first))],
        "end_us_min_p50_p99_max": [us(min(end)), us(pct(end, .5)), us(pct(end, .99)), us(max(end))],
        "wblocks_min_mean_max": [min(nwb), round(sum(nwb) / len(t), 1), max(nwb)],
    }
print(json.dumps(out, indent=1))
