#!/usr/bin/env python3
"""Per-wave timeline of one search launch (a diagnostic build with -DDPOW_WAVE_TRACE=1):
where the fixed per-launch overhead goes (wave start spread, first-claim delay, exit spread).
GPU box only:  DPOW_LIB_PATH=distributed-proof-of-work_amd/distpow/libdpow_trace.so python3 tools/wave_trace.py"""
import ctypes, json, os, sys
sys.path.insert(0, "distributed-proof-of-work_amd")
import distpow
from distpow import _lib

W = 6144  # worker waves of a full grid (6 four-wave workgroups per CU x 256 CUs)
F = 8  # words per wave (md5_search_kernel.h kTraceFields)
lib = ctypes.CDLL(_lib.LIB_PATH)
m = distpow.Miner(0)
m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 24))  # warm the clock


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


out = {}
for wbits, wb in ((3, 5), (0, 0), (3, 5)):
    nk = 1 << 24  # one launch (the host splits at every 2^24 k)
    k0 = (1 << 26) + (len(out) << 24)
    m.reset_stats()
    m.search([1, 2, 3, 4], 32, wb, wbits, k0, k0 + nk)
    st = m.stats()
    buf = (ctypes.c_ulonglong * (F * W))()
    assert lib.dpow_diag_wave_trace(buf, F * W) == 0
    t = [tuple(buf[F * i:F * i + 4]) for i in range(W)]
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/wave_trace_{len(out)}_wbits{wbits}.json", "w") as f:
        json.dump(t, f)
    t0 = min(x[0] for x in t)
    us = lambda v: round(v / 100.0, 2)  # 100 MHz ticks -> us
    start = [x[0] - t0 for x in t]
    first = [x[1] - x[0] for x in t]
    end = [x[2] - t0 for x in t]
    tend = max(end)
    idle_end = [tend - e for e in end]
    nwb = [x[3] for x in t]
    out[f"{len(out)}:wbits{wbits}"] = {
        "launches": st.launches, "kernel_us": round(st.kernel_ms * 1e3, 1),
        "wave_span_us": us(tend),
        "start_us_p50_p99_max": [us(pct(start, .5)), us(pct(start, .99)), us(max(start))],
        "first_claim_us_p50_p99_max": [us(pct(first, .5)), us(pct(first, .99)), us(max(first))],
        "exit_idle_us_mean_p50_p99": [us(sum(idle_end) / W), us(pct(idle_end, .5)), us(pct(idle_end, .99))],
        "end_us_min": us(min(end)),
        "wblocks_min_mean_max": [min(nwb), round(sum(nwb) / W, 1), max(nwb)],
    }
print(json.dumps(out, indent=1))
