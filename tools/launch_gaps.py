#!/usr/bin/env python3
"""Run one pipelined window per workerBits (0 and 3) for rocprofv3 --kernel-trace, to split the
per-launch overhead of small launches into in-kernel time and inter-launch gaps.  GPU box only:
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- python3 tools/launch_gaps.py
  python3 tools/launch_gaps.py --analyze gpurun_out/gaps/run_kernel_trace.csv"""
import csv, json, sys


def analyze(path):
    rows = sorted((r for r in csv.DictReader(open(path)) if "md5_search" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    groups = {}
    for r in rows:
        groups.setdefault(int(r["Grid_Size_X"]), []).append(r)
    out = {}
    for grid, rs in groups.items():
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs]
        gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rs, rs[1:])]
        gap = [g for g in gap if g < 1000]
        out[grid] = {"launches": len(rs), "avg_us": sum(dur) / len(dur), "min_us": min(dur),
                     "avg_gap_us": sum(gap) / max(1, len(gap)), "min_gap_us": min(gap) if gap else None}
    print(json.dumps(out, indent=1))


def main():
    sys.path.insert(0, "distributed-proof-of-work_amd")
    import distpow
    m = distpow.Miner(0)
    m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 20))  # warm
    res = {}
    for wbits, wb in ((0, 0), (3, 5)):
        R = 1 << (8 - wbits)
        nk = (1 << 34) // R  # 2^34 candidates: 4 launches at workerBits 0, 32 at workerBits 3
        m.reset_stats()
        r = m.search([1, 2, 3, 4], 32, wb, wbits, 1 << 25, (1 << 25) + nk)
        st = m.stats()
        res[f"wbits{wbits}"] = {"status": r.status, "launches": st.launches,
                                "kernel_ghs": round(st.candidates / (st.kernel_ms * 1e-3) / 1e9, 2),
                                "avg_launch_ms": round(st.kernel_ms / st.launches, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    analyze(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[1] == "--analyze" else main()
