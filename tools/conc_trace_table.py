#!/usr/bin/env python3
"""Per-search launch table of a rocprofv3 kernel trace of tools/concurrent_rate.py
(rocprofv3 --kernel-trace of tools/concurrent_rate.py): for each stream (one search), its md5 launches, their grids and
median length, and the trace's span.
    python3 tools/conc_trace_table.py gpurun_out/<tag>/w8/kt_kernel_trace.csv"""
import collections
import csv
import json
import sys


def table(path):
    rows = [r for r in csv.DictReader(open(path)) if "md5_search" in r["Kernel_Name"]]
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    by = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        by[f"queue {r['Queue_Id']} stream {r['Stream_Id']}"].append(
            ((s - t0) / 1e6, (e - s) / 1e6, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])))
    out = {"launches": len(rows), "span_ms": round((t1 - t0) / 1e6, 2), "streams": {}}
    for k, v in sorted(by.items()):
        v.sort()
        long = sorted(d for _, d, g in v if d > 0.05)
        out["streams"][k] = {"launches": len(v), "first_ms": round(v[0][0], 2), "last_end_ms": round(max(a + d for a, d, _ in v), 2),
                             "grids": dict(collections.Counter(g for _, _, g in v).most_common(4)),
                             "median_launch_ms": round(long[len(long) // 2], 3) if long else None}
    return out


if __name__ == "__main__":
    print(json.dumps(table(sys.argv[1]), indent=1))
