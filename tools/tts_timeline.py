#!/usr/bin/env python3
"""Launch timeline of single-GPU time-to-secret from a rocprofv3 kernel trace of
tools/tts_trace.py (`tools/gpu.sh check` runs both):

    python3 tools/tts_timeline.py gpurun_out/<tag>/tts/trace/run_kernel_trace.csv \
        gpurun_out/<tag>/tts/tts.json > profiles/<round>_tts_timeline.json

Each search's kernels are the ones that started between its call and its return (host
timestamps from tts_trace.py, on rocprofv3's clock); per search it lists the k = 0
kernel and every md5 launch (start relative to the call, duration, grid) and the gaps
between launches."""
import csv
import json
import sys


def main(trace_csv, tts_json):
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "md5_search" in r["Kernel_Name"] or "search_k0" in r["Kernel_Name"]]
    host = json.load(open(tts_json))
    out = []
    for h in host:
        # the kernels of one search: started between the call and its return (host clock =
        # CLOCK_MONOTONIC, rocprofv3's timestamp clock); times relative to the call
        t0 = h["t0_ns"]
        ks = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= h["t1_ns"]]
        launches = []
        prev_end = None
        for r in ks:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            launches.append({"kernel": "k0" if "search_k0" in r["Kernel_Name"] else "md5_search",
                             "start_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1),
                             "end_us": round((e - t0) / 1e3, 1),
                             "gap_us": None if prev_end is None else round((s - prev_end) / 1e3, 1),
                             "grid_threads": int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r.get("Grid_Size", 0))})
            prev_end = e
        out.append(dict(h, launches=launches))
    print(json.dumps({"note": "rocprofv3 --kernel-trace of tools/tts_trace.py (Miner.mine on one GPU); per "
                              "search its k = 0 kernel and md5 launches, times from the host's call; "
                              "ms = host time of the search call",
                      "searches": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
