#!/usr/bin/env python3
"""Launch timeline of single-GPU time-to-secret from a rocprofv3 kernel trace of
tools/tts_trace.py (tools/gpu_check.sh runs both):

    python3 tools/tts_timeline.py gpurun_out/<tag>/tts/trace/run_kernel_trace.csv \
        gpurun_out/<tag>/tts/tts.json > profiles/<round>_tts_timeline.json

The trace is cut into searches at each search_reset kernel (one per dpow_search call;
the first one is tts_trace.py's warm-up) and lined up in order with the searches
tts_trace.py timed; per search it lists the reset and every md5 launch (start
relative to the reset, duration, grid) and the gaps between launches."""
import csv
import json
import sys


def main(trace_csv, tts_json):
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    searches, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if ("search_reset" in name or "search_start" in name):
            cur = []
            searches.append(cur)
        if cur is not None and (("search_reset" in name or "search_start" in name) or "md5_search" in name):
            cur.append(r)
    host = json.load(open(tts_json))
    searches = searches[len(searches) - len(host):]  # drop the warm-up search(es)
    out = []
    for h, ks in zip(host, searches):
        t0 = int(ks[0]["Start_Timestamp"])
        launches = []
        prev_end = None
        for r in ks:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            launches.append({"kernel": "search_reset" if ("search_reset" in r["Kernel_Name"] or "search_start" in r["Kernel_Name"]) else "md5_search",
                             "start_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1),
                             "gap_us": None if prev_end is None else round((s - prev_end) / 1e3, 1),
                             "grid_threads": int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r.get("Grid_Size", 0))})
            prev_end = e
        out.append(dict(h, launches=launches))
    print(json.dumps({"note": "rocprofv3 --kernel-trace of tools/tts_trace.py (Miner.mine on one GPU); per "
                              "search its reset kernel and md5 launches; ms = host time of the search call",
                      "searches": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
