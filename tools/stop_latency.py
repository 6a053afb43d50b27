#!/usr/bin/env python3
"""Where the time goes between a stop signal and dpow_search returning.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/stop_latency.py > out.json
    python3 tools/stop_latency.py --analyze DIR/run_kernel_trace.csv out.json

A search over an unreachable window runs for 50 ms, then one of three signals ends it:
the node slot's best (another rank's hit, polled by the waiting host thread and
injected as a bound), dpow_search_bound (the same injection from this thread), or the
pinned cancel flag (polled by the kernel's watcher).  Host timestamps
(perf_counter_ns = CLOCK_MONOTONIC, the clock rocprofv3 reports kernel times in) of the
signal and of the return are printed; --analyze lines them up with the md5 launch's
end and the bound kernel's start and end."""
import ctypes
import csv
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))


def run():
    import torch  # noqa: F401
    import distpow
    lib = distpow.lib()
    slot = (ctypes.c_uint64 * 8)()
    addr = ctypes.addressof(slot)
    out = []
    with distpow.Miner(0) as m:
        m.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        for mech in ("slot", "bound", "cancel") * 3:
            lib.dpow_node_slot_reset(addr)
            m.attach_node(addr if mech == "slot" else None)
            res = {}
            k0 = 1 << 25

            def go():
                res["r"] = m.search([1, 2, 3, 4], 32, 0, 0, k0, k0 + (1 << 30))
                res["t_ret"] = time.perf_counter_ns()
            th = threading.Thread(target=go)
            th.start()
            time.sleep(0.05)
            g = ((k0 + (1 << 20)) << 8)  # behind the search's position after 50 ms
            t_sig = time.perf_counter_ns()
            if mech == "slot":
                lib.dpow_node_post(addr, g)
            elif mech == "bound":
                m.bound(g)
            else:
                m.cancel()
            th.join()
            m.clear_cancel()
            m.attach_node(None)
            out.append({"mech": mech, "status": res["r"].status, "t_sig": t_sig, "t_ret": res["t_ret"],
                        "latency_us": round((res["t_ret"] - t_sig) / 1e3, 1)})
            time.sleep(0.02)
    print(json.dumps(out, indent=1))


def analyze(trace_csv, host_json):
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    host = json.load(open(host_json))
    res = []
    for h in host:
        t_sig, t_ret = h["t_sig"], h["t_ret"]
        md5 = [r for r in rows if "md5_search" in r["Kernel_Name"] and int(r["Start_Timestamp"]) < t_sig
               and int(r["End_Timestamp"]) > t_sig]
        bnd = [r for r in rows if "search_bound" in r["Kernel_Name"] and t_sig <= int(r["Start_Timestamp"]) <= t_ret]
        e = {"mech": h["mech"], "latency_us": h["latency_us"]}
        if md5:
            e["md5_end_after_signal_us"] = round((int(md5[0]["End_Timestamp"]) - t_sig) / 1e3, 1)
            e["return_after_md5_end_us"] = round((t_ret - int(md5[0]["End_Timestamp"])) / 1e3, 1)
        if bnd:
            e["bound_kernel_start_after_signal_us"] = round((int(bnd[0]["Start_Timestamp"]) - t_sig) / 1e3, 1)
            e["bound_kernel_end_after_signal_us"] = round((int(bnd[0]["End_Timestamp"]) - t_sig) / 1e3, 1)
        res.append(e)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2], sys.argv[3])
    else:
        run()
