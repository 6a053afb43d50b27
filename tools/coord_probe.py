#!/usr/bin/env python3
"""BASELINE configs 3-5 through the coordinator mirror (bench.py coordinator_configs), repeated:
the spread of the first-arrived, concurrent-search timings.  GPU box only.
    python3 tools/coord_probe.py [reps] [only-config4] > gpurun_out/<tag>/coord.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def config4():
    from distpow.coordinator import Coordinator
    with Coordinator(8) as c:  # config 4: 8 workers (workerBits = 3), N = 8
        t = time.perf_counter()
        s = c.mine([1, 2, 3, 4], 8)
        assert bench.distpow.verify([1, 2, 3, 4], s, 8)
        return {"config4_8workers_n8_ms": round((time.perf_counter() - t) * 1e3, 3)}


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
fn = config4 if len(sys.argv) > 2 else bench.coordinator_configs
out = [fn() for _ in range(reps)]
for r in out:
    print(json.dumps(r), file=sys.stderr, flush=True)
print(json.dumps(out))
