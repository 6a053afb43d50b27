#!/usr/bin/env python3
"""BASELINE configs 3-5 through the coordinator mirror (bench.py coordinator_configs), repeated:
the spread of the coordinator's timings.  With `only-config4`: config 4's BASELINE nonce through
a fresh Coordinator(8) per repetition, next to one Miner.mine of it in the same process (the
workerBits = 0 search alone).  GPU box only.
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
        ms = round((time.perf_counter() - t) * 1e3, 3)
        shared = c.board.counters()[1] if c.board is not None else None
    with bench.distpow.Miner(0) as m:
        t = time.perf_counter()
        r = m.mine([1, 2, 3, 4], 8)
        mine_ms = round((time.perf_counter() - t) * 1e3, 3)
        # the board leader's first window: one search of k in [0, 2^28) at workerBits 0
        t = time.perf_counter()
        w = m.search([1, 2, 3, 4], 8, 0, 0, 0, 1 << 28)
        window_ms = round((time.perf_counter() - t) * 1e3, 3)
        assert w.global_idx == r.global_idx
    return {"config4_8workers_n8_ms": ms, "board_shared_gpu_tasks": shared, "miner_mine_ms": mine_ms,
            "miner_window_2p28_ms": window_ms, "global_idx": r.global_idx}


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
fn = config4 if len(sys.argv) > 2 else bench.coordinator_configs
out = [fn() for _ in range(reps)]
for r in out:
    print(json.dumps(r), file=sys.stderr, flush=True)
print(json.dumps(out))
