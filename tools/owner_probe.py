#!/usr/bin/env python3
"""The owning rank's search of an 8-GPU node at N = 8 ([1,2,3,4], workerBits 3, rank 0),
timed four ways: Miner.mine (windows of 2^26 k), one dpow_search over node_mine's window
(2^28 k), node_mine without a board, node_mine with a local board attached.  Median of 5;
prints one JSON object.  GPU box only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-proof-of-work_amd"))
import torch  # noqa: E402,F401

import distpow  # noqa: E402
from distpow.node import NodeBoard, node_mine  # noqa: E402


def med(v):
    return round(sorted(v)[len(v) // 2], 4)


def main():
    nonce, n, wb, wbits = [1, 2, 3, 4], 8, 0, 3
    out = {}
    with distpow.Miner(0) as m:
        m.search(nonce, 32, 0, 0, 1 << 24, (1 << 24) + (1 << 26))  # warm
        search = lambda *a: m.search(*a[:6], bound=a[6])  # noqa: E731
        board = NodeBoard.local()
        ways = {
            "mine_2p26": lambda: m.mine(nonce, n, wb, wbits),
            "search_2p28": lambda: m.search(nonce, n, wb, wbits, 0, 1 << 28),
            "node_mine_noboard": lambda: node_mine(search, nonce, n, wb, 8),
            "node_mine_board": lambda: node_mine(search, nonce, n, wb, 8, board=board, attach_fn=m.attach_node),
        }
        for rep in range(5):
            for name, fn in ways.items():
                torch.cuda.synchronize()
                m.reset_stats()
                t = time.perf_counter()
                r = fn()
                dt = (time.perf_counter() - t) * 1e3
                st = m.stats()
                assert r.global_idx == 4065377546, (name, r)
                out.setdefault(name, []).append((dt, st.kernel_ms, st.launches))
    print(json.dumps({k: {"ms": med([x[0] for x in v]), "kernel_ms": med([x[1] for x in v]),
                          "launches": v[0][2]} for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
