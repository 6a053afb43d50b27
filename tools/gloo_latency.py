#!/usr/bin/env python3
"""Host (gloo) all-reduce latency of a 3 x int64 tick at 2 / 4 / 8 processes: the cost of
node_mine_async's ticks when they run on a gloo group (CPU only)."""
import os, sys, time, torch, torch.distributed as dist, torch.multiprocessing as mp
def w(r, n, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=r, world_size=n)
    t = torch.zeros(3, dtype=torch.int64)
    for _ in range(100): dist.all_reduce(t, op=dist.ReduceOp.MIN)
    ts = []
    for _ in range(2000):
        t0 = time.perf_counter(); dist.all_reduce(t, op=dist.ReduceOp.MIN); ts.append(time.perf_counter() - t0)
    ts.sort()
    if r == 0: q.put((n, ts[len(ts)//2]*1e6, ts[int(len(ts)*.9)]*1e6))
    dist.destroy_process_group()
if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    for n in (2, 4, 8):
        q = ctx.Queue(); port = 29600 + n
        ps = [ctx.Process(target=w, args=(r, n, port, q)) for r in range(n)]
        [p.start() for p in ps]; print(q.get(timeout=120)); [p.join() for p in ps]
