"""The RCCL branch of the node's collective path on the MI355X.

One spawned process -- it initialises HIP itself, after the fork -- opens a world-1
"nccl" (RCCL) process group with device_id = cuda:0, as bench.py and an 8-GPU node
rank do, and runs node_mine over the real Miner.search through it: the batch
boundary's pinned host twin -> device copy, the RCCL MIN all-reduce of [best,
running, healthy], the copy back and the synchronize.  The answers must be the
workerBits = 0 goldens; a rank whose search raises must re-raise after the
all-reduce (the failure vote); and the per-batch cost of the boundary is measured
(it sets node.BATCH_OVERHEAD_S) and printed as one JSON line.
"""
import json
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(port, cases, out_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "distributed-proof-of-work_amd"))
    import time

    import torch
    import torch.distributed as dist

    import distpow
    from distpow.node import NodeBoard, node_mine

    out = {}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        out["backend"] = dist.get_backend()
        dev = torch.device("cuda", 0)
        res = []
        with distpow.Miner(0) as m:
            search = lambda *a: m.search(*a[:6], bound=a[6])  # noqa: E731
            board = NodeBoard.create()  # world 1, one host: a board of one rank
            out["board"] = board is not None
            for nonce, ntz in cases:
                r = node_mine(search, nonce, ntz, 0, 1, device=dev)
                res.append([r.status, r.global_idx, list(r.secret), r.owner, r.batches])
                r = node_mine(search, nonce, ntz, 0, 1, device=dev, board=board, attach_fn=m.attach_node)
                res.append([r.status, r.global_idx, list(r.secret), r.owner, r.batches])
            out["res"] = res

            class Boom(RuntimeError):
                pass
            calls = {"n": 0}

            def failing(*a):
                calls["n"] += 1
                if calls["n"] == 2:
                    raise Boom("injected")
                return search(*a)
            try:
                node_mine(failing, [1, 2, 3, 4], 32, 0, 1, batch_k=1 << 10, k_start=1 << 24, device=dev)
                out["fail"] = "returned"
            except Boom:
                out["fail"] = "raised"
            out["fail_calls"] = calls["n"]

            # the batch boundary alone, and one whole batch of 2^16 candidates
            buf = torch.zeros(3, dtype=torch.int64, device=dev)
            hbuf = torch.zeros(3, dtype=torch.int64, pin_memory=True)
            lat = []
            for i in range(300):
                t = time.perf_counter()
                hbuf[0], hbuf[1], hbuf[2] = i, 1, 1
                buf.copy_(hbuf, non_blocking=True)
                dist.all_reduce(buf, op=dist.ReduceOp.MIN)
                hbuf.copy_(buf, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                assert hbuf.tolist() == [i, 1, 1]
                if i >= 20:
                    lat.append((time.perf_counter() - t) * 1e6)
            batch = []
            for i in range(80):
                t = time.perf_counter()
                r = node_mine(search, [1, 2, 3, 4], 32, 0, 1, batch_k=256, k_start=(1 << 24) + 256 * i,
                              k_limit=(1 << 24) + 256 * (i + 1), device=dev)
                if i >= 20:
                    batch.append((time.perf_counter() - t) * 1e6)
                assert r.status == distpow.EXHAUSTED and r.batches == 1
            lat.sort()
            batch.sort()
            out["boundary_us"] = {"median": lat[len(lat) // 2], "p90": lat[int(len(lat) * 0.9)]}
            out["batch_2p16_us"] = {"median": batch[len(batch) // 2], "p90": batch[int(len(batch) * 0.9)]}
            board.close()
        dist.destroy_process_group()
    except BaseException as e:  # reported to the parent, which fails the test with it
        out["error"] = repr(e)
    out_q.put(out)


def test_rccl_world1_node_mine(golden):
    import torch.multiprocessing as mp

    want = [([1, 2, 3, 4], 6), ([1, 2, 3, 4], 8), ([2, 2, 2, 2], 8)]
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_main, args=(_free_port(), want, q))
    p.start()
    try:
        out = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert "error" not in out, out
    assert p.exitcode == 0
    assert out["backend"] == "nccl" and out["board"]
    for (nonce, ntz), pair in zip(want, zip(out["res"][0::2], out["res"][1::2])):
        e = exp[(tuple(nonce), ntz)]
        for status, g, secret, owner, batches in pair:
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (nonce, ntz, g)
            assert owner == 0
    assert out["fail"] == "raised" and out["fail_calls"] == 2
    print(json.dumps({"rccl_world1": {"boundary_us": out["boundary_us"], "batch_2p16_us": out["batch_2p16_us"]}}))
