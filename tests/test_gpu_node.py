"""The product collective path on the GPU: node_mine over the real Miner.search.

Two processes (spawned, each with its own HIP runtime) play two ranks of a
node -- both on device 0 of the one-GPU box -- with the gloo backend for the
batch-boundary all-reduce MIN of [best index, running].  Rank r owns the
workerBits = 1 partition r (coordinator.go:127,326); the node's answer must be
the workerBits = 0 golden (the min rule), owned by the
partition that holds it, and a cancel on one rank must stop both at the same
batch (coordinator.go:210-230 -> the vote in the all-reduce).
"""
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


def _rank_main(rank, world, port, cases, out_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "distributed-proof-of-work_amd"))
    import threading
    import time

    import torch  # noqa: F401  (one HIP runtime for torch and libdpow)
    import torch.distributed as dist

    import distpow
    from distpow.node import node_mine, node_mine_async

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    res = []
    with distpow.Miner(0) as m:
        search = lambda *a: m.search(*a[:6], bound=a[6])  # noqa: E731  (node_mine's search_fn)
        for nonce, ntz in cases:
            # the growing schedule (2^8 k, x4) and the default constant batch (auto_batch_candidates)
            r = node_mine(search, nonce, ntz, rank, world, batch_k=1 << 8)
            res.append((r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner, r.batches))
            r = node_mine(search, nonce, ntz, rank, world)
            res.append((r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner, r.batches))
        # the asynchronous node search: no batch boundaries, the node's best hit injected
        # into every rank's running search (Miner.bound -> dpow_search_bound)
        for nonce, ntz in cases:
            r = node_mine_async(search, nonce, ntz, rank, world, bound_fn=m.bound, cancel_fn=m.cancel,
                                clear_fn=m.clear_cancel)
            res.append(("async", r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner))
        # the node board (the shared-memory Found fan-out, dpow_node_slot): each rank's
        # context polls the slot, takes another rank's hit as its bound and posts its own
        from distpow.node import NodeBoard
        board = NodeBoard.create()
        assert board is not None
        for nonce, ntz in cases:
            r = node_mine(search, nonce, ntz, rank, world, board=board, attach_fn=m.attach_node)
            res.append(("board", r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner))
        # the native loop (dpow_node_mine, round 5): the same board, its vote in C; then with a
        # first window of twice the per-rank expected first hit (first_window_k)
        from distpow import DPOW_K_LIMIT
        from distpow.node import BOARD_BATCH_CANDIDATES, _node_mine_native, first_window_k
        for nonce, ntz in cases + [([1, 2, 3, 4], 3)]:
            r = node_mine(None, nonce, ntz, rank, world, board=board, miner=m)
            res.append(("native", r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner))
            r = _node_mine_native(m, board, nonce, ntz, rank, world, 0, DPOW_K_LIMIT, BOARD_BATCH_CANDIDATES >> 7,
                                  first_window_k(ntz, world, 2.0))
            res.append(("native-first", r.status, r.global_idx, None if r.secret is None else list(r.secret),
                        r.owner))
        # a cancel on one rank through the board: its search returns CANCELLED and raises
        # the slot's stop, which ends the other rank's search at once (not at a batch end)
        if rank == 0:
            threading.Timer(0.3, m.cancel).start()
        t0 = time.perf_counter()
        r = node_mine(search, [1, 2, 3, 4], 32, rank, world, batch_k=1 << 30, k_start=1 << 24, board=board,
                      attach_fn=m.attach_node)
        m.clear_cancel()
        res.append(("board-cancel", r.status, r.batches, time.perf_counter() - t0))
        # the same through the native loop
        if rank == 1:
            threading.Timer(0.3, m.cancel).start()
        t0 = time.perf_counter()
        r = node_mine(None, [1, 2, 3, 4], 32, rank, world, k_start=1 << 24, board=board, miner=m)
        m.clear_cancel()
        res.append(("native-cancel", r.status, r.batches, time.perf_counter() - t0))
        board.close()
        # a real cancel on the last rank: its pinned flag stops its kernel mid-launch, the
        # search returns CANCELLED and the all-reduce's running slot stops every rank
        if rank == world - 1:
            threading.Timer(0.3, m.cancel).start()
        t0 = time.perf_counter()
        r = node_mine(search, [1, 2, 3, 4], 32, rank, world, batch_k=1 << 20, k_start=1 << 24,
                      batch_k_max=1 << 24)
        m.clear_cancel()
        res.append((r.status, r.batches, time.perf_counter() - t0))
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_node_mine_two_ranks_on_gpu(golden):
    import torch.multiprocessing as mp

    want = [([1, 2, 3, 4], 6), ([1, 2, 3, 4], 8), ([2, 2, 2, 2], 8), ([5, 6, 7, 8], 5)]
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    assert (1, 2, 3, 4, 3) in {tuple(k[0]) + (k[1],) for k in exp}
    cases = [c for c in want if (tuple(c[0]), c[1]) in exp]
    assert len(cases) == len(want)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = dict(q.get(timeout=100) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    n = 2 * len(cases)
    for rank in range(world):
        for (nonce, ntz), (status, g, secret, owner, batches) in zip([c for c in cases for _ in (0, 1)],
                                                                     outs[rank][:n]):
            e = exp[(tuple(nonce), ntz)]
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (rank, nonce, ntz, g)
            assert owner == (g & 0xFF) >> 7
        for (nonce, ntz), (tag, status, g, secret, owner) in zip(cases, outs[rank][n:n + len(cases)]):
            e = exp[(tuple(nonce), ntz)]
            assert tag == "async" and status == 1 and g == e["global_idx"] and secret == e["secret"], \
                (rank, nonce, ntz, g)
            assert owner == (g & 0xFF) >> 7
        for (nonce, ntz), (tag, status, g, secret, owner) in zip(cases, outs[rank][n + len(cases):n + 2 * len(cases)]):
            e = exp[(tuple(nonce), ntz)]
            assert tag == "board" and status == 1 and g == e["global_idx"] and secret == e["secret"], \
                (rank, nonce, ntz, g)
            assert owner == (g & 0xFF) >> 7
        nat = [x for x in outs[rank] if x[0] in ("native", "native-first")]
        assert len(nat) == 2 * (len(cases) + 1)
        for (nonce, ntz), (tag, status, g, secret, owner) in zip([c for c in cases + [([1, 2, 3, 4], 3)]
                                                                   for _ in (0, 1)], nat):
            e = exp[(tuple(nonce), ntz)]
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (rank, tag, nonce, ntz, g)
            assert owner == (g & 0xFF) >> 7
        tag, status, batches, secs = outs[rank][-2]
        # (its windows are board batches of 2^33 candidates per rank, ~40 ms each on the shared GPU:
        # the stop ends the window in flight on both ranks, which voted the same windows)
        assert tag == "native-cancel" and status == 2 and secs < 1.0, outs[rank][-2]
        tag, status, batches, secs = outs[rank][-3]
        # the batch (2^37 candidates per rank, > 1 s on a shared GPU) ends at the stop
        assert tag == "board-cancel" and status == 2 and batches == 1 and secs < 1.0, outs[rank][-2]
        status, batches, secs = outs[rank][-1]
        assert status == 2, outs[rank][-1]  # CANCELLED on every rank
        assert secs < 5
    # the ranks agree batch by batch
    assert [r[4] for r in outs[0][:n]] == [r[4] for r in outs[1][:n]]
    assert outs[0][-1][1] == outs[1][-1][1]
    assert outs[0][-2][2] == outs[1][-2][2]
