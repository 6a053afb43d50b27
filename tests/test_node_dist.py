"""N>1 path of the node scheduler (distpow.node.node_mine) on CPU with gloo.

Each rank owns the prefix partition (worker_byte = rank, worker_bits = log2 W,
coordinator.go:127,326); all ranks scan the same k-window per batch and an
all-reduce MIN of [best index, running] ends the search.  The per-rank search
here is the oracle (test injection: the product passes Miner.search), so the
collective logic is checked against the golden workerBits = 0 answers.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_search_fn():
    from _oracle import Oracle
    from distpow import search as S
    o = Oracle()

    def fn(nonce, ntz, wb, wbits, k0, k1, bound):
        r = o.mine_window(list(nonce), ntz, wb, wbits, k0, k1)
        if r is None or r[1] >= bound:
            return S.SearchResult(S.EXHAUSTED)
        return S.SearchResult(S.FOUND, r[1], bytes(r[0]))
    return fn


def _worker_async(rank, world, port, cases, out_q, cancel_rank):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    import torch.distributed as dist
    from distpow.node import node_mine_async
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    fn = _oracle_search_fn()
    res = []
    for sync in (0, 1 << 12):  # purely ticked; and a synchronous first phase handing over to it
        for nonce, ntz in cases:
            r = node_mine_async(fn, nonce, ntz, rank, world, batch_k=64, batch_candidates_max=1 << 16,
                                sync_candidates=sync)
            res.append((r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner))
    # a window with no hit: every rank exhausts k_limit
    r = node_mine_async(fn, [1, 2, 3, 4], 32, rank, world, batch_k=16, k_limit=1 << 12, sync_candidates=0)
    res.append((r.status,))
    # cancellation vote: one rank reports cancelled -> every rank stops
    r = node_mine_async(fn, [1, 2, 3, 4], 32, rank, world, batch_k=16, k_limit=1 << 20,
                        cancelled=(lambda: rank == cancel_rank), sync_candidates=0)
    res.append((r.status,))
    out_q.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_node_mine_async_gloo_matches_wbits0_answer(golden, world):
    """node_mine_async: ranks search without batch boundaries and tick an all-reduce of
    [best, coverage, running]; the answer is still the workerBits = 0 golden."""
    cases = [(e["nonce"], e["ntz"]) for e in golden["first_hits"] if e["global_idx"] < 200_000]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_async, args=(r, world, port, cases, q, world - 1)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    for rank in range(world):
        res = outs[rank]
        assert len(res) == 2 * len(cases) + 2
        for (nonce, ntz), (status, g, secret, owner) in zip(cases + cases, res[:-2]):
            e = exp[(tuple(nonce), ntz)]
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (rank, nonce, ntz)
            assert owner == (g & 0xFF) >> (8 - (world.bit_length() - 1))
        assert res[-2] == (0,)  # EXHAUSTED
        assert res[-1] == (2,)  # CANCELLED


def _worker(rank, world, port, cases, out_q, cancel_rank):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    import torch.distributed as dist
    from distpow.node import node_mine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    fn = _oracle_search_fn()
    res = []
    for nonce, ntz in cases:
        r = node_mine(fn, nonce, ntz, rank, world, batch_k=64)
        res.append((r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner, r.batches))
    # cancellation vote: one rank reports cancelled -> every rank stops at the same batch
    r = node_mine(fn, [1, 2, 3, 4], 32, rank, world, batch_k=16, k_limit=1 << 20,
                  cancelled=(lambda: rank == cancel_rank))
    res.append((r.status, r.batches))
    out_q.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_node_mine_gloo_matches_wbits0_answer(golden, world):
    cases = [(e["nonce"], e["ntz"]) for e in golden["first_hits"] if e["global_idx"] < 200_000]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q, world - 1)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    for rank in range(world):
        res = outs[rank]
        for (nonce, ntz), (status, g, secret, owner, batches) in zip(cases, res[:-1]):
            e = exp[(tuple(nonce), ntz)]
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (rank, nonce, ntz)
            assert owner == (g & 0xFF) >> (8 - (world.bit_length() - 1))
        assert res[-1] == (2, 1)  # CANCELLED after the first batch on every rank
    # all ranks agree batch by batch
    assert len({tuple(map(tuple, [r[:2] for r in outs[k][:-1]])) for k in outs}) == 1


def test_auto_batch_schedule():
    """node_mine's default batch: sqrt(2 c rate / (world p)) with p = 16^-N, clamped."""
    import math
    from distpow.node import BATCH_OVERHEAD_S, RANK_RATE, auto_batch_candidates
    lo, hi = 1 << 16, 1 << 31
    for world in (1, 2, 4, 8):
        seq = [auto_batch_candidates(n, world) for n in range(0, 34)]
        assert all(lo <= b <= hi for b in seq)
        assert seq == sorted(seq)  # rarer hits -> longer batches
        assert seq[0] == lo and seq[-1] == hi
        for n in (5, 6, 7, 8, 9):  # unclamped: the expected-time optimum
            want = math.sqrt(2 * BATCH_OVERHEAD_S * RANK_RATE / (world * 16.0 ** -n))
            assert abs(auto_batch_candidates(n, world) - want) <= 1
    # more GPUs -> a shorter batch per rank (the node's hit rate grows), ratio sqrt(world)
    assert auto_batch_candidates(8, 1) / auto_batch_candidates(8, 8) == pytest.approx(math.sqrt(8), rel=1e-6)


def _worker_auto(rank, world, port, cases, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    import torch.distributed as dist
    from distpow.node import node_mine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    fn = _oracle_search_fn()
    res = []
    for nonce, ntz in cases:  # the product default: one constant batch sized for N and the node
        r = node_mine(fn, nonce, ntz, rank, world)
        res.append((r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner, r.batches))
    out_q.put((rank, res))
    dist.destroy_process_group()


def test_node_mine_default_schedule_gloo(golden):
    """node_mine's default (expected-time) batch schedule over gloo, world 2, with the oracle
    as each rank's search: the workerBits = 0 answers, every rank in step."""
    world = 2
    cases = [(e["nonce"], e["ntz"]) for e in golden["first_hits"] if e["ntz"] <= 4 and e["global_idx"] < 200_000]
    assert cases
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_auto, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    for rank in range(world):
        for (nonce, ntz), (status, g, secret, owner, batches) in zip(cases, outs[rank]):
            e = exp[(tuple(nonce), ntz)]
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (rank, nonce, ntz)
            assert owner == (g & 0xFF) >> 7
    assert [r[4] for r in outs[0]] == [r[4] for r in outs[1]]


class _Injected(RuntimeError):
    pass


def _worker_fail(rank, world, port, out_q, fail_rank, use_board):
    """One rank's search raises at its third batch (a failed GPU search, an EVERIFY, a
    lost device): every rank must leave node_mine within seconds -- the failing one with
    its own error, the others with NodeError -- instead of waiting in an all-reduce."""
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    import torch.distributed as dist
    from distpow.node import NodeBoard, NodeError, node_mine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    board = NodeBoard.create() if use_board else None
    fn = _oracle_search_fn()
    calls = {"n": 0}

    def search(*a):
        calls["n"] += 1
        if rank == fail_rank and calls["n"] == 3:
            raise _Injected("injected search failure")
        return fn(*a)

    t0 = time.perf_counter()
    try:
        node_mine(search, [1, 2, 3, 4], 32, rank, world, batch_k=16, k_limit=1 << 20, board=board)
        out = ("returned",)
    except _Injected:
        out = ("own-error",)
    except NodeError:
        out = ("node-error",)
    out_q.put((rank, out + (calls["n"], time.perf_counter() - t0)))
    # the node is still usable afterwards: the next search runs in step on every rank
    r = node_mine(fn, [1, 2, 3, 4], 3, rank, world, batch_k=64, board=board)
    out_q.put((rank, ("next", r.status, r.global_idx)))
    dist.destroy_process_group()


@pytest.mark.parametrize("use_board", [False, True])
def test_failing_rank_stops_the_node(use_board):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_fail, args=(r, world, port, q, 1, use_board)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(2 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    first = {r: o for r, o in got if o[0] != "next"}
    nxt = {r: o for r, o in got if o[0] == "next"}
    assert first[1][0] == "own-error" and first[0][0] == "node-error", first
    assert first[0][1] == first[1][1] == 3  # both left at the failing batch
    assert all(o[-1] < 5.0 for o in first.values()), first
    assert nxt[0] == nxt[1] == ("next", 1, 97)  # config 1's answer, [1,2,3,4]/3 -> idx 97


def _worker_board(rank, world, port, cases, out_q):
    """node_mine with a NodeBoard over gloo.  Each rank's search (the oracle) takes the
    slot's best as its bound when it starts and posts its hit, as dpow_search does for an
    attached context; the answers must stay the workerBits = 0 goldens over many
    consecutive searches (the slots cycle and are reset two calls ahead)."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    import torch.distributed as dist
    from distpow import search as S
    from distpow.node import NodeBoard, node_mine
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    board = NodeBoard.create()
    assert board is not None  # one host
    fn = _oracle_search_fn()
    att = {"slot": None, "attached": 0}

    def attach(slot):
        att["slot"] = slot
        att["attached"] += slot is not None

    def search(nonce, ntz, wb, wbits, k0, k1, bound):
        slot = att["slot"]
        r = fn(nonce, ntz, wb, wbits, k0, k1, min(bound, board.best(slot)))
        if r.status == S.FOUND:
            board.post(slot, r.global_idx)
        return r

    res = []
    for _ in range(3):
        for nonce, ntz in cases:
            r = node_mine(search, nonce, ntz, rank, world, batch_k=64, board=board, attach_fn=attach)
            res.append((r.status, r.global_idx, None if r.secret is None else list(r.secret), r.owner))
    assert att["slot"] is None and att["attached"] == 3 * len(cases)
    board.close()
    out_q.put((rank, res))
    dist.destroy_process_group()


def test_node_board_gloo_matches_wbits0_answer(golden):
    world = 2
    cases = [(e["nonce"], e["ntz"]) for e in golden["first_hits"] if e["global_idx"] < 200_000]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_board, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    for rank in range(world):
        for (nonce, ntz), (status, g, secret, owner) in zip(cases * 3, outs[rank]):
            e = exp[(tuple(nonce), ntz)]
            assert status == 1 and g == e["global_idx"] and secret == e["secret"], (rank, nonce, ntz)
            assert owner == (g & 0xFF) >> 7


def test_node_mine_world1_group_runs_the_collective():
    """At world 1 with a process group, node_mine takes the collective path (the same code
    the N-GPU node runs), here over gloo on the CPU."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import torch.distributed as dist
    from distpow.node import node_mine
    port = _free_port()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    calls = []
    orig = dist.all_reduce

    def spy(*a, **k):
        calls.append(a[0].tolist())
        return orig(*a, **k)
    dist.all_reduce = spy
    try:
        r = node_mine(_oracle_search_fn(), [1, 2, 3, 4], 3, 0, 1, batch_k=64)
    finally:
        dist.all_reduce = orig
        dist.destroy_process_group()
    assert r.status == 1 and r.global_idx == 97 and r.owner == 0
    assert calls == [[97, 1, 1]]


def _worker_vote(rank, world, shm_name, rounds, out_q):
    """dpow_node_vote from one process: every epoch votes [rank-dependent, ...] values and
    must get the MIN over all ranks; rank 0 is slow on odd epochs (the others wait)."""
    import ctypes
    import sys
    import time
    from multiprocessing import shared_memory
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    from distpow._lib import lib
    shm = shared_memory.SharedMemory(name=shm_name)
    base = ctypes.addressof(ctypes.c_char.from_buffer(shm.buf))
    got = []
    for e in range(1, rounds + 1):
        if rank == 0 and e % 2:
            time.sleep(0.002)
        vin = (ctypes.c_int64 * 3)(1000 * e + rank, e % world == rank, -rank)
        vout = (ctypes.c_int64 * 3)()
        rc = lib().dpow_node_vote(base, rank, world, e, vin, vout, 10 * 10**9)
        got.append((rc, list(vout)))
    out_q.put((rank, got))
    del base
    shm.close()


def test_node_vote_shared_memory():
    """The node vote (include/dpow.h dpow_node_vote): MIN over every rank's values at each
    epoch, the same on every rank, with ranks at most one epoch apart (double-buffered
    entries); and a rank whose peer never votes gets DPOW_EPROTO at its timeout."""
    import ctypes
    from multiprocessing import shared_memory
    world, rounds = 4, 200
    shm = shared_memory.SharedMemory(create=True, size=2 * world * 64)
    try:
        shm.buf[:2 * world * 64] = bytes(2 * world * 64)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_worker_vote, args=(r, world, shm.name, rounds, q)) for r in range(world)]
        for p in procs:
            p.start()
        outs = dict(q.get(timeout=120) for _ in procs)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for r in range(world):
            for e, (rc, v) in enumerate(outs[r], start=1):
                assert rc == 0 and v == [1000 * e, 0 if world > 1 else 1, -(world - 1)], (r, e, v)
        # a peer that never votes: DPOW_EPROTO (-6) after the timeout, not a hang
        here = os.path.dirname(os.path.abspath(__file__))
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
        from distpow._lib import lib
        shm.buf[:2 * world * 64] = bytes(2 * world * 64)
        base = ctypes.addressof(ctypes.c_char.from_buffer(shm.buf))
        vin, vout = (ctypes.c_int64 * 3)(1, 1, 1), (ctypes.c_int64 * 3)()
        assert lib().dpow_node_vote(base, 0, 2, 1, vin, vout, 50 * 10**6) == -6
        assert b"did not vote" in lib().dpow_last_error()
        del base
    finally:
        shm.close()
        shm.unlink()


def test_vote_latency_diagnostic():
    """dpow_diag_vote_latency (tools/node_probe.py's node-vote cost): the vote's MIN holds with
    the last rank arriving after the others wait, the medians are finite, the caller's CPU
    affinity is left as it was; bad arguments are errors."""
    import ctypes
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    from distpow._lib import lib
    before = os.sched_getaffinity(0)
    last, all_ = ctypes.c_double(), ctypes.c_double()
    assert lib().dpow_diag_vote_latency(2, 50, ctypes.byref(last), ctypes.byref(all_)) == 0
    assert 0 <= last.value <= all_.value < 1e6
    assert os.sched_getaffinity(0) == before
    assert lib().dpow_diag_vote_latency(1, 50, ctypes.byref(last), ctypes.byref(all_)) == -1
    assert lib().dpow_diag_vote_latency(2, 0, ctypes.byref(last), ctypes.byref(all_)) == -1


def _worker_board_fail(rank, world, port, out_q):
    """rank 0 cannot create the shared-memory segment (e.g. /dev/shm full):
    every rank returns None from NodeBoard.create together, at once, instead of the
    others waiting in broadcast_object_list until the process-group timeout."""
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "distributed-proof-of-work_amd"))
    import torch.distributed as dist
    from distpow.node import NodeBoard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    if rank == 0:
        def _full(*a, **k):
            raise OSError(28, "No space left on device")
        os.ftruncate = _full  # NodeBoard.create sizes its /dev/shm segment with it
    t0 = time.perf_counter()
    board = NodeBoard.create()
    out_q.put((rank, board is None, time.perf_counter() - t0))
    dist.barrier()  # the group is still in step
    dist.destroy_process_group()


def test_board_creation_failure_is_agreed():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_board_fail, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(none for _, none, _ in outs), outs
    assert all(dt < 10.0 for _, _, dt in outs), outs


def test_board_without_attach_keeps_expected_time_batches():
    """BOARD_BATCH_CANDIDATES (2^33 per rank: the board stops the kernels at the
    first hit) only when attach_fn attaches the slot to the rank's search context; a board
    without attach_fn gets node_mine's expected-time batch (auto_batch_candidates)."""
    from distpow.node import BOARD_BATCH_CANDIDATES, NodeBoard, auto_batch_candidates, node_mine
    board = NodeBoard.local()
    wins = []

    def search(nonce, ntz, wb, wbits, k0, k1, bound):
        from distpow.search import SearchResult
        wins.append(k1 - k0)
        return SearchResult(0)  # EXHAUSTED

    world, rank, n = 8, 3, 7
    node_mine(search, [1, 2, 3, 4], n, rank, world, k_limit=1 << 30, board=board)
    assert wins[0] == max(1, auto_batch_candidates(n, world) >> 5)
    wins.clear()
    node_mine(search, [1, 2, 3, 4], n, rank, world, k_limit=1 << 30, board=board, attach_fn=lambda s: None)
    assert wins[0] == min(BOARD_BATCH_CANDIDATES >> 5, 1 << 30)


def test_native_loop_only_where_the_board_decides(monkeypatch):
    """node_mine takes dpow_node_mine only when the board's votes decide the node (a
    board shared by exactly `world` ranks, or no process group at all) and no Python `cancelled`
    predicate is given; a local board under a process group takes the Python loop, whose
    boundary is the group's all-reduce."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import torch.distributed as dist
    from distpow import node as N
    from distpow.search import Miner

    def boom(*a, **k):
        raise AssertionError("the native loop was taken")

    monkeypatch.setattr(N, "_node_mine_native", boom)
    fake_miner = object.__new__(Miner)  # isinstance passes; never used by the Python loop
    board = N.NodeBoard.local()
    assert not board.shared
    port = _free_port()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    calls = []
    orig = dist.all_reduce

    def spy(*a, **k):
        calls.append(a[0].tolist())
        return orig(*a, **k)
    dist.all_reduce = spy
    try:
        # rank 0 of a 2-rank node on a local board: the Python loop's all-reduce decides
        r = N.node_mine(_oracle_search_fn(), [1, 2, 3, 4], 3, 0, 2, board=board, miner=fake_miner)
        assert r.status == 1 and calls, r
        assert N._native_applies(board, 1) is False  # a process group is up: not even at world 1
        # a Python cancel predicate also keeps the Python loop
        calls.clear()
        r = N.node_mine(_oracle_search_fn(), [1, 2, 3, 4], 3, 0, 2, board=board, miner=fake_miner,
                        cancelled=lambda: False)
        assert r.status == 1 and calls
    finally:
        dist.all_reduce = orig
        dist.destroy_process_group()
        board.close()
    # no process group: the rank's own values decide (one rank, or the one-GPU emulation)
    assert N._native_applies(N.NodeBoard.local(), 1) is True
    assert N._native_applies(N.NodeBoard.local(), 4) is True
