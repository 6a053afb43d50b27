"""End-to-end: the coordinator protocol (coordinator.go:139-320) over W native GPU workers.

BASELINE configs: 3 (4 workers, workerBits=2, N=7, cold then warm cache),
4 (8 workers, workerBits=3, N=8), 5 (two concurrent clients, mixed nonces, 5..7 zeros).
With W a power of two the workers share a node board (node mode, csrc/board.cpp): the
coordinator's first result is the node's first hit, so every answer is bit-exact with the
reference enumeration's workerBits = 0 first hit (tests/golden/pow_golden.json), and the
messages stay the reference's: 2 per worker, one WorkerResult per task (its owner's).
Non-power-of-two W keeps first-arrived (coordinator.go:326): the secret must verify.
"""
import hashlib
import threading
import time

import pytest

from distpow.coordinator import Coordinator

pytestmark = pytest.mark.gpu

N1 = [1, 2, 3, 4]


def ok(nonce, secret, n):
    return hashlib.md5(bytes(nonce) + bytes(secret)).hexdigest().endswith("0" * n)


def golden_secret(golden, nonce, ntz):
    for e in golden["first_hits"] + golden.get("deep_hits", []):
        if e["nonce"] == list(nonce) and e["ntz"] == ntz:
            return bytes(e["secret"]), e["global_idx"]
    raise KeyError((nonce, ntz))


def check_task_protocol(c, token, secret, g):
    """One task through node mode: exactly one result (the owner's, workerByte = the owner of
    the golden index g), each worker's actions in the reference's order (worker.go:177,363,
    383 for the owner; 177,322 for a worker killed while it searches), and no message left
    over (2W received, none dropped)."""
    W = len(c.workers)
    wbits = c.worker_bits
    owner = (g & 255) >> (8 - wbits)
    acts = [t for t in c.trace() if t["trace"] == token]
    res = [t for t in acts if t["action"] == "CoordinatorWorkerResult"]
    assert [(t["WorkerByte"], bytes(t["Secret"])) for t in res] == [(owner, secret)]
    assert not [t for t in c.trace() if t["action"] == "CoordinatorDroppedResult"]
    for w, wb in zip(c.workers, c.worker_bytes):
        seq = [t["action"] for t in w.trace() if t["trace"] == token and
               t["action"] in ("WorkerMine", "WorkerResult", "WorkerCancel")]
        want = ["WorkerMine", "WorkerResult", "WorkerCancel"] if wb == owner else ["WorkerMine", "WorkerCancel"]
        assert seq == want, (wb, seq)
        assert w.active_tasks() == 0
    assert c.board.tasks() == 0  # every rank left the task's entry


def _split(monkeypatch, split):
    """split: every rank searches its own partition (the multi-GPU role, DPOW_DIAG_BOARD_SPLIT);
    else the W workers, all on GPU 0 here, run each task as one search of rank 0."""
    if split:
        monkeypatch.setenv("DPOW_DIAG_BOARD_SPLIT", "1")
    else:
        monkeypatch.delenv("DPOW_DIAG_BOARD_SPLIT", raising=False)


def check_roles(c, split):
    tasks, shared = c.board.counters()
    assert tasks >= 1 and shared == (0 if split else tasks), (tasks, shared)


@pytest.mark.parametrize("split", [False, True], ids=["one_gpu", "per_rank"])
def test_config3_four_workers_cold_then_warm(golden, monkeypatch, split):
    _split(monkeypatch, split)
    want, g = golden_secret(golden, N1, 7)
    assert want == bytes([194, 170, 210, 13])
    with Coordinator(4) as c:
        assert c.board is not None and c.worker_bits == 2
        t0 = time.perf_counter()
        s = c.mine(N1, 7, token=101)
        cold = time.perf_counter() - t0
        assert s == want  # the golden, not whichever worker finished first
        check_task_protocol(c, 101, want, g)
        t0 = time.perf_counter()
        s2 = c.mine(N1, 7)
        warm = time.perf_counter() - t0
        assert s2 == want and c.cache_entry(N1) == (7, want)
        acts = [t["action"] for t in c.trace()]
        assert acts.count("CoordinatorWorkerMine") == 4
        assert acts[-3:] == ["CoordinatorMine", "CacheHit", "CoordinatorSuccess"]
        # lower N is a cache hit too (cached N >= requested)
        assert c.mine(N1, 5) == want
        check_roles(c, split)
        print(f"config3 cold {cold * 1e3:.1f} ms warm {warm * 1e3:.3f} ms secret {list(s)}")


@pytest.mark.parametrize("split", [False, True], ids=["one_gpu", "per_rank"])
def test_config4_eight_workers_n8(golden, monkeypatch, split):
    _split(monkeypatch, split)
    with Coordinator(8) as c:
        assert c.worker_bits == 3
        for tok, nonce in ((201, N1), (202, [2, 2, 2, 2])):
            want, g = golden_secret(golden, nonce, 8)
            assert c.mine(nonce, 8, token=tok) == want
            check_task_protocol(c, tok, want, g)
        check_roles(c, split)
    assert golden_secret(golden, N1, 8)[0] == bytes([10, 189, 80, 242])
    assert golden_secret(golden, [2, 2, 2, 2], 8)[0] == bytes([218, 55, 128, 17])


@pytest.mark.parametrize("W", [4, 8])
@pytest.mark.parametrize("split", [False, True], ids=["one_gpu", "per_rank"])
def test_sh3_nonces_both_kernels(oracle, monkeypatch, split, W):
    """Nonces whose layout has SH = 3 (md5_search_kernel.h: a narrow kernel for R >= 64, the
    general one for R < 64) through node mode: rank 0's workerBits-0 search (one_gpu) and the
    per-rank partitions (per_rank: workerBits 2 narrow at W = 4, 3 general at W = 8) return the
    oracle's workerBits = 0 first hit, from its owner alone."""
    _split(monkeypatch, split)
    with Coordinator(W) as c:
        for tok, nlen in ((301, 7), (302, 31), (303, 59)):
            nonce = [(37 * i + nlen) & 255 for i in range(nlen)]
            sec, g, _ = oracle.mine_window(nonce, 5, 0, 0, 0, 1 << 16)
            assert c.mine(nonce, 5, token=tok) == bytes(sec), nlen
            check_task_protocol(c, tok, bytes(sec), g)
        check_roles(c, split)


@pytest.mark.parametrize("split", [False, True], ids=["one_gpu", "per_rank"])
def test_config5_two_concurrent_clients(golden, monkeypatch, split):
    _split(monkeypatch, split)
    reqs = [(N1, 7), ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5), ([2, 2, 2, 2], 7)]
    with Coordinator(4) as c:
        out = {}

        def client(i, items):
            for nonce, n in items:
                out[(i, tuple(nonce), n)] = c.mine(nonce, n)

        a = threading.Thread(target=client, args=(0, reqs[:2]))
        b = threading.Thread(target=client, args=(1, reqs[2:]))
        a.start(); b.start(); a.join(120); b.join(120)
        assert len(out) == 4
        for (i, nonce, n), s in out.items():
            assert s == golden_secret(golden, nonce, n)[0], (nonce, n, list(s))
        assert out[(0, (5, 6, 7, 8), 5)] == bytes([84, 244, 3])
        # the later [2,2,2,2]/7 request dominates the /5 entry (coordinator.go:455-470)
        assert c.cache_entry([2, 2, 2, 2]) == (7, bytes([218, 55, 128, 17]))
        assert not [t for t in c.trace() if t["action"] == "CoordinatorDroppedResult"]
        assert c.board.tasks() == 0
        check_roles(c, split)


@pytest.mark.parametrize("split", [False, True], ids=["one_gpu", "per_rank"])
def test_worker_cache_hit_in_node_mode(golden, monkeypatch, split):
    """A worker answering from its cache (worker.go:261-299) never joins the task's entry; the
    other workers leave it on their kill (waiting for it to join, or in their votes), and the 2W
    messages still close."""
    _split(monkeypatch, split)
    want, _ = golden_secret(golden, N1, 6)
    with Coordinator(4) as c:
        # seed worker 2's cache only, as if it alone had served the nonce before; its Found ACK
        # reaches the coordinator outside any request (dropped, coordinator.go:318)
        c.workers[2].found(N1, 6, 2, want, 300)
        deadline = time.time() + 10
        while not [t for t in c.trace() if t["trace"] == 300] and time.time() < deadline:
            time.sleep(0.01)
        s = c.mine(N1, 6, token=301)
        assert s == want
        res = [t for t in c.trace() if t["trace"] == 301 and t["action"] == "CoordinatorWorkerResult"]
        assert [(t["WorkerByte"], bytes(t["Secret"])) for t in res] == [(2, want)]
        assert not [t for t in c.trace() if t["trace"] == 301 and t["action"] == "CoordinatorDroppedResult"]
        for w, wb in zip(c.workers, c.worker_bytes):
            seq = [t["action"] for t in w.trace() if t["trace"] == 301 and
                   t["action"] in ("WorkerMine", "CacheHit", "WorkerResult", "WorkerCancel")]
            want_seq = (["WorkerMine", "CacheHit", "WorkerResult", "WorkerCancel"] if wb == 2
                        else ["WorkerMine", "WorkerCancel"])
            assert seq == want_seq, (wb, seq)
        deadline = time.time() + 10
        while c.board.tasks() and time.time() < deadline:
            time.sleep(0.01)
        assert c.board.tasks() == 0


def test_first_arrived_mode_still_verifies():
    """node=False: the reference's race (coordinator.go:202), every answer verified."""
    with Coordinator(4, node=False) as c:
        assert c.board is None
        s = c.mine([9, 9, 9, 9], 5)
        assert ok([9, 9, 9, 9], s, 5)


def test_non_power_of_two_workers_quirk():
    """coordinator.go:326 floor(log2 3) = 1: worker 2's prefix (2 << 7) wraps onto worker 0's."""
    with Coordinator(3) as c:
        assert c.worker_bits == 1 and c.board is None
        s = c.mine([9, 9, 9, 9], 4)
        assert ok([9, 9, 9, 9], s, 4)


@pytest.mark.parametrize("split", [False, True], ids=["one_gpu", "per_rank"])
def test_worker_processes_share_a_named_board(golden, split):
    """The reference's topology: one worker process per GPU (here 4 processes on GPU 0), each
    opening the node's board by name (DPOW_NODE_BOARD in INTEGRATION.md), driven by the unchanged
    coordinator protocol over pipes (distpow.procworker).  Config 3's answer is the golden, sent
    by its owner's process only; the board holds no task afterwards."""
    import os
    import uuid

    from distpow.procworker import ProcessWorker
    from distpow.worker import Board
    name = f"/dpow_test_proc_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    env = {"DPOW_DIAG_BOARD_SPLIT": "1"} if split else {}
    want, g = golden_secret(golden, N1, 7)
    owner = (g & 255) >> 6
    try:
        with Board(name) as board:  # the parent's view of the same board (counters)
            workers = [ProcessWorker(0, name, env) for _ in range(4)]
            with Coordinator(4, workers=workers) as c:
                assert c.board is None and c.worker_bits == 2
                assert c.mine(N1, 7, token=401) == want
                res = [t for t in c.trace() if t["trace"] == 401 and t["action"] == "CoordinatorWorkerResult"]
                assert [(t["WorkerByte"], bytes(t["Secret"])) for t in res] == [(owner, want)]
                for w, wb in zip(c.workers, c.worker_bytes):
                    seq = [t["action"] for t in w.trace() if t["trace"] == 401 and
                           t["action"] in ("WorkerMine", "WorkerResult", "WorkerCancel")]
                    assert seq == (["WorkerMine", "WorkerResult", "WorkerCancel"] if wb == owner
                                   else ["WorkerMine", "WorkerCancel"]), (wb, seq)
                want8, _ = golden_secret(golden, [2, 2, 2, 2], 8)
                assert c.mine([2, 2, 2, 2], 8) == want8
                assert not [t for t in c.trace() if t["action"] == "CoordinatorDroppedResult"]
            assert board.tasks() == 0
            tasks, shared = board.counters()
            assert tasks == 2 and shared == (0 if split else 2), (tasks, shared)
    finally:
        import distpow
        distpow.lib().dpow_board_unlink(name.encode())
