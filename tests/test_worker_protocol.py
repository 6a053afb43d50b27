"""The native worker (include/dpow_worker.h) keeps the reference worker's protocol
(worker.go:169-232, 258-401): exactly two messages per Mine task, one nil ACK per
Found on an idle task, the cache dominance rules, and the trace action order.
CPU tests exercise the paths that never reach the GPU (cache hits, idle Found,
Cancel errors); gpu tests cover the search paths."""
import time

import pytest

import distpow
from distpow.worker import Worker

N1 = [1, 2, 3, 4]


def actions(w, token=None):
    return [t["action"] for t in w.trace() if token is None or t["trace"] == token]


def test_found_on_idle_task_acks_once():
    with Worker(0) as w:
        w.found(N1, 5, 0, [149, 103, 2], token=7)
        r = w.next_result(timeout_ms=1000)
        assert r.secret is None and r.token == 7 and r.nonce == bytes(N1) and r.worker_byte == 0
        assert w.next_result(timeout_ms=50) is None
        assert actions(w) == ["WorkerCancel", "CacheAdd"]


def test_cache_hit_mine_sends_result_then_ack():
    with Worker(0) as w:
        w.found(N1, 5, 2, [149, 103, 2], token=1)
        assert w.next_result(1000).secret is None
        w.mine(N1, 4, 2, 2, token=2)  # cached N=5 >= 4: served from the worker cache
        r = w.next_result(5000)
        assert r.secret == bytes([149, 103, 2]) and r.worker_byte == 2 and r.token == 2
        assert w.next_result(100) is None  # waits for the kill before the ACK
        w.found(N1, 4, 2, r.secret, token=2)
        a = w.next_result(5000)
        assert a.secret is None
        assert actions(w, 2) == ["WorkerMine", "CacheHit", "WorkerResult", "WorkerCancel"]
        assert w.active_tasks() == 0


def test_cancel_unknown_task_is_protocol_error():
    with Worker(0) as w:
        with pytest.raises(distpow.DpowError) as e:
            w.cancel(N1, 3, 0)
        assert e.value.code == -6


def test_cache_dominance_rules():
    """worker.go:454-506: replace on more zeros, or equal zeros and bytes.Compare(new, old) > 0."""
    with Worker(0) as w:
        seq = [(3, [97]), (3, [50]), (3, [98]), (2, [200]), (4, [1, 1]), (4, [1, 1, 0]), (4, [1, 0, 9])]
        for i, (n, s) in enumerate(seq):
            w.found(N1, n, 0, s, token=100 + i)
            assert w.next_result(1000).secret is None
        tr = [t for t in w.trace() if t["action"] in ("CacheAdd", "CacheRemove")]
        got = [(t["action"], t["NumTrailingZeros"], t["Secret"]) for t in tr]
        assert got == [("CacheAdd", 3, [97]),
                       ("CacheRemove", 3, [97]), ("CacheAdd", 3, [98]),
                       ("CacheRemove", 3, [98]), ("CacheAdd", 4, [1, 1]),
                       ("CacheRemove", 4, [1, 1]), ("CacheAdd", 4, [1, 1, 0])]
        w.mine(N1, 4, 0, 0, token=9)
        assert w.next_result(5000).secret == bytes([1, 1, 0])
        w.found(N1, 4, 0, [1, 1, 0], token=9)
        assert w.next_result(5000).secret is None


def test_bad_arguments():
    with Worker(0) as w:
        with pytest.raises(distpow.DpowError):
            w.mine(bytes(2000), 3, 0, 0)
        with pytest.raises(distpow.DpowError):
            w.mine(N1, 3, 300, 0)


# ------------------------------------------------------------------ GPU paths
@pytest.mark.gpu
def test_mine_found_protocol_on_gpu(golden):
    e = next(x for x in golden["first_hits"] if x["nonce"] == N1 and x["ntz"] == 6)
    with Worker(0) as w:
        w.mine(N1, 6, 0, 0, token=11)
        r = w.next_result(30000)
        assert r.secret == bytes(e["secret"]) and r.token == 11
        assert w.next_result(100) is None
        w.found(N1, 6, 0, r.secret, token=11)
        assert w.next_result(5000).secret is None
        assert w.next_result(100) is None
        assert actions(w, 11) == ["WorkerMine", "CacheMiss", "WorkerResult", "CacheAdd", "WorkerCancel"]


@pytest.mark.gpu
def test_cancel_while_mining_sends_two_nils():
    with Worker(0) as w:
        w.mine(N1, 32, 1, 1, token=5)  # unreachable: mines until killed
        time.sleep(0.5)
        t0 = time.perf_counter()
        w.cancel(N1, 32, 1)
        a = w.next_result(10000)
        lat = time.perf_counter() - t0
        b = w.next_result(10000)
        assert a.secret is None and b.secret is None
        assert w.next_result(100) is None
        assert actions(w, 5) == ["WorkerMine", "CacheMiss", "WorkerCancel"]
        print(f"worker cancel -> first ACK {lat * 1e3:.2f} ms")
        assert lat < 0.5


@pytest.mark.gpu
def test_found_while_mining_kills_search(golden):
    """The coordinator's Found (not Cancel) is what stops the other workers (coordinator.go:210-230)."""
    with Worker(0) as w:
        w.mine(N1, 32, 3, 2, token=8)
        time.sleep(0.3)
        w.found(N1, 32, 3, [1, 2, 3], token=8)
        assert w.next_result(10000).secret is None
        assert w.next_result(10000).secret is None
        assert actions(w, 8) == ["WorkerMine", "CacheMiss", "CacheAdd", "WorkerCancel"]


@pytest.mark.gpu
def test_partition_workers_race_and_min_rule(golden):
    """4 workers (workerBits=2) on one GPU: every worker's first hit matches the
    golden partition tables; their min is the workerBits=0 answer."""
    parts = {e["worker_byte"]: e for e in golden["partitions"]
             if e["worker_bits"] == 2 and e["ntz"] == 5 and e["worker_byte"] < 4}
    ws = [Worker(0) for _ in range(4)]
    try:
        for wb, w in enumerate(ws):
            w.mine(N1, 5, wb, 2, token=wb)
        got = {}
        for wb, w in enumerate(ws):
            r = w.next_result(30000)
            assert r.secret is not None
            got[wb] = list(r.secret)
            w.found(N1, 5, wb, r.secret, token=wb)
            assert w.next_result(5000).secret is None
        for wb in range(4):
            assert got[wb] == parts[wb]["secret"]
        g = min(parts[wb]["global_idx"] for wb in range(4))
        first = next(x for x in golden["first_hits"] if x["nonce"] == N1 and x["ntz"] == 5)
        assert g == first["global_idx"]
    finally:
        for w in ws:
            w.close()


def test_failed_search_is_reported_not_hung():
    """A miner whose GPU search fails (here: no HIP device) reports the error on the
    result channel at once -- one message, the task is over -- instead of waiting
    for a kill as if it were still searching (silent hang)."""
    if distpow.device_count() > 0:
        pytest.skip("needs a host without a visible GPU")
    with Worker(0) as w:
        t0 = time.perf_counter()
        w.mine(N1, 5, 0, 0, token=3)
        r = w.next_result(5000)
        assert r is not None and r.error == distpow.EHIP and r.secret is None and r.token == 3
        assert time.perf_counter() - t0 < 5
        assert w.next_result(100) is None
        assert w.active_tasks() == 0
        acts = actions(w, 3)
        assert acts == ["WorkerMine", "CacheMiss", "MinerError"]


def test_coordinator_fails_fast_on_worker_error():
    from distpow.coordinator import Coordinator, CoordinatorProtocolError
    if distpow.device_count() > 0:
        pytest.skip("needs a host without a visible GPU")
    with Coordinator(2, timeout_s=600) as c:
        t0 = time.perf_counter()
        with pytest.raises(CoordinatorProtocolError, match="search failed"):
            c.mine(N1, 5)
        assert time.perf_counter() - t0 < 10
        assert "CoordinatorWorkerError" in [t["action"] for t in c.trace()]


def test_process_workers_drive_like_in_process_ones():
    """distpow.procworker: the coordinator drives W worker processes over pipes exactly as it
    drives in-process workers -- Mine, the ResultChannel, the trace -- and, with no GPU visible
    here, fails the request at once on their error messages (no hang)."""
    from distpow.coordinator import Coordinator, CoordinatorProtocolError
    from distpow.procworker import ProcessWorker
    if distpow.device_count() > 0:
        pytest.skip("needs a host without a visible GPU")
    workers = [ProcessWorker(0) for _ in range(2)]
    with Coordinator(2, workers=workers, timeout_s=600) as c:
        assert c.board is None and c.worker_bits == 1
        t0 = time.perf_counter()
        with pytest.raises(CoordinatorProtocolError, match="search failed"):
            c.mine(N1, 5, token=9)
        assert time.perf_counter() - t0 < 30
        acts = [t["action"] for t in workers[0].trace() if t["trace"] == 9]
        assert acts[:2] == ["WorkerMine", "CacheMiss"] and "MinerError" in acts
    assert all(not w._proc.is_alive() for w in workers)
