"""BASELINE.json's five configs, one named GPU test each.

Each pins the deterministic answer -- the reference enumeration's first hit,
worker.go:301-400, for the workerBits = 0 order, which the min rule makes the
answer of every partitioned run -- against tests/golden/pow_golden.json, and runs
the configuration's own shape: 1 worker, 1 GPU, 4 workers (workerBits 2) with the
coordinator cache cold then warm, 8 workers (workerBits 3), and two concurrent
clients with mixed nonces and 5-9 trailing zeros.  The coordinator's workers share a node
board (W a power of two: csrc/board.cpp), so its first result -- the reference protocol,
coordinator.go:202 -- is the node's first hit, bit-exact with the golden; the partitions'
minimum is checked on its own as well.
"""
import hashlib
import threading

import pytest

import distpow
from distpow import FOUND
from distpow.coordinator import Coordinator

pytestmark = pytest.mark.gpu

N1 = [1, 2, 3, 4]


def _golden(golden, nonce, ntz):
    for e in golden["first_hits"] + golden.get("deep_hits", []):
        if e["nonce"] == list(nonce) and e["ntz"] == ntz:
            return e
    raise KeyError((nonce, ntz))


def _zeros(nonce, secret):
    h = hashlib.md5(bytes(nonce) + bytes(secret)).hexdigest()
    return len(h) - len(h.rstrip("0"))


def _partition_min(miner, nonce, ntz, wbits, g):
    """min over the 2^wbits partitions' first hits up to the golden's k (the node's answer)."""
    hits = []
    for wb in range(1 << wbits):
        r = miner.search(nonce, ntz, wb, wbits, 0, (g >> 8) + 1)
        if r.status == FOUND:
            assert _zeros(nonce, r.secret) >= ntz
            hits.append((r.global_idx, wb))
    return min(hits)


def test_config1_one_worker_n3(miner, golden):
    """Repo default: 1 client, coordinator + 1 worker (workerBits 0), [1,2,3,4], 3 zeros."""
    e = _golden(golden, N1, 3)
    r = miner.mine(N1, 3)
    assert (r.status, r.global_idx, list(r.secret)) == (FOUND, e["global_idx"], e["secret"]) == (FOUND, 97, [97])
    with Coordinator(1) as c:  # one worker: first-arrived is the deterministic answer
        assert list(c.mine(N1, 3)) == e["secret"]


def test_config2_single_gpu_n6(miner, golden):
    """Single MI355X, 1 worker, [1,2,3,4], 6 zeros: bit-exact with the Go enumeration."""
    e = _golden(golden, N1, 6)
    r = miner.mine(N1, 6)
    assert (r.global_idx, list(r.secret)) == (e["global_idx"], e["secret"]) == (2532284, [188, 163, 38])


def test_config3_four_workers_n7_cold_warm(miner, golden):
    """4 workers (workerBits 2), 7 zeros, coordinator cache cold then warm."""
    e = _golden(golden, N1, 7)
    assert _partition_min(miner, N1, 7, 2, e["global_idx"]) == (e["global_idx"], (e["global_idx"] & 255) >> 6)
    with Coordinator(4) as c:
        cold = c.mine(N1, 7)
        assert list(cold) == e["secret"] == [194, 170, 210, 13]
        warm = c.mine(N1, 7)  # served by the coordinator cache (coordinator.go:150-166)
        assert warm == cold and c.cache_entry(N1) == (7, cold)
        assert [t["action"] for t in c.trace()][-3:] == ["CoordinatorMine", "CacheHit", "CoordinatorSuccess"]


def test_config4_eight_workers_n8(miner, golden):
    """8 workers (workerBits 3), 8 zeros: the min over the 8 partitions is the golden, owned
    by partition 0 (GPU 0 of the node); the coordinator run returns a verified secret."""
    for nonce in (N1, [2, 2, 2, 2]):
        e = _golden(golden, nonce, 8)
        g = e["global_idx"]
        assert _partition_min(miner, nonce, 8, 3, g) == (g, (g & 255) >> 5)
    assert (4065377546 & 255) >> 5 == 0
    with Coordinator(8) as c:
        for nonce, want in ((N1, [10, 189, 80, 242]), ([2, 2, 2, 2], [218, 55, 128, 17])):
            assert list(c.mine(nonce, 8)) == _golden(golden, nonce, 8)["secret"] == want


def test_config5_two_clients_mixed_n5_to_n9(miner, golden):
    """2 concurrent clients, mixed nonces, 5-9 zeros: cmd/client/main.go's four requests
    through one coordinator, plus N = 9 on the fresh Random(416) nonces, bit-exact."""
    reqs = [(N1, 7), ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5), ([2, 2, 2, 2], 7)]
    out = {}
    with Coordinator(4) as c:
        def client(items):
            for nonce, n in items:
                out[(tuple(nonce), n)] = c.mine(nonce, n)
        th = [threading.Thread(target=client, args=(reqs[:2],)), threading.Thread(target=client, args=(reqs[2:],))]
        for t in th:
            t.start()
        for t in th:
            t.join(120)
        assert len(out) == 4
        for (nonce, z), s in out.items():
            assert list(s) == _golden(golden, list(nonce), z)["secret"], (nonce, z, list(s))
        assert list(out[((5, 6, 7, 8), 5)]) == [84, 244, 3]
        # dominance: the /7 entry replaces the /5 one (coordinator.go:455-470)
        assert c.cache_entry([2, 2, 2, 2]) == (7, bytes([218, 55, 128, 17]))
    for e in golden["deep_hits"]:
        if e["case"].startswith("config5-fresh"):
            r = miner.mine(e["nonce"], 9)
            assert (r.global_idx, list(r.secret)) == (e["global_idx"], e["secret"])
