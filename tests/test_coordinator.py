"""End-to-end: the coordinator protocol (coordinator.go:139-320) over W native GPU workers.

BASELINE configs: 3 (4 workers, workerBits=2, N=7, cold then warm cache),
4 (8 workers, workerBits=3, N=8), 5 (two concurrent clients, mixed nonces, 5..7 zeros).
With W > 1 the reference's answer is whichever worker reports first; every
returned secret must verify, and the message accounting must close (2W per task).
"""
import hashlib
import threading
import time

import pytest

import distpow
from distpow.coordinator import Coordinator

pytestmark = pytest.mark.gpu


def ok(nonce, secret, n):
    return hashlib.md5(bytes(nonce) + bytes(secret)).hexdigest().endswith("0" * n)


def test_config3_four_workers_cold_then_warm(golden):
    with Coordinator(4) as c:
        t0 = time.perf_counter()
        s = c.mine([1, 2, 3, 4], 7)
        cold = time.perf_counter() - t0
        assert ok([1, 2, 3, 4], s, 7)
        t0 = time.perf_counter()
        s2 = c.mine([1, 2, 3, 4], 7)
        warm = time.perf_counter() - t0
        # warm: the coordinator cache may hold a lexicographically larger secret of a later worker
        assert ok([1, 2, 3, 4], s2, 7) and c.cache_entry([1, 2, 3, 4])[1] == s2
        acts = [t["action"] for t in c.trace()]
        assert acts.count("CoordinatorWorkerMine") == 4
        assert acts[-3:] == ["CoordinatorMine", "CacheHit", "CoordinatorSuccess"]
        # lower N is a cache hit too (cached N >= requested)
        assert c.mine([1, 2, 3, 4], 5) == s2
        print(f"config3 cold {cold * 1e3:.1f} ms warm {warm * 1e3:.3f} ms secret {list(s)}")


def test_config4_eight_workers_n8(golden):
    with Coordinator(8) as c:
        assert c.worker_bits == 3
        s = c.mine([1, 2, 3, 4], 8)
        assert ok([1, 2, 3, 4], s, 8)
        s = c.mine([2, 2, 2, 2], 8)
        assert ok([2, 2, 2, 2], s, 8)


def test_config5_two_concurrent_clients():
    reqs = [([1, 2, 3, 4], 7), ([5, 6, 7, 8], 5), ([2, 2, 2, 2], 5), ([2, 2, 2, 2], 7)]
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
            assert ok(list(nonce), s, n)
        # the later [2,2,2,2]/7 request (or its cache) dominates the /5 entry
        assert c.cache_entry([2, 2, 2, 2])[0] >= 7


def test_non_power_of_two_workers_quirk():
    """coordinator.go:326 floor(log2 3) = 1: worker 2's prefix (2 << 7) wraps onto worker 0's."""
    with Coordinator(3) as c:
        assert c.worker_bits == 1
        s = c.mine([9, 9, 9, 9], 4)
        assert ok([9, 9, 9, 9], s, 4)
