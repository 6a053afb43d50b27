"""Pin the CPU oracle (oracle/dpow_oracle.c) before trusting it as the checker.

The reference ships no tests or fixtures and cannot be run here (Go absent), so
the oracle is pinned by RFC 1321's test suite and by the golden vectors of an
independent Python restatement (tests/golden/gen_golden.py), which in turn
match SURVEY.md Appendix A.
"""
import hashlib

import pytest


def test_rfc1321_suite(oracle, golden):
    assert len(golden["rfc1321"]) == 7
    for e in golden["rfc1321"]:
        msg = bytes.fromhex(e["msg_hex"])
        assert oracle.md5(msg).hex() == e["md5"]


@pytest.mark.parametrize("ln", [0, 1, 54, 55, 56, 63, 64, 65, 119, 120, 127, 128, 1000])
def test_md5_lengths_vs_hashlib(oracle, ln):
    msg = bytes((i * 131 + 7) & 0xFF for i in range(ln))
    assert oracle.md5(msg) == hashlib.md5(msg).digest()


def test_next_chunk_is_minimal_le(oracle):
    # worker.go:234-244: chunk_k == minimal little-endian bytes of k (survey: k < 70,000)
    chunk = []
    for k in range(70000):
        assert chunk == oracle.chunk_of(k), k
        chunk = oracle.next_chunk(chunk)
    # growth points
    for k in (255, 65535, (1 << 24) - 1, (1 << 32) - 1):
        assert oracle.next_chunk(oracle.chunk_of(k)) == oracle.chunk_of(k + 1)


def test_has_num_zeroes_suffix(oracle):
    assert oracle.has_suffix("abc000", 3)
    assert not oracle.has_suffix("abc000", 4)
    assert oracle.has_suffix("abc", 0)
    assert oracle.has_suffix("0000", 4)
    assert not oracle.has_suffix("00a0", 2)


@pytest.mark.parametrize("wb,wbits", [(0, 0), (1, 1), (3, 2), (5, 3), (2, 1), (3, 9), (1, 10), (7, 8), (200, 0)])
def test_thread_bytes(oracle, wb, wbits):
    rb = 8 - wbits % 9
    exp = [((wb << rb) | i) & 0xFF for i in range(1 << rb)]
    assert oracle.thread_bytes(wb, wbits) == exp


def test_first_hits_small(oracle, golden):
    for e in golden["first_hits"]:
        if e["global_idx"] > 3_000_000:
            continue  # big cases: see test_first_hits_big
        r = oracle.mine_window(e["nonce"], e["ntz"], 0, 0, 0, (e["global_idx"] >> 8) + 1)
        assert r is not None
        assert r[0] == e["secret"] and r[1] == e["global_idx"], e
        assert hashlib.md5(bytes(e["nonce"] + e["secret"])).hexdigest() == e["md5"]


def test_partitions(oracle, golden):
    for e in golden["partitions"]:
        r = oracle.mine_window(e["nonce"], e["ntz"], e["worker_byte"], e["worker_bits"], 0,
                               (e["global_idx"] >> 8) + 1)
        assert r == (e["secret"], e["global_idx"], e["local_idx"]), e


def test_windows(oracle, golden):
    for e in golden["windows"]:
        r = oracle.mine_window(e["nonce"], e["ntz"], e["worker_byte"], e["worker_bits"], e["k_begin"], e["k_end"])
        assert r == (e["secret"], e["global_idx"], e["local_idx"]), e


def test_nonce_lengths(oracle, golden):
    for e in golden["nonce_lengths"][::3]:
        r = oracle.mine_window(e["nonce"], e["ntz"], 0, 0, 0, (e["global_idx"] >> 8) + 1)
        assert r[0] == e["secret"] and r[1] == e["global_idx"], e


def test_min_over_partitions_is_wbits0_answer(golden):
    # The multi-GPU determinism rule: min over workers of each
    # worker's first hit (by global index) == the workerBits = 0 answer.
    first = {(tuple(e["nonce"]), e["ntz"]): e["global_idx"] for e in golden["first_hits"]}
    by = {}
    for e in golden["partitions"]:
        if e["worker_bits"] in (1, 2, 3) and e["worker_byte"] < (1 << e["worker_bits"]):
            key = (tuple(e["nonce"]), e["ntz"], e["worker_bits"])
            by.setdefault(key, []).append(e["global_idx"])
    assert by
    for (nonce, ntz, wbits), gs in by.items():
        assert len(gs) == 1 << wbits
        assert min(gs) == first[(nonce, ntz)]


def test_first_hits_big_present(golden):
    big = [e for e in golden["first_hits"] if e["global_idx"] > 3_000_000]
    # N=6 (2.5M) is below the cut; N=7/8 cases come from the C oracle (gen_golden.py --big)
    assert {(tuple(e["nonce"]), e["ntz"]) for e in big} >= {((1, 2, 3, 4), 7), ((1, 2, 3, 4), 8),
                                                           ((2, 2, 2, 2), 7), ((2, 2, 2, 2), 8)}
    for e in big:
        h = hashlib.md5(bytes(e["nonce"] + e["secret"])).hexdigest()
        assert h == e["md5"] and h.endswith("0" * e["ntz"])
