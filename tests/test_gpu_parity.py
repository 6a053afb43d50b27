"""GPU parity: the gfx950 search (through the C ABI) vs the oracle and the golden vectors.

Bit-exact: secrets, global indices and "no hit" outcomes must equal the
reference enumeration's (worker.go:301-400) for the same nonce, trailing-zero
count and worker partition.  Run on the GPU box:  pytest -m gpu
"""
import hashlib
import random
import ctypes
import threading
import time

import pytest

import distpow
from distpow import CANCELLED, DPOW_NO_HIT, EXHAUSTED, FOUND

pytestmark = pytest.mark.gpu


def _hexz(nonce, secret):
    return hashlib.md5(bytes(nonce) + bytes(secret)).hexdigest()


def test_first_hits_golden(miner, golden):
    """Configs 1, 2, 4 of BASELINE.json and SURVEY Appendix A (N = 0..8, workerBits = 0)."""
    for e in golden["first_hits"]:
        r = miner.mine(e["nonce"], e["ntz"])
        assert r.status == FOUND, e
        assert r.global_idx == e["global_idx"] and list(r.secret) == e["secret"], (e, r)
        assert _hexz(e["nonce"], r.secret) == e["md5"]


def test_partitions_golden(miner, golden):
    for e in golden["partitions"]:
        r = miner.mine(e["nonce"], e["ntz"], e["worker_byte"], e["worker_bits"])
        assert r.status == FOUND and r.global_idx == e["global_idx"] and list(r.secret) == e["secret"], (e, r)


def test_windows_golden(miner, golden):
    for e in golden["windows"]:
        r = miner.search(e["nonce"], e["ntz"], e["worker_byte"], e["worker_bits"], e["k_begin"], e["k_end"])
        assert r.status == FOUND and r.global_idx == e["global_idx"] and list(r.secret) == e["secret"], (e, r)


def test_nonce_lengths_golden(miner, golden):
    """Every final-block layout (NBLK 1/2, W0, SH) and midstate nonces up to 200 bytes."""
    for e in golden["nonce_lengths"]:
        r = miner.mine(e["nonce"], e["ntz"])
        assert r.status == FOUND and r.global_idx == e["global_idx"] and list(r.secret) == e["secret"], \
            (len(e["nonce"]), e["ntz"], r)


def test_chunk_length_spanning_launch_vs_oracle(miner, oracle):
    """One md5 launch spans chunk lengths 1..3 (SH = 0 layouts, R >= 2: plan.cpp; the kernel
    re-derives the pad and bit-length words per chunk length) after the start kernel has
    hashed k = 0.  Walk each window's hits one by one -- every search starts right after
    the previous hit's k, so launches start on both sides of k = 1, 256 and 65536 -- and
    compare every first hit with the oracle."""
    K_END = 70000
    cases = [([1, 2, 3, 4], 5, 3, 3), ([1, 2, 3, 4], 7, 2, 3), ([], 6, 2, 3), (list(range(8)), 2, 4, 3),
             (list(range(48)), 1, 5, 3), ([7] * 52, 3, 3, 3), (list(range(60)), 9, 5, 3), ([9] * 64, 0, 6, 2),
             ([5, 6, 7, 8], 0, 2, 4)]
    for nonce, wb, wbits, ntz in cases:
        rb = 8 - wbits % 9
        plan = distpow.plan_window(nonce, wb, wbits, 0, K_END)
        assert plan[0].start_kernel == 1 and plan[1].k_begin == 1 and plan[1].chunk_len == 1
        assert plan[1].chunk_len_last == (2 if len(nonce) == 52 else 3), (len(nonce), [(p.k_begin, p.k_end) for p in plan])
        k, hits = 0, 0
        while k < K_END and hits < 12:
            exp = oracle.mine_window(nonce, ntz, wb, wbits, k, K_END)
            r = miner.search(nonce, ntz, wb, wbits, k, K_END)
            if exp is None:
                assert r.status == EXHAUSTED, (len(nonce), wb, wbits, k, r)
                break
            assert r.status == FOUND and r.global_idx == exp[1] and list(r.secret) == list(exp[0]), \
                (len(nonce), wb, wbits, k, r, exp)
            hits += 1
            k = (r.global_idx >> 8) + 1
        assert hits >= 3, (len(nonce), wb, wbits)
    # R = 256, hits across k = 65536 (the L = 2 -> 3 boundary inside the launch)
    for nonce in ([1, 2, 3, 4], [2, 2, 2, 2]):
        for k0 in (65530, 65000, 60000):
            exp = oracle.mine_window(nonce, 4, 0, 0, k0, 66000)
            r = miner.search(nonce, 4, 0, 0, k0, 66000)
            assert (r.status == FOUND and (r.global_idx, list(r.secret)) == (exp[1], list(exp[0]))) if exp else \
                r.status == EXHAUSTED, (nonce, k0, r, exp)


def test_random_windows_vs_oracle(miner, oracle):
    """Random nonces, partitions and windows (hits and misses), oracle-sized."""
    rnd = random.Random(416)
    for it in range(150):
        nlen = rnd.choice([0, 1, 2, 3, 4, 4, 4, 5, 7, 8, 16, 31, 50, 53, 54, 55, 56, 60, 61, 62, 63, 64, 65, 70, 127])
        nonce = [rnd.randrange(256) for _ in range(nlen)]
        wbits = rnd.choice([0, 0, 1, 2, 3, 4, 6, 8, 9, 10])
        wb = rnd.randrange(1 << (wbits % 9)) if wbits % 9 else rnd.randrange(256)
        rb = 8 - wbits % 9
        ntz = rnd.choice([1, 2, 3, 3, 4, 4, 5])
        seg = rnd.choice([0, 1, 2, 3, 4, 5])
        k0 = rnd.randrange(1 << (8 * seg)) if seg else 0
        if seg >= 3 and rnd.random() < 0.3:  # straddle a segment / 2^24 boundary
            k0 = max(0, (1 << (8 * seg)) - rnd.randrange(1, 40))
        nk = max(1, rnd.randrange(1, 1 + (1 << 16) // (1 << rb)))
        k1 = min(k0 + nk, 1 << 40)
        exp = oracle.mine_window(nonce, ntz, wb, wbits, k0, k1)
        r = miner.search(nonce, ntz, wb, wbits, k0, k1)
        if exp is None:
            assert r.status == EXHAUSTED, (it, nonce, ntz, wb, wbits, k0, k1, r)
        else:
            assert r.status == FOUND and r.global_idx == exp[1] and list(r.secret) == exp[0], \
                (it, nonce, ntz, wb, wbits, k0, k1, r, exp)


def test_top_of_k_range(miner, oracle):
    """The chunk-length boundaries 2^40 / 2^48 (6- and 7-byte chunks) and the last k
    before DPOW_K_LIMIT = 2^55 - 1 (7-byte secrets whose global index k * 256 + t stays
    below DPOW_NO_HIT); a window past the limit is an error, not a wrapped index."""
    top = distpow.DPOW_K_LIMIT
    for k0, k1 in (((1 << 40) - 2048, 1 << 40), ((1 << 40) - 700, (1 << 40) + 700),
                   ((1 << 48) - 700, (1 << 48) + 700), (top - 2048, top)):
        for ntz in (1, 2, 3):
            exp = oracle.mine_window([9, 8, 7, 6], ntz, 0, 0, k0, k1)
            r = miner.search([9, 8, 7, 6], ntz, 0, 0, k0, k1)
            assert r.status == FOUND and (list(r.secret), r.global_idx) == (exp[0], exp[1]), (k0, ntz)
    # every thread byte of the last k (workerBits 0: the largest global indices there are)
    exp = oracle.mine_window([9, 8, 7, 6], 1, 0, 0, top - 1, top)
    r = miner.search([9, 8, 7, 6], 1, 0, 0, top - 1, top)
    assert (r.status, r.global_idx) == ((FOUND, exp[1]) if exp else (EXHAUSTED, DPOW_NO_HIT))
    if exp:
        assert list(r.secret) == exp[0] and len(r.secret) == 8  # thread byte + 7 chunk bytes
    with pytest.raises(distpow.DpowError):
        miner.search([1], 1, 0, 0, 0, top + 1)


def test_long_chunks_vs_oracle(miner, oracle):
    """6- and 7-byte chunks (k in [2^40, 2^55 - 1)) for every byte shift and both block
    counts, random partitions, windows at and across the launch splits the planner puts
    there (2^24-k segments, word W0+2's period for SH 1-2, 2^48), oracle-sized."""
    rnd = random.Random(4855)
    top = distpow.DPOW_K_LIMIT
    for it in range(120):
        nlen = rnd.choice([0, 1, 2, 3, 4, 5, 6, 7, 13, 46, 47, 48, 49, 50, 52, 55, 57, 59, 60, 61, 62, 63, 64, 66])
        nonce = [rnd.randrange(256) for _ in range(nlen)]
        wbits = rnd.choice([0, 0, 2, 3, 6, 8])
        wb = rnd.randrange(1 << (wbits % 9)) if wbits % 9 else rnd.randrange(256)
        rb = 8 - wbits % 9
        ntz = rnd.choice([1, 2, 3, 3, 4])
        edge = rnd.choice([1 << 40, 1 << 48, rnd.randrange(1 << 40, 1 << 48) >> 24 << 24,
                           rnd.randrange(1 << 48, top) >> 24 << 24, rnd.randrange(2, 255) << 40,
                           rnd.randrange(2, 127) << 48, rnd.randrange(1 << 40, top)])
        nk = max(1, rnd.randrange(1, 1 + (1 << 16) // (1 << rb)))
        k0 = max(1 << 40, edge - rnd.randrange(0, nk + 1))
        k1 = min(k0 + nk, top)
        exp = oracle.mine_window(nonce, ntz, wb, wbits, k0, k1)
        r = miner.search(nonce, ntz, wb, wbits, k0, k1)
        if exp is None:
            assert r.status == EXHAUSTED, (it, nlen, ntz, wb, wbits, k0, k1, r)
        else:
            assert r.status == FOUND and r.global_idx == exp[1] and list(r.secret) == exp[0], \
                (it, nlen, ntz, wb, wbits, k0, k1, r, exp)


def test_empty_window_and_unreachable(miner):
    assert miner.search([1, 2, 3, 4], 3, 0, 0, 10, 10).status == EXHAUSTED
    assert miner.search([1, 2, 3, 4], 33, 0, 0, 0, 1 << 16).status == EXHAUSTED  # N > 32 never matches
    assert miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + (1 << 20)).status == EXHAUSTED


def test_ntz_zero_is_first_candidate(miner):
    for wb, wbits in [(0, 0), (3, 2), (7, 3)]:
        r = miner.mine([5, 6, 7, 8], 0, wb, wbits)
        tb = distpow.thread_bytes(wb, wbits)[0]
        assert r.status == FOUND and r.global_idx == tb and list(r.secret) == [tb]


def test_bound_excludes_later_hits(miner, golden):
    e = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 6)
    g = e["global_idx"]
    k1 = (g >> 8) + 10
    assert miner.search(e["nonce"], 6, 0, 0, 0, k1, bound=g).status == EXHAUSTED
    r = miner.search(e["nonce"], 6, 0, 0, 0, k1, bound=g + 1)
    assert r.status == FOUND and r.global_idx == g


def test_deterministic_repeats(miner):
    rs = {miner.mine([1, 2, 3, 4], 7).global_idx for _ in range(3)}
    assert rs == {231910082}


def test_min_over_partitions_equals_wbits0_on_gpu(miner):
    """Size-independent property at N = 9 (6.9e10 expected candidates, beyond the oracle):
    the hit verifies by hashlib, and min over the 8 partitions (workerBits = 3) equals
    the workerBits = 0 answer (the multi-GPU min-reduce rule)."""
    nonce = [1, 2, 3, 4]
    r0 = miner.mine(nonce, 9)
    assert r0.status == FOUND
    assert _hexz(nonce, r0.secret).endswith("0" * 9)
    k_stop = (r0.global_idx >> 8) + 1
    parts = [miner.search(nonce, 9, wb, 3, 0, k_stop) for wb in range(8)]
    found = [p.global_idx for p in parts if p.status == FOUND]
    assert min(found) == r0.global_idx
    for p in parts:
        if p.status == FOUND:
            assert _hexz(nonce, p.secret).endswith("0" * 9)


def test_cancel_flag_before_search(miner):
    miner.cancel()
    try:
        assert miner.search([1, 2, 3, 4], 32, 0, 0, 0, 1 << 30).status == CANCELLED
    finally:
        miner.clear_cancel()
    assert miner.search([1, 2, 3, 4], 3, 0, 0, 0, 1 << 10).status == FOUND


def test_cancel_mid_search_latency(miner):
    """Found/Cancel (worker.go:194,209) raise the pinned flag: the running kernel stops mid-launch."""
    out = {}

    def run():
        t0 = time.perf_counter()
        out["r"] = miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, 1 << 40)  # 2.8e14 candidates, 65k launches
        out["t_end"] = time.perf_counter()
        out["t0"] = t0

    th = threading.Thread(target=run)
    th.start()
    time.sleep(0.3)
    t_cancel = time.perf_counter()
    miner.cancel()
    th.join(timeout=30)
    miner.clear_cancel()
    assert not th.is_alive()
    assert out["r"].status == CANCELLED
    latency = out["t_end"] - t_cancel
    print(f"cancel latency {latency * 1e3:.2f} ms")
    assert latency < 0.25


def test_stats_count_candidates(miner):
    miner.reset_stats()
    r = miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + 4096)
    assert r.status == EXHAUSTED
    s = miner.stats()
    assert s.candidates == 4096 * 256 and s.launches == 1 and s.kernel_ms > 0


def test_min_over_8_partitions_n8_full_size(miner, golden):
    """BASELINE config 4 at full size: 8 partitions (workerBits = 3), N = 8; the
    minimum of the per-partition first hits is the golden workerBits = 0 answer,
    owned by partition 0."""
    e = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 8)
    hits = []
    for wb in range(8):
        r = miner.search([1, 2, 3, 4], 8, wb, 3, 0, (e["global_idx"] >> 8) + 1)
        if r.status == FOUND:
            assert distpow.verify([1, 2, 3, 4], r.secret, 8)
            hits.append((r.global_idx, wb))
    assert min(hits) == (e["global_idx"], 0)


def test_native_cli(tmp_path):
    """The C++ harness (distpow/dpow_cli) drives the C ABI without Python."""
    import json
    import os
    import subprocess
    cli = os.path.join(os.path.dirname(distpow.LIB_PATH), "dpow_cli")
    out = json.loads(subprocess.check_output([cli, "mine", "01020304", "7"], timeout=120).decode().strip())
    assert out["status"] == 1 and out["global_idx"] == 231910082 and out["secret"] == [194, 170, 210, 13]
    assert out["verified"] == 1
    out = json.loads(subprocess.check_output([cli, "mine", "01020304", "6", "2", "2"], timeout=120).decode())
    assert out["secret"] == [188, 163, 38]
    out = json.loads(subprocess.check_output([cli, "worker", "05060708", "5"], timeout=120).decode())
    assert out["secret"] == [84, 244, 3] and out["ack_is_nil"] == 1
    out = json.loads(subprocess.check_output([cli, "sweep", "32"], timeout=120).decode())
    assert out["status"] == 0 and out["candidates"] == 1 << 32
    print("cli sweep", out)


def test_window_spanning_80_segments(miner, oracle):
    """A window of 80 2^24-k segments (worker_bits = 8: one thread byte per k, 2^24
    candidates per segment) runs as one launch whose waves re-derive the segment
    words' constants 80 times: the whole window is hashed exactly once."""
    k0 = 1 << 24
    k1 = k0 + 80 * (1 << 24)
    miner.reset_stats()
    assert miner.search([1, 2, 3, 4], 32, 77, 8, k0, k1).status == EXHAUSTED
    s = miner.stats()
    assert s.launches == 1 and s.candidates == 80 * (1 << 24)
    # A late first hit in the same partition: hashlib-valid, and the oracle
    # agrees on the 4097 candidates ending at it (no earlier hit there).
    r = miner.search([1, 2, 3, 4], 8, 77, 8, k0, k1 + 400 * (1 << 24))
    assert r.status == FOUND and _hexz([1, 2, 3, 4], r.secret).endswith("0" * 8)
    k_hit = r.global_idx >> 8
    exp = oracle.mine_window([1, 2, 3, 4], 8, 77, 8, max(k0, k_hit - 4096), k_hit + 1)
    assert exp is not None and (exp[0], exp[1]) == (list(r.secret), r.global_idx)
    # The same window cut just below the hit: nothing before it, the same hit after.
    assert miner.search([1, 2, 3, 4], 8, 77, 8, k0, k_hit).status == EXHAUSTED
    r2 = miner.search([1, 2, 3, 4], 8, 77, 8, k_hit, k1 + 400 * (1 << 24))
    assert r2.status == FOUND and r2.global_idx == r.global_idx


def test_back_to_back_after_early_returns(miner, golden):
    """A search that returns at a hit leaves up to 3 queued launches behind it
    (they claim nothing); the next searches on the context must not see them."""
    e5 = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 5)
    for _ in range(20):
        r = miner.search([1, 2, 3, 4], 3, 0, 0, 0, 1 << 26)
        assert r.status == FOUND and r.global_idx == 97
        miner.reset_stats()
        assert miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, (1 << 24) + 4096).status == EXHAUSTED
        s = miner.stats()
        assert s.launches == 1 and s.candidates == 4096 * 256
        r = miner.search([1, 2, 3, 4], 5, 0, 0, 0, 1 << 26)
        assert r.status == FOUND and r.global_idx == e5["global_idx"]


def test_small_launch_grids_vs_oracle(miner, oracle):
    """Launches of 1..40 k per partition: grids of a few workgroups, fewer than
    the 8 claim counters, chunks of the minimum size."""
    rnd = random.Random(8)
    for wbits in (0, 3, 6, 8):
        wb = rnd.randrange(1 << wbits) if wbits else 0
        for n in list(range(1, 18)) + [24, 33, 40]:
            k0 = rnd.choice([0, 1, 200, 300, 70000, (1 << 24) + 5])
            ntz = rnd.choice([1, 2, 3])
            exp = oracle.mine_window([7, 7, 7, 7], ntz, wb, wbits, k0, k0 + n)
            r = miner.search([7, 7, 7, 7], ntz, wb, wbits, k0, k0 + n)
            if exp is None:
                assert r.status == EXHAUSTED, (wbits, wb, k0, n, ntz)
            else:
                assert r.status == FOUND and (list(r.secret), r.global_idx) == (exp[0], exp[1]), \
                    (wbits, wb, k0, n, ntz, r, exp)


def _secret_of(g):
    k = g >> 8
    return bytes([g & 255]) + k.to_bytes((k.bit_length() + 7) // 8, "little")


def _tz(nonce, secret):
    h = hashlib.md5(bytes(nonce) + bytes(secret)).hexdigest()
    return len(h) - len(h.rstrip("0"))


@pytest.mark.parametrize("nlen,wbits,wb", [(4, 0, 0), (11, 0, 0), (23, 0, 0), (46, 2, 3), (70, 0, 0),
                                           (129, 3, 5), (60, 0, 0)])
def test_n8_first_hit_vs_n7_walk(miner, nlen, wbits, wb):
    """The N >= 8 kernels (one final block: the D-equality test, raw state word ==
    -iv[3]) against the N = 7 kernels (prefilter D <= 0xFF + nibble mask), beyond the
    oracle's reach: walking the N = 7 hits in order up to the N = 8 answer g8, every
    candidate of every visited k below g8 (all of the partition's thread bytes, by
    hashlib) has < 8 trailing zeros, and g8 has >= 8.  Nonce lengths cover the
    plain, midstate (70, 129) and two-final-block (60) layouts."""
    rnd = random.Random(nlen * 131 + wbits)
    nonce = [1, 2, 3, 4] if nlen == 4 else [rnd.randrange(256) for _ in range(nlen)]
    r8 = miner.mine(nonce, 8, wb, wbits)
    assert r8.status == FOUND
    g8 = r8.global_idx
    assert bytes(r8.secret) == _secret_of(g8) and _tz(nonce, r8.secret) >= 8
    rb = 8 - wbits % 9
    tbs = [((wb << rb) | j) & 255 for j in range(1 << rb)]
    k, kend, walked = 0, (g8 >> 8) + 1, 0
    while True:
        r7 = miner.search(nonce, 7, wb, wbits, k, kend)
        assert r7.status == FOUND and r7.global_idx <= g8, (k, kend, r7)
        assert _tz(nonce, r7.secret) >= 7
        ks = r7.global_idx >> 8
        for t in tbs:
            g = (ks << 8) | t
            if g < g8:
                assert _tz(nonce, _secret_of(g)) < 8, (nonce, g, g8)
        walked += 1
        if ks == g8 >> 8:
            break
        k = ks + 1
    assert walked >= 1


SH3_LENGTHS = list(range(3, 64, 4)) + [67, 71, 119, 123]  # every <NBLK, W0, 3> layout, midstate too


def test_sh3_narrow_and_general_kernels_vs_oracle(miner, oracle):
    """SH = 3 layouts have two kernels (md5_search_kernel.h hash_wave_block KSPAN): the narrow
    one for launches with R >= 64 (workerBits 0-2), whose word W0 + 1 is wave-uniform, and the
    general one for R < 64, where a wave-block's lanes span several k.  Every SH = 3 layout,
    both kernels, windows in the L = 4 and L = 5 segments and across a 2^24-k segment boundary,
    against the oracle."""
    rnd = random.Random(3)
    for nlen in SH3_LENGTHS:
        nonce = [rnd.randrange(256) for _ in range(nlen)]
        for wbits in (0, 1, 2, 3, 5, 8):
            wb = rnd.randrange(1 << wbits) if wbits else 0
            rb = 8 - wbits
            nk = (1 << 16) >> rb  # ~65k candidates per window
            for k0 in ((1 << 24) + rnd.randrange(1 << 20), (1 << 32) + (rnd.randrange(256) << 24),
                       (3 << 24) - nk // 2):
                exp = oracle.mine_window(nonce, 3, wb, wbits, k0, k0 + nk)
                r = miner.search(nonce, 3, wb, wbits, k0, k0 + nk)
                if exp is None:
                    assert r.status == EXHAUSTED, (nlen, wb, wbits, k0, r)
                else:
                    assert r.status == FOUND and r.global_idx == exp[1] and list(r.secret) == exp[0], \
                        (nlen, wb, wbits, k0, r, exp)


@pytest.mark.parametrize("nlen", [7, 39, 51, 59])
def test_sh3_n9_narrow_equals_min_over_general_partitions(miner, nlen):
    """N = 9 (the full-digest check behind the D prefilter) beyond the oracle's reach: the
    workerBits = 0 answer of an SH = 3 layout (its narrow kernel) equals the minimum over the 8
    partitions of workerBits = 3 (its general kernel), each searched up to that answer's k, and
    every partition's hit verifies with hashlib (<1,1,3>, <1,9,3>, <2,12,3>, <2,14,3>)."""
    rnd = random.Random(9000 + nlen)
    nonce = [rnd.randrange(256) for _ in range(nlen)]
    r0 = miner.mine(nonce, 9)
    assert r0.status == FOUND and bytes(r0.secret) == _secret_of(r0.global_idx) and _tz(nonce, r0.secret) >= 9
    kend = (r0.global_idx >> 8) + 1
    gs = []
    for wb in range(8):
        r = miner.search(nonce, 9, wb, 3, 0, kend)
        if r.status == FOUND:
            assert _tz(nonce, r.secret) >= 9 and (r.global_idx & 255) >> 5 == wb, (wb, r)
            gs.append(r.global_idx)
        else:
            assert r.status == EXHAUSTED, (wb, r)
    assert min(gs) == r0.global_idx, (gs, r0.global_idx)


def _all_hits(miner, nonce, ntz, wb, wbits, k0, k1, cap=2000):
    """Every hit of a window, in order: repeated searches resuming after each hit."""
    hits, bound_k = [], k0
    rb = 8 - wbits % 9
    while bound_k < k1 and len(hits) < cap:
        r = miner.search(nonce, ntz, wb, wbits, bound_k, k1)
        if r.status != FOUND:
            break
        hits.append(r.global_idx)
        # resume at the same k for partitions with several thread bytes per k
        k = r.global_idx >> 8
        tbs = [((wb << rb) | j) & 255 for j in range(1 << rb)]
        later = [t for t in tbs if t > (r.global_idx & 255)]
        for t in later:  # the rest of this k, candidate by candidate (the window API is per k)
            g = (k << 8) | t
            if distpow.verify(nonce, _secret_of(g), ntz):
                hits.append(g)
        bound_k = k + 1
    return hits


@pytest.mark.parametrize("nlen,first_k,nseg", [
    (4, (1 << 24) + 12345, 12),                # SH 0, L = 4
    (5, (7 << 24) - 999, 10),                  # SH 1
    (6, (200 << 24) + 1, 9),                   # SH 2
    (7, (1 << 32) + (250 << 24) + 77, 12),     # SH 3, L = 5: k >> 24 carries from word W0+1 into W0+2
    (8, (1 << 32) + (3 << 24) - 5, 6),         # L = 5, SH 0
    (60, (1 << 24) + 3, 6),                    # two final blocks, W0 = 15: the segment word is block 1's word 0
    (63, (1 << 32) + (254 << 24), 5),          # two final blocks, SH 3, L = 5: words 16 and 17
    # chunks of 6 and 7 bytes (k >= 2^40; DPOW_K_LIMIT = 2^55 - 1)
    (4, (1 << 40) + (0xFE << 32) + (250 << 24) + 5, 10),      # SH 0, L = 6: k >> 24 carries over two bytes
    (5, (7 << 40) + (0xFFFF << 24) - 3, 6),                   # SH 1, L = 6: three bytes in word W0+1
    (6, (5 << 40) - (3 << 24) - 7, 6),                        # SH 2, L = 6: word W0+2 changes at 5 * 2^40
    (7, (3 << 48) + (0x12 << 40) + (0xFF << 32) + (0xFD << 24) + 11, 6),  # SH 3, L = 7: W0+1 -> W0+2 carry
    (5, (9 << 48) - (2 << 24) - 1, 5),                        # SH 1, L = 7: word W0+2 changes at 9 * 2^48
    (60, (1 << 50) + (0xFF << 24) + 9, 5),                    # two blocks, W0 = 15, SH 0, L = 7
    (62, (2 << 40) - (2 << 24) + 1, 5),                       # two blocks, SH 2, L = 6, across 2 * 2^40
    (4, (1 << 55) - 1 - (3 << 24) - 100, 3),                  # the top of the k range
])
def test_spanning_launch_equals_per_segment_windows(miner, oracle, nlen, first_k, nseg):
    """The segment-word path (launches spanning 2^24-k segments): one search over a window spanning nseg 2^24-k
    segments from an unaligned k finds exactly the hits that searches confined to one
    segment each find (there the template holds the segment's own k >> 24 bytes), and
    the first one agrees with the byte-wise oracle on the 4096 k before it."""
    rnd = random.Random(nlen)
    nonce = [1, 2, 3, 4] if nlen == 4 else [rnd.randrange(256) for _ in range(nlen)]
    wb, wbits, ntz = rnd.randrange(256), 8, 5  # ~16 hits per segment: every segment's constants are checked
    k1 = first_k + nseg * (1 << 24)
    span = _all_hits(miner, nonce, ntz, wb, wbits, first_k, k1)
    per = []
    k = first_k
    while k < k1:
        ke = min(k1, ((k >> 24) + 1) << 24)
        per += _all_hits(miner, nonce, ntz, wb, wbits, k, ke)
        k = ke
    assert span == per and len(span) >= 4 * nseg, (nlen, len(span), len(per))
    assert len({g >> 32 for g in span}) >= nseg  # hits in every segment the window covers
    for g in span:
        assert distpow.verify(nonce, _secret_of(g), ntz)
    kh = span[0] >> 8
    exp = oracle.mine_window(nonce, ntz, wb, wbits, max(first_k, kh - 4096), kh + 1)
    assert exp is not None and exp[1] == span[0]


def test_spanning_launch_partition_wbits3(miner):
    """The same at workerBits 3 (32 thread bytes per k, the 8-GPU partition): a window of
    8 segments from an unaligned k, one search vs per-segment searches, N = 6."""
    nonce, wb, wbits, ntz = [2, 2, 2, 2], 5, 3, 6
    k0 = (1 << 24) + 4321
    k1 = k0 + 8 * (1 << 24)
    span = _all_hits(miner, nonce, ntz, wb, wbits, k0, k1)
    per, k = [], k0
    while k < k1:
        ke = min(k1, ((k >> 24) + 1) << 24)
        per += _all_hits(miner, nonce, ntz, wb, wbits, k, ke)
        k = ke
    assert span == per and len(span) >= 8 * 4


def test_deep_hits_golden(miner, golden):
    """N = 9 / 10 first hits (tests/golden/gen_golden.py --deep): BASELINE config 5's fresh
    nonces seeded random.Random(416) at N = 9, the
    config-1/2/5 nonces at N = 9 and [1,2,3,4] at N = 10 -- the full-digest path
    (C word, then B, A) that N > 8 needs beyond the D-word test (worker.go:246-256)."""
    deep = golden["deep_hits"]
    assert {tuple(e["nonce"]) for e in deep if e["case"].startswith("config5-fresh")} == \
        {(129, 3, 150, 161), (226, 19, 170, 24), (111, 251, 228, 114), (199, 4, 151, 255)}
    for e in deep:
        r = miner.mine(e["nonce"], e["ntz"])
        assert r.status == FOUND, e
        assert (r.global_idx, list(r.secret)) == (e["global_idx"], e["secret"]), (e, r)
        assert _hexz(e["nonce"], r.secret) == e["md5"] and e["md5"].endswith("0" * e["ntz"])


def test_concurrent_deep_hits_in_shared_launches(golden):
    """The four config-5 fresh nonces at N = 9 mined at once on one GPU: while the device is
    shared, dpow_search cuts each window into ~8 ms launches and re-sizes every grid
    (plan.h grid_share, cap_shared_launch), so each hit (4.5e10-1.1e11 candidates in) lies
    behind hundreds of launch boundaries.  Every answer is still the golden."""
    deep = [e for e in golden["deep_hits"] if e["case"].startswith("config5-fresh")]
    assert len(deep) == 4
    miners = [distpow.Miner(0) for _ in deep]
    out = {}
    try:
        def run(i, e):
            miners[i].reset_stats()
            out[i] = (miners[i].mine(e["nonce"], e["ntz"]), miners[i].stats().launches)
        ths = [threading.Thread(target=run, args=(i, e)) for i, e in enumerate(deep)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=90)
        assert not any(t.is_alive() for t in ths)
        for i, e in enumerate(deep):
            r, launches = out[i]
            assert r.status == FOUND and (r.global_idx, list(r.secret)) == (e["global_idx"], e["secret"]), (e, r)
        # the shortest search ran beside the three others throughout: many short launches
        assert min(n for _, n in out.values()) >= 20, {i: n for i, (_, n) in out.items()}
    finally:
        for m in miners:
            m.close()


def test_shared_capped_windows_vs_oracle(oracle, monkeypatch):
    """Searches sharing the GPU cut their windows into short launches (plan.h
    cap_shared_launch), each re-planned from where the last ended and re-sized to the searches
    in flight.  With the launch length forced down to 2 us (DPOW_DIAG_SHARE_LAUNCH_US, read at
    dpow_open), four concurrent searches over oracle-sized windows -- across the chunk-length
    boundaries k = 256, 65536 and 2^24, every nonce-length family, hits anywhere in the window
    or none -- run as 2-15 launches each, and every answer is the oracle's."""
    rnd = random.Random(2026)
    cases = []
    for _ in range(16):
        nonce = [rnd.randrange(256) for _ in range(rnd.choice([0, 3, 4, 4, 7, 50, 53, 55, 56, 59, 60, 63, 64]))]
        wbits = rnd.choice([0, 0, 1, 2, 3, 5])
        wb = rnd.randrange(1 << wbits) if wbits else 0
        rb = 8 - wbits
        ntz = rnd.choice([4, 5, 5, 5, 6])
        nk = max(1, (1 << rnd.choice([18, 19, 20])) >> rb)
        edge = rnd.choice([0, 256, 1 << 16, 1 << 24, None])
        k0 = rnd.randrange(1, 1 << 30) if edge is None else max(0, edge - rnd.randrange(0, nk))
        cases.append((nonce, ntz, wb, wbits, k0, k0 + nk))
    expected = [oracle.mine_window(*c) for c in cases]
    monkeypatch.setenv("DPOW_DIAG_SHARE_LAUNCH_US", "2")
    miners = [distpow.Miner(0) for _ in range(4)]
    monkeypatch.delenv("DPOW_DIAG_SHARE_LAUNCH_US")
    out, launches = {}, {}
    try:
        go = threading.Barrier(4)

        def run(t):
            go.wait()
            for i in range(t, len(cases), 4):
                miners[t].reset_stats()
                out[i] = miners[t].search(*cases[i])
                launches[i] = miners[t].stats().launches
        ths = [threading.Thread(target=run, args=(t,)) for t in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=60)
        assert not any(t.is_alive() for t in ths)
        for i, (c, exp) in enumerate(zip(cases, expected)):
            r = out[i]
            if exp is None:
                assert r.status == EXHAUSTED, (i, c, r)
            else:
                assert r.status == FOUND and r.global_idx == exp[1] and list(r.secret) == exp[0], (i, c, r, exp)
        assert max(launches.values()) >= 4, launches  # the cap cut the windows
    finally:
        for m in miners:
            m.close()


def test_n10_min_over_8_partitions(miner, golden):
    """N = 10 on [1,2,3,4] (1.1e12 candidates expected; about 5 s per pass): the minimum of
    the 8 workerBits = 3 partitions' first hits is the workerBits = 0 golden, and the
    N = 9 first hit comes no later."""
    e = next(x for x in golden["deep_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 10)
    g10 = e["global_idx"]
    k_stop = (g10 >> 8) + 1
    hits = []
    for wb in range(8):
        r = miner.search([1, 2, 3, 4], 10, wb, 3, 0, k_stop)
        if r.status == FOUND:
            assert _tz([1, 2, 3, 4], r.secret) >= 10
            hits.append((r.global_idx, wb))
    assert min(hits) == (g10, (g10 & 255) >> 5)
    e9 = next(x for x in golden["deep_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 9)
    assert e9["global_idx"] <= g10
    r9 = miner.search([1, 2, 3, 4], 9, 0, 0, 0, k_stop)
    assert r9.status == FOUND and r9.global_idx == e9["global_idx"]


def test_search_bound_from_another_thread(miner, golden):
    """dpow_search_bound (Miner.bound): a bound injected into the running search stops it
    at that index.  Below the bound the search's own hit still wins; above it, nothing is
    wanted and the search returns EXHAUSTED; the bound does not leak into the next search."""
    e8 = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 8)
    g8 = e8["global_idx"]  # ~19 ms into the search

    def run_with_bound(ntz, k0, k1, g, delay, repeat=False):
        out = {}
        th = threading.Thread(target=lambda: out.update(r=miner.search([1, 2, 3, 4], ntz, 0, 0, k0, k1),
                                                       t=time.perf_counter()))
        th.start()
        time.sleep(delay)
        t0 = time.perf_counter()
        miner.bound(g)
        # a bound that lands before the thread's search has opened applies to nothing
        # (dpow_search_bound: no search in flight): repeat it until the search returns
        while repeat and th.is_alive():
            time.sleep(0.001)
            miner.bound(g)
        th.join(timeout=30)
        assert not th.is_alive()
        return out["r"], out["t"] - t0

    r, _ = run_with_bound(8, 0, 1 << 32, g8 + 1000, 0.002, repeat=True)  # own hit below the bound: FOUND
    assert r.status == FOUND and r.global_idx == g8
    r, _ = run_with_bound(8, 0, 1 << 32, g8 - 1, 0.002, repeat=True)     # the bound is below the hit: nothing wanted
    assert r.status == EXHAUSTED
    # unreachable N, bound below the point the search has reached after 0.3 s (~2^28 k):
    # the running kernel stops at its next group
    r, lat = run_with_bound(32, 1 << 24, 1 << 40, ((1 << 24) + (1 << 20)) << 8, 0.3)
    assert r.status == EXHAUSTED and lat < 0.25, lat
    print(f"bound -> return {lat * 1e3:.2f} ms")
    e6 = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 6)
    r = miner.search([1, 2, 3, 4], 6, 0, 0, 0, 1 << 30)
    assert r.status == FOUND and r.global_idx == e6["global_idx"]
    miner.bound(5)  # no search in flight: no effect
    r = miner.search([1, 2, 3, 4], 6, 0, 0, 0, 1 << 30)
    assert r.status == FOUND and r.global_idx == e6["global_idx"]


class _Slot(ctypes.Structure):
    """dpow_node_slot (include/dpow.h)."""
    _fields_ = [("best", ctypes.c_uint64), ("stop", ctypes.c_uint32), ("pad", ctypes.c_uint32 * 13)]


def test_bound_beyond_a_chunk_length_split(miner, golden):
    """a bound from another partition that lies past the launch being
    consumed must not end the search -- later launches of the window (here the L = 3
    segment after the L = 2 one: the window splits at k = 2^16) still hold candidates
    below it, among them this search's own first hit.  The bound is the node slot's best
    at the search's start (deterministic: the first launch's record already shows it)."""
    e7 = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 8)
    g7 = e7["global_idx"]  # k = 15,880,380: in the L = 3 launch of a window from k = 256
    assert (g7 >> 8) > (1 << 16)
    # N = 8 expects its first hit too late to merge chunk lengths 2 and 3 into one launch
    # (plan.cpp lspan_layout): the window is two launches, split at k = 2^16
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window([1, 2, 3, 4], 0, 0, 256, 1 << 24, 8)] == \
        [(256, 1 << 16), (1 << 16, 1 << 24)]
    slot = _Slot()
    lib = distpow.lib()
    addr = ctypes.addressof(slot)
    try:
        miner.attach_node(addr)
        for b, want in ((g7 + 1000, (FOUND, g7)),          # beyond launch 0's end, above our hit
                        ((1 << 24) << 8, (FOUND, g7)),     # at the window's end
                        (g7 - 1, (EXHAUSTED, None)),       # below our hit: nothing wanted
                        (((1 << 16) - 7) << 8, (EXHAUSTED, None))):  # inside launch 0
            lib.dpow_node_slot_reset(addr)
            lib.dpow_node_post(addr, b)
            r = miner.search([1, 2, 3, 4], 8, 0, 0, 256, 1 << 24)
            assert (r.status, r.global_idx if r.status == FOUND else None) == want, (b, r)
            # a hit is posted to the slot (atomic min); a bounded search leaves it alone
            assert slot.best == (min(b, g7) if r.status == FOUND else b) and slot.stop == 0
        # a raised stop: the search returns CANCELLED at once and does not hash
        lib.dpow_node_slot_reset(addr)
        lib.dpow_node_stop(addr)
        t0 = time.perf_counter()
        assert miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, 1 << 40).status == CANCELLED
        assert time.perf_counter() - t0 < 0.05
    finally:
        miner.attach_node(None)
    # detached: the same window finds the hit without any bound
    r = miner.search([1, 2, 3, 4], 8, 0, 0, 256, 1 << 24)
    assert r.status == FOUND and r.global_idx == g7


def test_node_stop_ends_a_running_search(miner):
    """The node slot's stop raised from another thread (another rank was cancelled or
    failed) ends a running search within a fraction of a second: DPOW_CANCELLED."""
    slot = _Slot()
    addr = ctypes.addressof(slot)
    lib = distpow.lib()
    lib.dpow_node_slot_reset(addr)
    miner.attach_node(addr)
    try:
        out = {}
        th = threading.Thread(target=lambda: out.update(r=miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, 1 << 40),
                                                       t=time.perf_counter()))
        th.start()
        time.sleep(0.3)
        t0 = time.perf_counter()
        lib.dpow_node_stop(addr)
        th.join(timeout=30)
        assert not th.is_alive() and out["r"].status == CANCELLED
        lat = out["t"] - t0
        assert lat < 0.25, lat
        print(f"node stop -> return {lat * 1e3:.2f} ms")
    finally:
        miner.attach_node(None)
    # nothing leaks into the next search (stale launches stopped, flag untouched)
    r = miner.search([1, 2, 3, 4], 6, 0, 0, 0, 1 << 30)
    assert r.status == FOUND


def _stopped_by_node(miner, lib, addr):
    """A running unreachable search on `miner` ends CANCELLED when the slot's stop is raised."""
    lib.dpow_node_slot_reset(addr)
    out = {}
    th = threading.Thread(target=lambda: out.update(r=miner.search([1, 2, 3, 4], 32, 0, 0, 1 << 24, 1 << 40),
                                                   t=time.perf_counter()))
    th.start()
    time.sleep(0.2)
    t0 = time.perf_counter()
    lib.dpow_node_stop(addr)
    th.join(timeout=30)
    assert not th.is_alive() and out["r"].status == CANCELLED
    return out["t"] - t0


def test_two_contexts_share_a_slot_one_closes(miner, golden):
    """the slot's host page is registered once per process and held by
    every context that attached it (dpow_api.cpp page registry).  Two contexts attach one
    slot; closing one must not unregister the page under the other, whose kernels' watcher
    still stops at the node's stop and bound.  dpow_node_release refuses while a context is
    attached and, once detached, drops the registration; attaching again registers afresh."""
    slot = _Slot()
    addr = ctypes.addressof(slot)
    lib = distpow.lib()
    lib.dpow_node_slot_reset(addr)
    other = distpow.Miner(distpow.device_count() - 1)  # another GPU when the box has one
    try:
        other.attach_node(addr)
        miner.attach_node(addr)
        # each context's watcher reads the slot through its own device's alias
        for m in (other, miner):
            cached, lookup = ctypes.c_void_p(), ctypes.c_void_p()
            assert lib.dpow_diag_node_alias(m._ctx, ctypes.byref(cached), ctypes.byref(lookup)) == 0
            assert cached.value == lookup.value and cached.value
        assert other.search([1, 2, 3, 4], 3, 0, 0, 0, 1 << 10).status == FOUND  # other's launches used the page
    finally:
        other.close()  # drops other's hold; the miner's keeps the page registered
    cached, lookup = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.dpow_diag_node_alias(miner._ctx, ctypes.byref(cached), ctypes.byref(lookup)) == 0
    assert cached.value == lookup.value
    try:
        assert _stopped_by_node(miner, lib, addr) < 0.25
        # the node's best through the page: a bound below the answer leaves nothing to find
        e = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 7)
        lib.dpow_node_slot_reset(addr)
        lib.dpow_node_post(addr, e["global_idx"] - 1)
        assert miner.search([1, 2, 3, 4], 7, 0, 0, 0, 1 << 26).status == EXHAUSTED
        lib.dpow_node_slot_reset(addr)
        assert lib.dpow_node_release(addr, ctypes.sizeof(slot)) == -1  # still attached
    finally:
        miner.attach_node(None)
    assert lib.dpow_node_release(addr, ctypes.sizeof(slot)) == 0
    miner.attach_node(addr)  # registered afresh
    try:
        assert _stopped_by_node(miner, lib, addr) < 0.25
    finally:
        miner.attach_node(None)
    r = miner.search([1, 2, 3, 4], 7, 0, 0, 0, 1 << 26)
    assert r.status == FOUND and r.global_idx == e["global_idx"]


def test_early_found_fan_out(miner, golden):
    """Round 4: a search attached to a node slot posts its verified hit to the slot while its
    launch still drains (the watcher relays Ctrl::best to a pinned word, the searching thread
    verifies and posts it: dpow_diag_search_times[7]), before the search returns ([3]); the
    posted value is the search's own answer, and a bound that is not a hit (posted by the
    test) is never taken for one.  Partition case: workerBits 3, the owner of [1,2,3,4]/7."""
    e = next(x for x in golden["first_hits"] if x["nonce"] == [1, 2, 3, 4] and x["ntz"] == 7)
    g = e["global_idx"]
    wb = (g & 0xFF) >> 5
    slot = _Slot()
    addr = ctypes.addressof(slot)
    lib = distpow.lib()
    tl = (ctypes.c_int64 * 8)()
    miner.attach_node(addr)
    try:
        for _ in range(3):
            lib.dpow_node_slot_reset(addr)
            r = miner.search([1, 2, 3, 4], 7, wb, 3, 0, 1 << 24)
            assert r.status == FOUND and r.global_idx == g
            assert slot.best == g
            lib.dpow_diag_search_times(miner._ctx, tl)
            assert 0 <= tl[7] < tl[3], list(tl)
        # a bound that is no hit, above the answer: still our hit, and nothing else posted
        lib.dpow_node_slot_reset(addr)
        lib.dpow_node_post(addr, g + 3)
        r = miner.search([1, 2, 3, 4], 7, wb, 3, 0, 1 << 24)
        assert r.status == FOUND and r.global_idx == g and slot.best == g
    finally:
        miner.attach_node(None)


def test_concurrent_searches_share_the_gpu(golden):
    """Four contexts searching at once on one GPU (each sizes its grids to its share of the
    device, dpow_api.cpp ActiveSearch): every answer is still the golden, and a concurrent
    unreachable search is cancelled without disturbing the others."""
    cases = [([1, 2, 3, 4], 7), ([2, 2, 2, 2], 8), ([5, 6, 7, 8], 5), ([1, 2, 3, 4], 8)]
    exp = {(tuple(e["nonce"]), e["ntz"]): e for e in golden["first_hits"]}
    miners = [distpow.Miner(0) for _ in range(len(cases) + 1)]
    out = {}
    try:
        def run(i, nonce, ntz):
            out[i] = miners[i].mine(nonce, ntz)

        def run_forever():
            out["inf"] = miners[-1].search([9, 9, 9, 9], 32, 0, 0, 1 << 24, 1 << 40)

        ths = [threading.Thread(target=run, args=(i, n, z)) for i, (n, z) in enumerate(cases)]
        ths.append(threading.Thread(target=run_forever))
        for t in ths:
            t.start()
        for t in ths[:-1]:
            t.join(timeout=60)
        miners[-1].cancel()
        ths[-1].join(timeout=30)
        miners[-1].clear_cancel()
        assert not any(t.is_alive() for t in ths)
        for i, (nonce, ntz) in enumerate(cases):
            e = exp[(tuple(nonce), ntz)]
            assert out[i].status == FOUND and (out[i].global_idx, list(out[i].secret)) == (e["global_idx"], e["secret"])
        assert out["inf"].status == CANCELLED
    finally:
        for m in miners:
            m.close()


def test_windows_from_k0_vs_oracle(miner, oracle):
    """Windows from k = 0 (the search's k = 0 kernel, search_ctrl.hip, ahead of its first md5
    launch; k = 0 alone, k = 0 with one more k, with chunk lengths 1-2, 1-3): hits at k = 0 and
    above it, partition widths 0-5 bits, nonces of 4, 5, 8 and 12 bytes, a bound inside k = 0."""
    rnd = random.Random(5150)
    checked = 0
    for nlen in (4, 5, 8, 12):
        for ntz in (1, 2, 3):
            for wbits in (0, 1, 3, 5):
                nonce = [rnd.randrange(256) for _ in range(nlen)]
                wb = rnd.randrange(1 << wbits)
                for k1 in (1, 2, 300, 70000):
                    exp = oracle.mine_window(nonce, ntz, wb, wbits, 0, k1)
                    r = miner.search(nonce, ntz, wb, wbits, 0, k1)
                    if exp is None:
                        assert r.status == EXHAUSTED, (nonce, ntz, wb, wbits, k1, r)
                    else:
                        assert r.status == FOUND and (list(r.secret), r.global_idx) == (exp[0], exp[1]), \
                            (nonce, ntz, wb, wbits, k1, r, exp)
                    checked += 1
                # a bound inside k = 0: only a hit below it counts
                exp = oracle.mine_window(nonce, ntz, wb, wbits, 0, 300)
                if exp is not None and exp[1] < 256:
                    r = miner.search(nonce, ntz, wb, wbits, 0, 300, bound=exp[1] + 1)
                    assert r.status == FOUND and r.global_idx == exp[1], (nonce, ntz, wb, wbits, r, exp)
                    r = miner.search(nonce, ntz, wb, wbits, 0, 300, bound=exp[1])
                    assert r.status == EXHAUSTED, (nonce, ntz, wb, wbits, r, exp)
    assert checked == 4 * 3 * 4 * 4

