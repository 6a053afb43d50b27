"""Host logic of the product (libdpow.so), checked on CPU against the oracle.

Covers the planner that turns a search window into kernel launches and the
per-lane message assembly the kernel performs (dpow_plan_candidate shares the
kernel's lane arithmetic), plus the host MD5 used to re-verify every hit.
"""
import hashlib
import random

import pytest

import _md5py
import distpow


def test_host_md5_rfc1321(golden):
    for e in golden["rfc1321"]:
        assert distpow.md5(bytes.fromhex(e["msg_hex"])).hex() == e["md5"]


@pytest.mark.parametrize("ln", [0, 3, 55, 56, 64, 100, 128, 300])
def test_host_md5_vs_hashlib(ln):
    m = bytes(random.Random(ln).randrange(256) for _ in range(ln))
    assert distpow.md5(m) == hashlib.md5(m).digest()


def test_trailing_zero_nibbles_matches_hex():
    rnd = random.Random(1)
    for _ in range(2000):
        d = bytes(rnd.randrange(256) for _ in range(16))
        # force some zero tails
        z = rnd.randrange(0, 33)
        h = d.hex()
        h = h[:32 - z] + "0" * z
        d = bytes.fromhex(h)
        exp = len(h) - len(h.rstrip("0"))
        assert distpow.trailing_zero_nibbles(d) == exp


def test_verify_and_secret_from_index(golden):
    for e in golden["first_hits"]:
        s = distpow.secret_from_index(e["global_idx"])
        assert list(s) == e["secret"]
        assert distpow.verify(e["nonce"], s, e["ntz"])
        assert not distpow.verify(e["nonce"], s, 33)


def test_thread_bytes_mirror(oracle):
    for wb, wbits in [(0, 0), (3, 2), (5, 3), (3, 9), (1, 10), (7, 8)]:
        assert distpow.thread_bytes(wb, wbits) == oracle.thread_bytes(wb, wbits)


def test_plan_window_segments():
    pl = distpow.plan_window(b"\x01\x02\x03\x04", 0, 0, 0, (1 << 24) + 5)
    spans = [(p.k_begin, p.k_end, p.chunk_len, p.chunk_len_last, p.start_kernel) for p in pl]
    # k = 0 in the start kernel; chunk lengths 1..3 in one launch (SH = 0); then L = 4
    assert spans == [(0, 1, 0, 0, 1), (1, 1 << 24, 1, 3, 0), (1 << 24, (1 << 24) + 5, 4, 4, 0)]
    for p in pl:
        assert (p.nblk, p.w0, p.sh) == (1, 1, 0)  # 4-byte nonce: V lands in word 1
        assert p.i_begin == p.k_begin * 256 and p.i_end == p.k_end * 256
    # a first hit expected late (N = 8 at R = 256: 2^32 candidates) merges chunk lengths 1 and
    # 2 only: the chunk length 3 launch runs the per-length kernel, which hashes ~2 % faster
    # (plan.cpp lspan_end)
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window(b"\x01\x02\x03\x04", 0, 0, 0, 70000, 8)] == \
        [(0, 1), (1, 65536), (65536, 70000)]
    assert len(distpow.plan_window(b"\x01\x02\x03\x04", 0, 0, 0, 70000, 7)) == 2
    assert len(distpow.plan_window(b"\x01\x02\x03\x04", 5, 3, 0, 70000, 8)) == 3  # 2^29 > 2^28
    # a window inside the merged range, and one from k = 300
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window(b"\x01\x02\x03\x04", 0, 0, 200, 70000)] == \
        [(200, 70000)]
    # SH != 0 layouts and R = 1 (workerBits 8) keep one launch per chunk length
    for nonce, wb, wbits in ((b"abc", 0, 0), (b"abcde", 0, 0), (b"abcd", 3, 8)):
        assert [(p.k_begin, p.k_end, p.chunk_len) for p in distpow.plan_window(nonce, wb, wbits, 0, 70000)] == \
            [(0, 1, 0), (1, 256, 1), (256, 65536, 2), (65536, 70000, 3)], nonce
    # 52-byte nonce (W0 = 13, SH = 0): chunk length 3 needs a second block -- merged up to it
    pl = distpow.plan_window(bytes(52), 0, 0, 0, 70000)
    assert [(p.k_begin, p.k_end, p.nblk) for p in pl] == [(0, 1, 1), (1, 65536, 1), (65536, 70000, 2)]
    # L >= 4: one launch spans the 2^24-k segments (the kernel re-derives the constants
    # of the words holding k >> 24); windows split only where the chunk length changes
    pl = distpow.plan_window(b"ab", 2, 2, (3 << 24) - 7, (5 << 24) + 3)
    assert [(p.k_begin, p.k_end, p.chunk_len) for p in pl] == [((3 << 24) - 7, (5 << 24) + 3, 4)]
    assert all(p.i_begin == p.k_begin * 64 for p in pl)
    pl = distpow.plan_window(b"ab", 0, 0, (1 << 32) - 9, (1 << 32) + 2 * (1 << 24))
    assert [(p.k_begin, p.k_end, p.chunk_len) for p in pl] == [((1 << 32) - 9, 1 << 32, 4),
                                                               (1 << 32, (1 << 32) + (2 << 24), 5)]
    # L = 6 / 7 (k >= 2^40): for SH = 1-2 the top chunk bytes reach word W0 + 2, which
    # the kernel holds launch-uniform, so launches also end where it changes (every
    # 2^40 k for SH = 2, 2^48 for SH = 1); SH = 0 / 3 windows split only at chunk lengths
    w = ((3 << 40) - 5, (4 << 40) + 9)
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window(b"ab", 0, 0, *w)] == \
        [((3 << 40) - 5, 3 << 40), (3 << 40, (4 << 40)), (4 << 40, (4 << 40) + 9)]  # SH = 2
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window(b"abc", 0, 0, *w)] == [w]  # SH = 3
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window(b"abcd", 0, 0, *w)] == [w]  # SH = 0
    assert [(p.k_begin, p.k_end) for p in distpow.plan_window(b"a", 0, 0, *w)] == [w]  # SH = 1: 2^48
    w = ((2 << 48) - 3, (2 << 48) + 3)
    assert [(p.k_begin, p.k_end, p.chunk_len) for p in distpow.plan_window(b"a", 0, 0, *w)] == \
        [((2 << 48) - 3, 2 << 48, 7), (2 << 48, (2 << 48) + 3, 7)]
    assert len(distpow.plan_window(b"abc", 0, 0, *w)) == 1
    # the top of the k range: k < DPOW_K_LIMIT = 2^55 - 1, so every global index
    # k * 256 + t is below DPOW_NO_HIT = 2^63 - 1
    assert distpow.DPOW_K_LIMIT == (1 << 55) - 1
    assert ((distpow.DPOW_K_LIMIT - 1) << 8 | 255) < distpow.DPOW_NO_HIT
    pl = distpow.plan_window(b"x", 0, 0, distpow.DPOW_K_LIMIT - 4, distpow.DPOW_K_LIMIT)
    assert [(p.k_begin, p.k_end, p.chunk_len) for p in pl] == [(distpow.DPOW_K_LIMIT - 4, distpow.DPOW_K_LIMIT, 7)]
    # beyond the k limit
    with pytest.raises(distpow.DpowError):
        distpow.plan_window(b"x", 0, 0, 0, distpow.DPOW_K_LIMIT + 1)


def _expected_words(nonce: bytes, secret: bytes):
    msg = nonce + secret
    blocks = _md5py.padded_blocks(msg)
    blk_v = len(nonce) // 64
    st = _md5py.IV
    for b in blocks[:blk_v]:
        st = _md5py.compress(st, b)
    words = [w for b in blocks[blk_v:] for w in b]
    return list(st), words, len(blocks) - blk_v


def _check_candidate(nonce, wb, wbits, local_idx):
    rb = 8 - wbits % 9
    k, t = local_idx >> rb, local_idx & ((1 << rb) - 1)
    tb = ((wb << rb) | t) & 0xFF
    chunk = []
    kk = k
    while kk:
        chunk.append(kk & 0xFF)
        kk >>= 8
    secret = bytes([tb] + chunk)
    iv, words, nblk = distpow.plan_candidate(nonce, wb, wbits, local_idx)
    eiv, ewords, enblk = _expected_words(bytes(nonce), secret)
    assert (iv, words, nblk) == (eiv, ewords, enblk), (len(nonce), wb, wbits, local_idx)
    # and the digest of that chain is MD5(nonce || secret)
    st = tuple(iv)
    for i in range(nblk):
        st = _md5py.compress(st, words[16 * i:16 * i + 16])
    assert _md5py.digest_from_state(st) == hashlib.md5(bytes(nonce) + secret).digest()


@pytest.mark.parametrize("nlen", list(range(0, 72)) + [100, 119, 120, 121, 127, 128, 190, 250])
def test_candidate_words_every_layout(nlen):
    """Every (NBLK, W0, SH) layout: per-lane words == padded MD5 message of nonce || secret."""
    rnd = random.Random(nlen)
    nonce = bytes(rnd.randrange(256) for _ in range(nlen))
    for wb, wbits in [(0, 0), (1, 2), (6, 3), (3, 8), (2, 1), (5, 9)]:
        rb = 8 - wbits % 9
        for k in (0, 1, 200, 255, 256, 4097, 65535, 65536, 1 << 20, (1 << 24) - 1, 1 << 24,
                  (1 << 24) + 77, (1 << 32) - 1, 1 << 32, (1 << 33) + 12345, (1 << 40) - 1, 1 << 40,
                  (5 << 40) + 99, (1 << 48) - 1, 1 << 48, (0x3456 << 40) + 7, (1 << 55) - 2):
            for t in {0, (1 << rb) - 1, rnd.randrange(1 << rb)}:
                _check_candidate(nonce, wb, wbits, (k << rb) | t)


def test_candidate_words_random_lanes():
    rnd = random.Random(7)
    for _ in range(3000):
        nlen = rnd.choice([0, 1, 3, 4, 5, 8, 13, 50, 51, 52, 53, 54, 55, 60, 61, 62, 63, 64, 70])
        nonce = bytes(rnd.randrange(256) for _ in range(nlen))
        wbits = rnd.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11])
        wb = rnd.randrange(256) if wbits in (0, 9) else rnd.randrange(1 << (wbits % 9) if wbits % 9 else 1)
        rb = 8 - wbits % 9
        k = rnd.choice([rnd.randrange(1 << 8), rnd.randrange(1 << 16), rnd.randrange(1 << 24),
                        rnd.randrange(1 << 32), rnd.randrange(1 << 40), rnd.randrange(1 << 48),
                        rnd.randrange((1 << 55) - 1)])
        _check_candidate(nonce, wb, wbits, (k << rb) | rnd.randrange(1 << rb))
