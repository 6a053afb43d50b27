"""Claim geometry of dpow_search's launches (host logic; no GPU): plan.cpp size_launch via
dpow_diag_launch_geometry.  Invariants the kernel relies on (md5_search_kernel.h):

* the wave-blocks from wb_begin (a multiple of the wave-block size, <= i_begin) cover
  i_end, and the claims -- n_big of `chunk` wave-blocks, then tail claims of
  `chunk_tail` -- cover exactly those wave-blocks;
* every claim counter that holds a claim has a worker workgroup (block b serves
  counter (b - 1) % 8), and the grid never exceeds max_blocks;
* in a launch that spans 2^24-k segments no claim straddles a segment boundary (the
  kernel re-derives the segment words' constants per claim group);
* static first claims (claim w to worker wave w) never outnumber the waves or the claims.

Round 2's parity soak found a launch of a few wave-blocks across a 2^24-k boundary
whose realigned wave-block count left a counter without waves; these cases pin it.
"""
import ctypes
import random

import pytest

import distpow

CLAIM_COUNTERS = 8
WPB = 4  # waves per workgroup


class DiagLaunch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("k_begin", "k_end", "i_begin", "i_end", "wb_begin", "n_wblocks",
                                                "n_big", "n_chunks", "worker_blocks")] + \
               [(n, ctypes.c_uint32) for n in ("chunk", "chunk_tail", "rbits", "wave_block")] + \
               [("n_static", ctypes.c_uint64), ("poll_wb", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


def geometry(nonce, wb, wbits, k0, k1, cus, share=1, ntz=32):
    """The launches dpow_search(nonce, ntz, wb, wbits, k0, k1) queues on a device of `cus`
    CUs shared by `share` searches, sized by the search's own function (size_search_launch)."""
    L = distpow.lib()
    fn = L.dpow_diag_launch_geometry
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                   ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(DiagLaunch),
                   ctypes.c_size_t]
    n = bytes(nonce)
    cnt = fn(n, len(n), ntz, wb, wbits, k0, k1, cus, share, None, 0)
    assert cnt >= 0, distpow._lib.last_error()
    arr = (DiagLaunch * max(cnt, 1))()
    assert fn(n, len(n), ntz, wb, wbits, k0, k1, cus, share, arr, cnt) == cnt
    return list(arr[:cnt])


SHARE_MAX = 2  # plan.h kShareMax: a grid is at most 1/2 of the device's however many searches share it
EST_RATE = 2.3e11  # plan.h kEstRate
SHARE_LAUNCH_NS = 8_000_000  # plan.h kShareLaunchNs


def grid_cap(cus, share=1):
    """The most worker workgroups a launch can get: the full 6-per-CU grid's share (searches in
    flight, capped at SHARE_MAX), at least one per claim counter."""
    return max(cus * 6 // min(share, SHARE_MAX), CLAIM_COUNTERS)


def check(d, max_blocks):
    W = d.wave_block
    assert d.wb_begin % W == 0 and d.wb_begin <= d.i_begin < d.i_end
    assert d.wb_begin + d.n_wblocks * W >= d.i_end > d.wb_begin + (d.n_wblocks - 1) * W
    tails = d.n_chunks - d.n_big
    covered = d.n_big * d.chunk + tails * d.chunk_tail
    assert covered >= d.n_wblocks > covered - d.chunk_tail  # the last (tail) claim is the only partial one
    holders = min(d.n_chunks, CLAIM_COUNTERS)
    assert holders <= d.worker_blocks <= max(max_blocks, CLAIM_COUNTERS)
    # static first claims (the chunk-length-0 template launches below k = 2^24): claim w goes
    # to worker wave w, so there are at most as many as waves, and the counters hand out the
    # rest -- every counter holding one of those still has a workgroup (holders above)
    assert d.n_static <= min(d.n_chunks, d.worker_blocks * WPB)
    if d.k_begin >= (1 << 24):
        assert d.n_static == 0
    # no more workgroups than the claims need (one wave per claim, rounded up to a workgroup)
    assert d.worker_blocks <= max(-(-d.n_chunks // WPB), holders)
    # a launch spanning chunk lengths 1..3 (plan.cpp lspan): no claim straddles k = 256 or
    # 65536 (the kernel takes a claim group's chunk length from its first index >= i_begin)
    def clen(k):
        return (k > 0) + (k > 0xFF) + (k > 0xFFFF)
    if d.k_begin < (1 << 24) and clen(d.k_begin) != clen(d.k_end - 1):
        assert d.k_begin >= 1 and d.rbits >= 1
        assert d.chunk & (d.chunk - 1) == 0 and d.chunk % d.chunk_tail == 0 and d.chunk <= 2 << d.rbits
        assert d.wb_begin % (d.chunk * W) == 0
        for b in (256 << d.rbits, 65536 << d.rbits):  # local index of the boundary
            if not d.i_begin < b < d.i_end:
                continue
            wbb = (b - d.wb_begin) // W  # its wave-block, which must start a claim
            assert (b - d.wb_begin) % W == 0
            big = d.n_big * d.chunk
            assert (wbb % d.chunk == 0) if wbb < big else ((wbb - big) % d.chunk_tail == 0), \
                (d.k_begin, d.k_end, d.rbits, b)
    seg_i = 1 << (24 + d.rbits)  # local indices per 2^24-k segment
    if d.k_begin >> 24 != (d.k_end - 1) >> 24:
        assert d.chunk & (d.chunk - 1) == 0 and d.chunk % d.chunk_tail == 0
        assert d.wb_begin % (d.chunk * W) == 0  # claim starts fall on multiples of the claim size
        starts = [(c * d.chunk, d.chunk) for c in range(min(d.n_big, 4000))]
        starts += [(d.n_big * d.chunk + t * d.chunk_tail, d.chunk_tail) for t in range(min(tails, 4000))]
        for s, sz in starts:
            lo = d.wb_begin + s * W
            hi = d.wb_begin + (s + sz) * W - 1
            assert lo // seg_i == hi // seg_i, (d.k_begin, d.k_end, s, sz)


@pytest.mark.parametrize("cus", [1, 32, 256])
def test_boundary_straddling_windows(cus):
    max_blocks = grid_cap(cus)
    rnd = random.Random(cus)
    for _ in range(400):
        wbits = rnd.choice([0, 1, 2, 3, 5, 8, 9, 10])
        wb = rnd.randrange(1 << (wbits % 9)) if wbits % 9 else 0
        m = rnd.randrange(1, 300)
        u = rnd.random()
        if u < 0.4:
            m += 256  # k >= 2^32 too (L = 5)
        elif u < 0.6:
            m += rnd.choice([1 << 16, 1 << 24, rnd.randrange(1 << 16, 1 << 31)])  # L = 6 / 7
        edge = m << 24
        k0 = max(1 << 24, edge - rnd.randrange(1, 3000))
        k1 = min(distpow.DPOW_K_LIMIT, edge + rnd.randrange(1, 3000))
        nonce = [rnd.randrange(256) for _ in range(rnd.choice([0, 3, 4, 7, 55, 60, 64]))]
        for d in geometry(nonce, wb, wbits, k0, k1, cus, ntz=rnd.choice([32, 7, 8, 9])):
            check(d, max_blocks)


def test_large_and_small_windows():
    rnd = random.Random(3)
    for _ in range(300):
        wbits = rnd.choice([0, 3, 8])
        wb = rnd.randrange(1 << wbits) if wbits else 0
        k0 = rnd.choice([0, 1, 255, 70000, (1 << 24) - 1, 1 << 24, rnd.randrange(1 << 32), (1 << 32) + 5,
                         rnd.randrange(1 << 40, 1 << 48), rnd.randrange(1 << 48, distpow.DPOW_K_LIMIT)])
        k1 = min(distpow.DPOW_K_LIMIT, k0 + rnd.choice([1, 2, 7, 64, 5000, 1 << 20, 1 << 26, 1 << 31]))
        ntz = rnd.choice([32, 3, 5, 6, 7, 8, 9])
        for cus, share in ((1, 1), (16, 1), (256, 8), (256, 2), (256, 1)):  # shares, the 2 / 3 / 4 / 6-per-CU grids
            for nonce in ([1, 2, 3, 4], [1, 2]):  # SH 0; SH 2 (word W0+2 splits at L = 6)
                ds = geometry(nonce, wb, wbits, k0, k1, cus, share, ntz)
                assert (not ds and k1 == 1) or ds[-1].k_end == k1
                assert all(a.k_end == b.k_begin for a, b in zip(ds, ds[1:]))
                for d in ds if len(ds) <= 64 else ds[:32] + ds[-32:]:  # a shared device's ~8 ms launches
                    check(d, grid_cap(cus, share))


def lspan_end(ntz, rbits):
    """plan.cpp lspan_end: chunk lengths 1..3 share a launch (up to k = 2^24) when the first
    hit is expected within 2^28 candidates of the partition, else only lengths 1..2."""
    expect = ((16 ** ntz) << rbits) >> 8 if ntz < 14 else None
    return 1 << 24 if expect is not None and expect <= 1 << 28 else 1 << 16


@pytest.mark.parametrize("ntz", [3, 4, 5, 6, 7, 8, 9, 32])
def test_chunk_length_spanning_launches(ntz):
    """Windows across k = 1, 256 and 65536 for SH = 0 nonces, at every N a short search runs
    with (the grids, chunks and static first claims of short searches): one md5
    launch spans the chunk lengths (after the start kernel's k = 0) up to lspan_end, and its
    claims respect the boundaries."""
    rnd = random.Random(7 + ntz)
    for _ in range(150):
        wbits = rnd.choice([0, 1, 2, 3, 5, 7])
        wb = rnd.randrange(1 << wbits) if wbits else 0
        k0 = rnd.choice([0, 1, 2, 200, 255, 256, 300, 65000, 65535])
        k1 = min(1 << 24, k0 + rnd.choice([2, 60, 300, 5000, 70000, 1 << 20, 1 << 24]))
        nonce = [rnd.randrange(256) for _ in range(rnd.choice([0, 4, 8, 44, 48, 60, 64]))]
        cus, share = rnd.choice([(1, 1), (128, 1), (256, 1), (256, 8)])
        ds = geometry(nonce, wb, wbits, k0, k1, cus, share, ntz)
        le = lspan_end(ntz, 8 - wbits)
        assert ds[0].k_begin == max(k0, 1) and ds[-1].k_end == k1
        assert all(a.k_end == b.k_begin for a, b in zip(ds, ds[1:]))
        if share > 1:  # a shared device: launches of at most ~8 ms at 1/share of the rate
            for d in ds:
                check(d, grid_cap(cus, share))
            continue
        if k1 <= le or max(k0, 1) >= le:
            assert len(ds) == 1, (len(nonce), k0, k1, [(d.k_begin, d.k_end) for d in ds])
        else:
            assert len(ds) == 2 and ds[0].k_end == le
        for d in ds:
            check(d, grid_cap(cus, share))
            assert d.poll_wb in (1, 2, 4, 8, 16)


def test_bench_step_is_one_launch():
    """The bench step (2^28 k from 2^24 at workerBits 0) and an 8-GPU rank's step (2^31 k at
    workerBits 3) are one launch each: launches span the 2^24-k segments."""
    for wb, wbits, nk in ((0, 0, 1 << 28), (5, 3, 1 << 31)):
        ds = geometry([1, 2, 3, 4], wb, wbits, 1 << 24, (1 << 24) + nk, 256)
        assert len(ds) == 1 and ds[0].chunk == 32 and ds[0].worker_blocks == 1536 and ds[0].poll_wb == 16
        check(ds[0], 1536)


def test_short_search_grids():
    """The grids dpow_search gives short searches (the geometry diagnostic runs the search's
    own sizing): an 8-GPU rank's N = 6 window gets 2 workgroups per CU, claims of 2
    wave-blocks, a poll after every wave-block and static first claims; one GPU's N = 7 5
    workgroups per CU with 8-wave-block poll groups, its N = 6 4 workgroups per CU with
    4-wave-block claims and 2-wave-block poll groups, an 8-GPU rank's N = 7 4 per CU with
    claims of 8 and poll groups of 4."""
    # [1,2,3,4]/6 on a workerBits-3 rank (R = 32): 16^6 * 32 / 256 = 2^21 expected candidates
    d, = geometry([1, 2, 3, 4], 5, 3, 1, 1 << 24, 256, ntz=6)
    assert d.worker_blocks <= 2 * 256 and d.chunk_tail <= 2 and d.poll_wb == 1 and d.n_static > 0
    check(d, grid_cap(256))
    # [1,2,3,4]/7 at one GPU: 2^28 expected candidates, past kMidExpect (2^26) and within
    # kFiveExpect (2^31): 5 per CU; below kFastPollCands (2^30): poll groups of 8
    d, = geometry([1, 2, 3, 4], 0, 0, 1, 1 << 20, 256, ntz=7)
    assert d.worker_blocks == 1280 and d.poll_wb == 8
    check(d, grid_cap(256))
    d, = geometry([1, 2, 3, 4], 0, 0, 1, 1 << 20, 256, ntz=6)  # 2^24 expected: 4 per CU, claims of 4, polls of 2
    assert d.worker_blocks == 1024 and d.poll_wb == 2 and d.chunk == 4
    check(d, grid_cap(256))
    # an 8-GPU rank's [1,2,3,4]/7 (2^25 expected): the same mid tier
    d, = geometry([1, 2, 3, 4], 6, 3, 1, 1 << 24, 256, ntz=7)
    assert d.worker_blocks == 1024 and d.poll_wb == 4 and d.chunk == 8
    check(d, grid_cap(256))


def test_grid_policy_for_short_launches():
    """dpow_search's workgroups per CU (plan.cpp launch_blocks_per_cu): the full persistent
    grid for long launches with no early hit expected (the sweep), smaller grids for short
    launches or an expected early hit (16^N R / 256 candidates of this partition), 5 when the
    hit is expected within 2^31."""
    from distpow._lib import lib
    f = lib().dpow_diag_blocks_per_cu
    assert f(1 << 36, 32, 0) == 6 and f(1 << 36, 32, 3) == 6       # the bench sweep, 1 and 8 GPUs
    assert f(1 << 22, 32, 0) == 3 and f(1 << 26, 32, 0) == 4 and f((1 << 26) + 1, 32, 0) == 6
    assert f(1 << 21, 32, 0) == 2 and f((1 << 21) + 1, 32, 0) == 3  # tiny launches (plan.h kTinyExpect)
    assert f(1 << 32, 6, 0) == 4 and f(1 << 32, 5, 0) == 2 and f(1 << 32, 7, 0) == 5  # 16^N expected
    assert f(1 << 32, 6, 3) == 2        # 16^6 * 32 / 256 = 2^21 candidates of a workerBits-3 partition
    assert f(1 << 32, 6, 1) == 2 and f(1 << 32, 6, 2) == 2  # 2^23 / 2^22 expected: tiny since round 5
    assert f(1 << 22, 32, 0) == 3 and f(1 << 23, 32, 0) == 4  # a short window expected late: by its size
    assert f(1 << 32, 7, 3) == 4 and f(1 << 32, 7, 2) == 4 and f(1 << 32, 7, 1) == 5  # 2^25 / 2^26 / 2^27
    # 5 per CU while a hit is expected within 2^31 candidates (plan.h kFiveExpect): an 8-GPU rank's
    # N = 8 (2^29); one GPU's N = 8 (2^32) and an 8-GPU rank's N = 9 (2^33) keep the full grid
    assert f(1 << 32, 8, 3) == 5 and f(1 << 32, 8, 0) == 6 and f(1 << 36, 9, 3) == 6
    assert f(1 << 32, 0, 0) == 2 and f(0, 32, 0) == 2
    for n in range(0, 40, 3):  # never more than the full grid, monotone in the launch size
        seq = [f(1 << n, z, 0) for z in range(0, 34)]
        assert all(2 <= b <= 6 for b in seq) and seq == sorted(seq)


def test_shared_device_launches():
    """Searches sharing a device (dpow_search's g_active; plan.h grid_share, cap_shared_launch):
    launches of about kShareLaunchNs at 1/active of the device's rate, tiling the window, each
    grid 1/min(active, 2) of the device's, and the workgroups per CU chosen on the launch's
    device time (BASELINE config 4: 8 workers on one GPU at N = 8, 2^29 candidates expected
    each, keep the full 6-per-CU grid; alone, an 8-GPU rank's N = 8 gets 5)."""
    nonce = [1, 2, 3, 4]
    for active in (2, 4, 8):
        for wbits, ntz, k0, k1 in ((3, 8, 1 << 16, 1 << 24), (2, 7, 1 << 16, 1 << 24), (0, 32, 1 << 24, 1 << 30),
                                    (3, 32, 1 << 24, (1 << 24) + (1 << 27))):
            ds = geometry(nonce, 5 % (1 << wbits), wbits, k0, k1, 256, active, ntz)
            rbits = 8 - wbits
            cap_k = max(1, int(EST_RATE / active * SHARE_LAUNCH_NS * 1e-9) >> rbits)
            assert ds[0].k_begin == k0 and ds[-1].k_end == k1
            assert all(a.k_end == b.k_begin for a, b in zip(ds, ds[1:]))
            assert all(d.k_end - d.k_begin <= cap_k for d in ds)
            assert len(ds) == -(-(k1 - k0) // cap_k) or k0 < (1 << 24) < k1
            for d in ds:
                check(d, grid_cap(256, active))
            if ntz == 32 or (wbits, ntz) == (3, 8):  # 2^29 x active > 2^31 (plan.h kFiveExpect): the full grid
                bpc = 6 if ntz == 32 or active > 4 else 5
                assert all(d.worker_blocks == 256 * bpc // min(active, SHARE_MAX) for d in ds), \
                    [d.worker_blocks for d in ds]
    # alone: one launch per segment, the tiers of the search's own expected first hit
    d, = geometry(nonce, 5, 3, 1 << 16, 1 << 24, 256, 1, 8)
    assert d.worker_blocks == 256 * 5
    d, = geometry(nonce, 5, 3, 1 << 16, 1 << 24, 256, 8, 32)[:1]
    assert d.worker_blocks == 256 * 6 // SHARE_MAX
    # the tiers judge device time: 4 workers at N = 7 (2^26 expected each, 2^28 of device time)
    assert {d.worker_blocks for d in geometry(nonce, 1, 2, 1 << 16, 1 << 24, 256, 4, 7)} == {256 * 5 // 2}
    assert {d.worker_blocks for d in geometry(nonce, 1, 2, 1 << 16, 1 << 24, 256, 1, 7)} == {256 * 4}
