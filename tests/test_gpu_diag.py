"""The timeline diagnostics on the GPU (include/dpow_diag.h, round 5): dpow_diag_clock_sync pairs
the device's s_memrealtime with the host's CLOCK_MONOTONIC, dpow_diag_search_launches lists the
last search's launches (tools/search_timeline.py reads both).  Structural checks only: the
k = 0 kernel first for a window from k = 0, every consumed record seen after it was queued,
each record's device interval mapped inside the search's host interval (the offset is late by
the stamp's write latency, ~1 us), the hit in the launch that consumed it."""
import ctypes
import time

import pytest
import torch

import distpow
from distpow._lib import LaunchTime

pytestmark = pytest.mark.gpu


def test_search_launches_on_the_host_clock(miner):
    lib = distpow.lib()
    off = ctypes.c_int64()
    t0 = ctypes.c_int64()
    buf = (LaunchTime * 32)()
    for nonce, ntz, g in (([5, 6, 7, 8], 5, 259156), ([1, 2, 3, 4], 3, 97), ([1, 2, 3, 4], 6, 2532284)):
        assert lib.dpow_diag_clock_sync(miner._ctx, 8, ctypes.byref(off)) == 0
        t_call = time.perf_counter_ns()
        r = miner.search(nonce, ntz, 0, 0, 0, 1 << 24)
        t_ret = time.perf_counter_ns()
        assert r.status == distpow.FOUND and r.global_idx == g
        torch.cuda.synchronize()  # records of launches left in flight are written
        n = lib.dpow_diag_search_launches(miner._ctx, ctypes.byref(t0), buf, 32)
        assert 2 <= n <= 32, n
        assert t_call <= t0.value <= t_ret
        ls = buf[:n]
        assert ls[0].kind == 0 and all(x.kind == 1 for x in ls[1:])  # the k = 0 kernel, then md5 launches
        assert [x.seq for x in ls] == list(range(ls[0].seq, ls[0].seq + n))
        for x in ls:
            assert t0.value <= x.queued_ns <= t_ret
            if x.seen_ns >= 0:
                assert x.queued_ns <= x.seen_ns <= t_ret
                assert x.recorded == 1 and 0 < x.t_start_tick <= x.t_end_tick
                start = x.t_start_tick * 10 + off.value
                end = x.t_end_tick * 10 + off.value
                # on the host clock: after it was queued (less the write latency's slack), before it was seen
                assert x.queued_ns - 20_000 <= start <= end <= x.seen_ns + 20_000, (nonce, ntz, x.seq)
        seen = [x for x in ls if x.seen_ns >= 0]
        assert seen and seen[-1].best == g  # the search ended at the record holding its hit
    # bad arguments are errors
    assert lib.dpow_diag_clock_sync(miner._ctx, 0, ctypes.byref(off)) == -1
