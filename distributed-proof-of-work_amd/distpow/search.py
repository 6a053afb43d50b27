"""Host-side mirror of the reference worker's search (worker.go:258-401) over libdpow.

`Miner` is one GPU's search engine.  `Miner.mine` reproduces the reference
miner's loop (worker.go:318-400: k = 0, 1, 2, ... until a hit or a kill) as a
sequence of GPU windows; `Miner.search` is one window (the C ABI dpow_search).
Names and argument meaning follow the reference: nonce, num_trailing_zeros
(NumTrailingZeros), worker_byte (WorkerByte), worker_bits (WorkerBits).
"""
import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

from . import _lib
from ._lib import (CANCELLED, DPOW_K_LIMIT, DPOW_MAX_SECRET, DPOW_NO_HIT, EXHAUSTED, FOUND, DpowError,
                   PlanLaunch, Stats, check, lib)

__all__ = ["Miner", "SearchResult", "secret_from_index", "md5", "verify", "trailing_zero_nibbles",
           "thread_bytes", "remainder_bits", "global_index", "plan_window", "plan_candidate",
           "device_count", "DPOW_NO_HIT", "FOUND", "EXHAUSTED", "CANCELLED"]


@dataclass
class SearchResult:
    status: int                   # FOUND / EXHAUSTED / CANCELLED
    global_idx: int = DPOW_NO_HIT  # k * 256 + threadByte of the hit
    secret: Optional[bytes] = None  # threadByte || chunk_k  (WorkerResult.Secret, worker.go:361)

    @property
    def found(self):
        return self.status == FOUND


def _b(x) -> bytes:
    return bytes(x)


def remainder_bits(worker_bits: int) -> int:
    """worker.go:302: remainderBits := 8 - (args.WorkerBits % 9)."""
    return 8 - (worker_bits % 9)


def thread_bytes(worker_byte: int, worker_bits: int) -> List[int]:
    """worker.go:312-316: threadBytes[i] = uint8((WorkerByte << remainderBits) | i)."""
    rb = remainder_bits(worker_bits)
    return [((worker_byte << rb) | i) & 0xFF for i in range(1 << rb)]


def global_index(k: int, thread_byte: int) -> int:
    return k * 256 + thread_byte


def secret_from_index(g: int) -> bytes:
    buf = (ctypes.c_uint8 * DPOW_MAX_SECRET)()
    n = ctypes.c_size_t()
    check(lib().dpow_secret_from_index(g, buf, ctypes.byref(n)), "dpow_secret_from_index")
    return bytes(buf[:n.value])


def md5(msg) -> bytes:
    out = (ctypes.c_uint8 * 16)()
    m = _b(msg)
    lib().dpow_md5(m, len(m), out)
    return bytes(out)


def trailing_zero_nibbles(digest: bytes) -> int:
    assert len(digest) == 16
    return lib().dpow_trailing_zero_nibbles(digest)


def verify(nonce, secret, num_trailing_zeros: int) -> bool:
    n, s = _b(nonce), _b(secret)
    return lib().dpow_verify(n, len(n), s, len(s), num_trailing_zeros) == 1


def plan_window(nonce, worker_byte, worker_bits, k_begin, k_end, num_trailing_zeros: int = 0) -> List[PlanLaunch]:
    """The launches dpow_search would queue for this window (dpow_plan_window)."""
    n = _b(nonce)
    cnt = check(lib().dpow_plan_window(n, len(n), num_trailing_zeros, worker_byte, worker_bits, k_begin, k_end,
                                       None, 0), "dpow_plan_window")
    arr = (PlanLaunch * max(cnt, 1))()
    check(lib().dpow_plan_window(n, len(n), num_trailing_zeros, worker_byte, worker_bits, k_begin, k_end, arr, cnt),
          "dpow_plan_window")
    return list(arr[:cnt])


def plan_candidate(nonce, worker_byte, worker_bits, local_idx):
    """(iv[4], words[16*nblk], nblk) the kernel hashes for one candidate."""
    n = _b(nonce)
    iv = (ctypes.c_uint32 * 4)()
    words = (ctypes.c_uint32 * 32)()
    nblk = ctypes.c_uint32()
    check(lib().dpow_plan_candidate(n, len(n), worker_byte, worker_bits, local_idx, iv, words,
                                    ctypes.byref(nblk)), "dpow_plan_candidate")
    return list(iv), list(words[:16 * nblk.value]), nblk.value


def device_count() -> int:
    return lib().dpow_device_count()


class Miner:
    """One GPU's search context (dpow_ctx): persistent device buffers, a HIP stream
    and the pinned cancel flag that Found/Cancel raise (worker.go:194,209)."""

    # k-window per dpow_search call.  Launches inside a window are queued
    # back-to-back (split where the chunk length changes); a call returns
    # at the first window holding a hit.
    DEFAULT_WINDOW = 1 << 26

    def __init__(self, device: int = 0):
        self._ctx = ctypes.c_void_p()
        check(lib().dpow_open(device, ctypes.byref(self._ctx)), "dpow_open")
        self.device = device
        self._cancel = lib().dpow_cancel_flag(self._ctx)

    def close(self):
        if self._ctx:
            lib().dpow_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- cancellation (killChan) ------------------------------------------------
    def cancel(self):
        """Raise the pinned cancel flag: a running search stops mid-launch."""
        self._cancel[0] = 1

    def clear_cancel(self):
        self._cancel[0] = 0

    def bound(self, global_idx: int):
        """Lower the bound of the search running on this context (from another thread):
        it stops at global_idx and returns EXHAUSTED unless it has a hit below it
        (dpow_search_bound).  No effect when no search runs."""
        check(lib().dpow_search_bound(self._ctx, global_idx), "dpow_search_bound")

    def attach_node(self, slot: Optional[int]):
        """Attach a node slot (NodeBoard.begin(): the address of a dpow_node_slot in the
        node's shared memory) to this context's searches, or detach it (None)
        (dpow_node_attach)."""
        check(lib().dpow_node_attach(self._ctx, slot or None), "dpow_node_attach")

    @property
    def cancelled(self) -> bool:
        return self._cancel[0] != 0

    # -- the hot path -----------------------------------------------------------
    def search(self, nonce: Sequence[int], num_trailing_zeros: int, worker_byte: int = 0,
               worker_bits: int = 0, k_begin: int = 0, k_end: int = 1, bound: int = DPOW_NO_HIT) -> SearchResult:
        n = _b(nonce)
        best = ctypes.c_uint64(bound)
        sec = (ctypes.c_uint8 * DPOW_MAX_SECRET)()
        slen = ctypes.c_size_t()
        r = check(lib().dpow_search(self._ctx, n, len(n), num_trailing_zeros, worker_byte, worker_bits,
                                    k_begin, k_end, ctypes.byref(best), sec, ctypes.byref(slen)), "dpow_search")
        if r == FOUND:
            return SearchResult(FOUND, best.value, bytes(sec[:slen.value]))
        return SearchResult(r)

    def mine(self, nonce: Sequence[int], num_trailing_zeros: int, worker_byte: int = 0, worker_bits: int = 0,
             k_start: int = 0, k_limit: int = DPOW_K_LIMIT, window: int = DEFAULT_WINDOW) -> SearchResult:
        """worker.go:318-400: search k = k_start, k_start + 1, ... until a hit, the
        cancel flag, or k_limit (the reference has no limit; DPOW_K_LIMIT = 2^55 - 1 k)."""
        k = k_start
        while k < k_limit:
            ke = min(k_limit, k + window)
            res = self.search(nonce, num_trailing_zeros, worker_byte, worker_bits, k, ke)
            if res.status != EXHAUSTED:
                return res
            k = ke
        return SearchResult(EXHAUSTED)

    # -- measurement ------------------------------------------------------------
    def stats(self) -> Stats:
        s = Stats()
        check(lib().dpow_get_stats(self._ctx, ctypes.byref(s)), "dpow_get_stats")
        return s

    def reset_stats(self):
        lib().dpow_reset_stats(self._ctx)

    def stream_handle(self) -> int:
        return lib().dpow_stream(self._ctx) or 0

    def geometry(self):
        cus, bpc, tpb = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().dpow_geometry(self._ctx, ctypes.byref(cus), ctypes.byref(bpc), ctypes.byref(tpb)),
              "dpow_geometry")
        return cus.value, bpc.value, tpb.value
