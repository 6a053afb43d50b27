"""distpow -- MI355X-native proof-of-work search (philipjesic/Distributed-Proof-Of-Work hot path).

The worker's brute-force search (worker.go:258-401) runs as a hand-written gfx950
HIP kernel in libdpow.so; this package is the host side above its C ABI.
"""
from ._lib import (CANCELLED, DPOW_K_LIMIT, DPOW_MAX_SECRET, DPOW_NO_HIT, EHIP, EINVAL, EPROTO, ERANGE,
                   EVERIFY, EXHAUSTED, FOUND, LIB_PATH, DpowError, build_id, lib)
from .search import (Miner, SearchResult, device_count, global_index, md5, plan_candidate, plan_window,
                     remainder_bits, secret_from_index, thread_bytes, trailing_zero_nibbles, verify)

__all__ = ["Miner", "SearchResult", "DpowError", "lib", "LIB_PATH", "device_count", "md5", "verify",
           "secret_from_index", "trailing_zero_nibbles", "thread_bytes", "remainder_bits", "global_index",
           "plan_window", "plan_candidate", "DPOW_NO_HIT", "DPOW_K_LIMIT", "DPOW_MAX_SECRET", "FOUND",
           "EXHAUSTED", "CANCELLED", "EINVAL", "EHIP", "EVERIFY", "ERANGE", "EPROTO", "build_id"]
