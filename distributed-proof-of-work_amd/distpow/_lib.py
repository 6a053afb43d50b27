"""ctypes binding of libdpow.so (include/dpow.h, include/dpow_worker.h).

The product path is the HIP library: there is no CPU fallback.  Loading fails
loudly (ImportError/OSError) when the library is missing; GPU entry points fail
with DpowError when no HIP device is visible.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdpow.so")

DPOW_NO_HIT = 0x7FFFFFFFFFFFFFFF
DPOW_MAX_SECRET = 16
DPOW_K_LIMIT = 1 << 40
EXHAUSTED, FOUND, CANCELLED = 0, 1, 2
EINVAL, EHIP, EVERIFY, ERANGE, ENOMEM = -1, -2, -3, -4, -5


class DpowError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"dpow error {code}: {msg}")
        self.code = code


class PlanLaunch(ctypes.Structure):
    _fields_ = [("k_begin", ctypes.c_uint64), ("k_end", ctypes.c_uint64),
                ("i_begin", ctypes.c_uint64), ("i_end", ctypes.c_uint64),
                ("nblk", ctypes.c_uint32), ("w0", ctypes.c_uint32), ("sh", ctypes.c_uint32),
                ("chunk_len", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("searches", ctypes.c_uint64), ("launches", ctypes.c_uint64),
                ("candidates", ctypes.c_uint64), ("kernel_ms", ctypes.c_double)]


_lib = None


def _preload_torch_hip():
    # torch ships its own libamdhip64 (soname libamdhip64.so.7).  Loading torch
    # first makes libdpow bind to that same runtime instead of a second copy,
    # so torch streams/events/collectives and our kernels share one HIP runtime.
    try:
        import torch  # noqa: F401
    except Exception:  # torch is plumbing only; the library works without it
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libdpow.so not built at {LIB_PATH}; run __graft_entry__.build() "
                          f"(make -C distributed-proof-of-work_amd/csrc)")
    _preload_torch_hip()
    L = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    szp = ctypes.POINTER(ctypes.c_size_t)
    vp = ctypes.c_void_p
    sig = {
        "dpow_open": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
        "dpow_close": (None, [vp]),
        "dpow_cancel_flag": (u32p, [vp]),
        "dpow_search": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, u64p, u8p, szp]),
        "dpow_secret_from_index": (ctypes.c_int, [ctypes.c_uint64, u8p, szp]),
        "dpow_md5": (None, [ctypes.c_char_p, ctypes.c_size_t, u8p]),
        "dpow_trailing_zero_nibbles": (ctypes.c_uint32, [ctypes.c_char_p]),
        "dpow_verify": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.c_uint32]),
        "dpow_plan_window": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(PlanLaunch),
                                            ctypes.c_size_t]),
        "dpow_plan_candidate": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint64, u32p, u32p, u32p]),
        "dpow_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(Stats)]),
        "dpow_reset_stats": (None, [vp]),
        "dpow_stream": (vp, [vp]),
        "dpow_device": (ctypes.c_int, [vp]),
        "dpow_geometry": (ctypes.c_int, [vp, u32p, u32p, u32p]),
        "dpow_last_error": (ctypes.c_char_p, []),
        "dpow_abi_version": (ctypes.c_int, []),
        "dpow_device_count": (ctypes.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    return lib().dpow_last_error().decode(errors="replace")


def check(code, what="dpow"):
    if code < 0:
        raise DpowError(code, f"{what}: {last_error()}")
    return code
