"""ctypes binding of libdpow.so (include/dpow.h, include/dpow_worker.h).

The product path is the HIP library: there is no CPU fallback.  Loading fails
loudly (ImportError/OSError) when the library is missing; GPU entry points fail
with DpowError when no HIP device is visible.
"""
import ctypes
import fcntl
import glob
import hashlib
import os
import re
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include")
# DPOW_LIB_PATH overrides the in-tree library (A/B builds in tools/ab_variants.py only;
# such a library is not checked against the source hash, but its ABI version must be
# this binding's: check_abi).
LIB_OVERRIDE = os.environ.get("DPOW_LIB_PATH")
LIB_PATH = LIB_OVERRIDE or os.path.join(_HERE, "libdpow.so")

DPOW_NO_HIT = 0x7FFFFFFFFFFFFFFF
DPOW_MAX_SECRET = 16
DPOW_K_LIMIT = (1 << 55) - 1  # include/dpow.h: chunks of up to 7 bytes, every index < DPOW_NO_HIT
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
                ("chunk_len", ctypes.c_uint32), ("chunk_len_last", ctypes.c_uint32),
                ("start_kernel", ctypes.c_uint32)]


DPOW_MAX_NONCE = 1024
EPROTO, ETIMEOUT = -6, -7


class LaunchTime(ctypes.Structure):
    """dpow_diag_launch_time (include/dpow_diag.h)."""
    _fields_ = [("seq", ctypes.c_uint64), ("kind", ctypes.c_int32), ("recorded", ctypes.c_int32),
                ("queued_ns", ctypes.c_int64), ("seen_ns", ctypes.c_int64),
                ("t_start_tick", ctypes.c_uint64), ("t_end_tick", ctypes.c_uint64),
                ("candidates", ctypes.c_uint64), ("g_end", ctypes.c_uint64), ("best", ctypes.c_uint64)]


class WorkerResult(ctypes.Structure):
    _fields_ = [("num_trailing_zeros", ctypes.c_uint32), ("worker_byte", ctypes.c_uint32),
                ("has_secret", ctypes.c_uint32), ("secret_len", ctypes.c_uint32), ("error", ctypes.c_int32),
                ("secret", ctypes.c_uint8 * DPOW_MAX_SECRET), ("token", ctypes.c_uint64),
                ("nonce_len", ctypes.c_uint64), ("nonce", ctypes.c_uint8 * DPOW_MAX_NONCE)]


class Stats(ctypes.Structure):
    _fields_ = [("searches", ctypes.c_uint64), ("launches", ctypes.c_uint64),
                ("candidates", ctypes.c_uint64), ("kernel_ms", ctypes.c_double)]


_lib = None


def source_build_id(nc=2, extra=""):
    """The build id the Makefile embeds (dpow_build_id) for the sources in this tree:
    sha256 over csrc/{*.cpp,*.h,*.hip} (sorted), csrc/Makefile, include/*.h (sorted)
    and the default build flags; first 16 hex digits."""
    names = sorted({os.path.basename(p) for pat in ("*.cpp", "*.h", "*.hip")
                    for p in glob.glob(os.path.join(CSRC, pat))})
    files = [os.path.join(CSRC, n) for n in names] + [os.path.join(CSRC, "Makefile")]
    files += [os.path.join(INCLUDE, n) for n in sorted(os.path.basename(p)
                                                       for p in glob.glob(os.path.join(INCLUDE, "*.h")))]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(f"NC={nc} EXTRA={extra}\n".encode())
    return h.hexdigest()[:16]


def library_build_id(path=None):
    """The build id stored in a libdpow.so file (read from the file, without loading it:
    a dlopen'ed stale library could not be replaced in-process)."""
    path = path or LIB_PATH
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(rb"dpow-build-id:([0-9a-f]{16})", f.read())
    return m.group(1).decode() if m else None


def _rebuild():
    """make -C csrc under a lock (several test/bench processes may start at once)."""
    if not (shutil.which("make") and (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc"))):
        return False
    jobs = str(min(16, os.cpu_count() or 8))
    with open(os.path.join(CSRC, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        print(f"distpow: libdpow.so does not match the sources; rebuilding (make -j{jobs})",
              file=sys.stderr, flush=True)
        # output captured (sys.stderr may be a pytest capture object without a file descriptor)
        r = subprocess.run(["make", "-s", "-j", jobs, "-C", CSRC], capture_output=True, text=True)
        if r.returncode != 0:
            raise ImportError(f"rebuilding libdpow.so failed:\n{(r.stdout + r.stderr)[-4000:]}")
    return True


def check_build():
    """Make sure LIB_PATH was built from the sources in this tree: returns its build id.

    A stale library is rebuilt when make/hipcc are available (DPOW_NO_AUTOBUILD=1 turns
    that off) and refused otherwise, so nothing ever tests or benches an old build."""
    want = source_build_id()
    have = library_build_id(LIB_PATH)
    if have == want:
        return have
    if os.environ.get("DPOW_NO_AUTOBUILD") != "1" and _rebuild():
        have = library_build_id(LIB_PATH)
        if have == want:
            return have
    raise ImportError(f"libdpow.so at {LIB_PATH} has build id {have!r}, but the sources in this tree hash to "
                      f"{want!r}: rebuild it (make -C distributed-proof-of-work_amd/csrc)")


def header_abi_version(header=None):
    """DPOW_ABI_VERSION as include/dpow.h of this tree defines it: the ABI this binding's
    argtypes and structs were written for."""
    path = header or os.path.join(INCLUDE, "dpow.h")
    with open(path) as f:
        m = re.search(r"^#define\s+DPOW_ABI_VERSION\s+(\d+)\s*$", f.read(), re.M)
    if not m:
        raise ImportError(f"{path} defines no DPOW_ABI_VERSION")
    return int(m.group(1))


def check_abi(L, path):
    """Refuse a library built for another ABI (include/dpow.h: a consumer built against
    another version must refuse it).  dpow_abi_version() is the only entry point called
    before the check; a library without it is refused too."""
    want = header_abi_version()
    fn = getattr(L, "dpow_abi_version", None)
    if fn is None:
        raise ImportError(f"{path} exports no dpow_abi_version: not a libdpow.so")
    fn.restype = ctypes.c_int
    fn.argtypes = []
    have = fn()
    if have != want:
        raise ImportError(f"{path} implements DPOW_ABI_VERSION {have}, but this binding (include/dpow.h) is "
                          f"version {want}: refusing it (rebuild the library from this tree, or use the binding "
                          f"of the tree it was built from)")
    return have


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
    if LIB_OVERRIDE is None:
        check_build()
    elif not os.path.exists(LIB_PATH):
        raise ImportError(f"DPOW_LIB_PATH={LIB_PATH} does not exist")
    _preload_torch_hip()
    L = ctypes.CDLL(LIB_PATH)
    check_abi(L, LIB_PATH)  # every library, the DPOW_LIB_PATH overrides included
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
        "dpow_search_bound": (ctypes.c_int, [vp, ctypes.c_uint64]),
        "dpow_node_attach": (ctypes.c_int, [vp, vp]),
        "dpow_node_slot_reset": (None, [vp]),
        "dpow_node_release": (ctypes.c_int, [vp, ctypes.c_size_t]),
        "dpow_node_post": (None, [vp, ctypes.c_uint64]),
        "dpow_node_stop": (None, [vp]),
        "dpow_node_vote": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                          ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                          ctypes.c_int64]),
        "dpow_node_mine": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, u64p, ctypes.c_int64,
                                          ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u64p, u8p, szp, u32p]),
        "dpow_board_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(vp)]),
        "dpow_board_close": (None, [vp]),
        "dpow_board_unlink": (ctypes.c_int, [ctypes.c_char_p]),
        "dpow_board_join": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        "dpow_board_leave": (ctypes.c_int, [vp, vp]),
        "dpow_board_tasks": (ctypes.c_int, [vp]),
        "dpow_board_counters": (ctypes.c_int, [vp, u64p, u64p]),
        "dpow_board_search": (ctypes.c_int, [vp, vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint32, u64p, u8p, szp, u32p]),
        "dpow_secret_from_index": (ctypes.c_int, [ctypes.c_uint64, u8p, szp]),
        "dpow_md5": (None, [ctypes.c_char_p, ctypes.c_size_t, u8p]),
        "dpow_trailing_zero_nibbles": (ctypes.c_uint32, [ctypes.c_char_p]),
        "dpow_verify": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.c_uint32]),
        "dpow_plan_window": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
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
        "dpow_build_id": (ctypes.c_char_p, []),
        "dpow_device_count": (ctypes.c_int, []),
        "dpow_diag_valu_rate": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(ctypes.c_double)]),
        "dpow_diag_dword_test": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64,
                                                ctypes.c_uint32, ctypes.c_uint32]),
        "dpow_diag_blocks_per_cu": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]),
        "dpow_diag_search_times": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64)]),
        "dpow_diag_node_post_at": (ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_int64]),
        "dpow_diag_node_alias": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        "dpow_diag_search_launches": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(LaunchTime),
                                                     ctypes.c_size_t]),
        "dpow_diag_clock_sync": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
        "dpow_diag_vote_latency": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                  ctypes.POINTER(ctypes.c_double)]),
        "dpow_worker_new": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
        "dpow_worker_free": (None, [vp]),
        "dpow_worker_mine": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint64]),
        "dpow_worker_found": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]),
        "dpow_worker_cancel": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                              ctypes.c_uint32]),
        "dpow_worker_next_result": (ctypes.c_int, [vp, ctypes.POINTER(WorkerResult), ctypes.c_int]),
        "dpow_worker_trace": (ctypes.c_size_t, [vp, ctypes.c_char_p, ctypes.c_size_t]),
        "dpow_worker_active_tasks": (ctypes.c_int, [vp]),
        "dpow_worker_set_board": (ctypes.c_int, [vp, vp]),
    }
    missing = [name for name in sig if not hasattr(L, name)]
    if missing:  # same ABI version, yet entry points missing: not a library of this ABI either
        raise ImportError(f"{LIB_PATH} lacks entry points of DPOW_ABI_VERSION {header_abi_version()}: {missing}")
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


VALU_KINDS = {0: "v_add_u32", 1: "v_add3_u32", 2: "v_alignbit_b32", 3: "v_bitop3_b32", 4: "v_fma_f32",
              5: "md5_step_mix", 6: "v_lshl_add_u32", 7: "v_lshl_or_b32", 8: "v_xad_u32", 9: "v_perm_b32",
              10: "v_lshlrev_b32", 11: "v_or3_b32", 12: "v_add_u32_literal", 13: "v_alignbyte_b32",
              14: "v_bfi_b32", 15: "v_add_lshl_u32", 16: "v_xor_b32", 17: "v_add3_u32_sgpr", 18: "v_pk_add_u16",
              19: "md5_mix_interleave8", 20: "md5_mix_interleave2", 21: "md5_mix_2add_interleave2",
              22: "md5_mix_alternating2", 23: "md5_mix_sgpr_k",
              24: "md5_chain_compiler", 25: "md5_chain_alternating",
              26: "alt_pairs_banks_distinct", 27: "alt_pairs_banks_same", 28: "v_mad_u32_u24",
              29: "v_dot2_u32_u16", 30: "v_bitop3_b16", 31: "v_lshlrev_b64", 32: "v_lshl_add_u64",
              33: "v_pk_mov_b32",
              34: "v_add_u32_sdwa_word1", 35: "v_add_u16_sdwa_dst_word1",
              36: "md5_pair_rot16_alignbit", 37: "md5_pair_rot16_sdwa"}


def valu_rate(device=0, kind=5):
    """(lane-ops/s, in-kernel clock GHz) of one VALU instruction kind with every CU busy."""
    r, c = ctypes.c_double(), ctypes.c_double()
    code = lib().dpow_diag_valu_rate(device, kind, ctypes.byref(r), ctypes.byref(c))
    if code < 0:
        raise DpowError(code, "dpow_diag_valu_rate failed")
    return r.value, c.value


def build_id():
    """Source hash libdpow.so was built from (dpow_build_id)."""
    return lib().dpow_build_id().decode()


def last_error():
    return lib().dpow_last_error().decode(errors="replace")


def check(code, what="dpow"):
    if code < 0:
        raise DpowError(code, f"{what}: {last_error()}")
    return code
