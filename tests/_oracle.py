"""ctypes loader for the CPU oracle (oracle/build/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

The oracle restates the reference worker's search (worker.go:234-400) in plain C;
it is the checker for parity tests and the CPU baseline in bench.py, never the product.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")


def build_oracle():
    # make is a no-op when the library is current (a stale one would lack new entry points)
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(
            os.path.join(ORACLE_DIR, "dpow_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    return ORACLE_SO


class Oracle:
    def __init__(self):
        self.lib = ctypes.CDLL(build_oracle())
        L = self.lib
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_md5.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u8p]
        L.oracle_md5.restype = None
        L.oracle_next_chunk.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_next_chunk.restype = ctypes.c_size_t
        L.oracle_chunk_of.argtypes = [ctypes.c_uint64, u8p]
        L.oracle_chunk_of.restype = ctypes.c_size_t
        L.oracle_has_num_zeroes_suffix.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint]
        L.oracle_has_num_zeroes_suffix.restype = ctypes.c_int
        L.oracle_thread_bytes.argtypes = [ctypes.c_uint8, ctypes.c_uint, u8p]
        L.oracle_thread_bytes.restype = ctypes.c_uint
        L.oracle_mine_window.argtypes = [
            ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint8, ctypes.c_uint,
            ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t),
            ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_mine_window.restype = ctypes.c_int
        L.oracle_cpu_bench.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint,
                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_cpu_bench.restype = ctypes.c_double
        L.oracle_bench_workers.argtypes = [ctypes.c_uint]
        L.oracle_bench_workers.restype = ctypes.c_uint
        L.oracle_cpu_mine.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_uint,
                                      ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint)]
        L.oracle_cpu_mine.restype = ctypes.c_double

    def md5(self, msg: bytes) -> bytes:
        out = (ctypes.c_uint8 * 16)()
        self.lib.oracle_md5(bytes(msg), len(msg), out)
        return bytes(out)

    def next_chunk(self, chunk):
        buf = (ctypes.c_uint8 * 16)(*chunk)
        n = self.lib.oracle_next_chunk(buf, len(chunk))
        return list(buf[:n])

    def chunk_of(self, k):
        buf = (ctypes.c_uint8 * 16)()
        n = self.lib.oracle_chunk_of(k, buf)
        return list(buf[:n])

    def has_suffix(self, s: str, n: int) -> bool:
        b = s.encode()
        return bool(self.lib.oracle_has_num_zeroes_suffix(b, len(b), n))

    def thread_bytes(self, wb, wbits):
        buf = (ctypes.c_uint8 * 256)()
        n = self.lib.oracle_thread_bytes(wb, wbits, buf)
        return list(buf[:n])

    def mine_window(self, nonce, ntz, wb=0, wbits=0, k_begin=0, k_end=1):
        """-> (secret list, global idx, local idx) or None."""
        sec = ctypes.create_string_buffer(32)
        slen = ctypes.c_size_t()
        g = ctypes.c_uint64()
        loc = ctypes.c_uint64()
        r = self.lib.oracle_mine_window(bytes(nonce), len(nonce), ntz, wb, wbits, k_begin, k_end, sec,
                                        ctypes.byref(slen), ctypes.byref(g), ctypes.byref(loc))
        assert r >= 0
        if r == 0:
            return None
        return list(sec.raw[:slen.value]), g.value, loc.value

    def cpu_mine(self, nonce, ntz, nthreads, k_end):
        """(seconds, min global idx or None, candidates hashed, workers) of the W-worker
        prefix fan-out on host threads (oracle_cpu_mine)."""
        g, h, w = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint()
        secs = self.lib.oracle_cpu_mine(bytes(nonce), len(nonce), ntz, nthreads, k_end, ctypes.byref(g),
                                        ctypes.byref(h), ctypes.byref(w))
        return secs, (None if g.value == (1 << 64) - 1 else g.value), h.value, w.value

    def cpu_bench(self, nonce, ntz, nthreads, k_begin, k_count):
        h = ctypes.c_uint64()
        secs = self.lib.oracle_cpu_bench(bytes(nonce), len(nonce), ntz, nthreads, k_begin, k_count,
                                         ctypes.byref(h))
        return secs, h.value
