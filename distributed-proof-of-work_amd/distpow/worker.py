"""Python handle on the native GPU worker (include/dpow_worker.h).

Mirrors the reference worker's RPC surface (worker.go:108-232): Mine, Found,
Cancel, and the ResultChannel drained by cmd/worker/main.go:27-36.  The miner
(worker.go:258-401), its cache (worker.go:424-506) and its trace actions run
natively in libdpow.so; the search loop runs on the GPU.
"""
import ctypes
import json
from dataclasses import dataclass
from typing import List, Optional

from ._lib import ETIMEOUT, DpowError, WorkerResult, check, lib


@dataclass
class WorkerResultWithToken:
    """worker.go:38-44; secret None is the nil-secret cancellation ACK.  error != 0 (a
    negative DPOW_E* code) reports a failed GPU search: the task is over."""
    nonce: bytes
    num_trailing_zeros: int
    worker_byte: int
    secret: Optional[bytes]
    token: int
    error: int = 0


class Board:
    """The node board (include/dpow.h dpow_board_*): the task entries through which the W
    workers of one host run each task's node search, so the coordinator's first result is the
    node's deterministic first hit.  name None: private to this process (the workers of one
    process, e.g. the coordinator mirror); "/name": a POSIX shared-memory object every worker
    process of the host opens."""

    def __init__(self, name: Optional[str] = None):
        self._b = ctypes.c_void_p()
        self.name = name
        check(lib().dpow_board_open(name.encode() if name else None, ctypes.byref(self._b)), "dpow_board_open")

    @property
    def handle(self):
        return self._b

    def tasks(self) -> int:
        """Task entries in use (0 once every rank of every task has left)."""
        return check(lib().dpow_board_tasks(self._b), "dpow_board_tasks")

    def counters(self):
        """(task entries created, of which all ranks shared one GPU) over the board's life."""
        t, sh = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().dpow_board_counters(self._b, ctypes.byref(t), ctypes.byref(sh)), "dpow_board_counters")
        return t.value, sh.value

    def join(self, nonce, num_trailing_zeros, world, rank):
        """(slot, votes) addresses of the task's entry for this rank (dpow_board_join)."""
        n = bytes(nonce)
        slot, votes = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().dpow_board_join(self._b, n, len(n), num_trailing_zeros, world, rank, ctypes.byref(slot),
                                    ctypes.byref(votes)), "dpow_board_join")
        return slot.value, votes.value

    def leave(self, slot):
        check(lib().dpow_board_leave(self._b, slot), "dpow_board_leave")

    def close(self, unlink: bool = False):
        if self._b:
            lib().dpow_board_close(self._b)
            self._b = ctypes.c_void_p()
            if unlink and self.name:
                check(lib().dpow_board_unlink(self.name.encode()), "dpow_board_unlink")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Worker:
    def __init__(self, device: int = 0):
        self._w = ctypes.c_void_p()
        check(lib().dpow_worker_new(device, ctypes.byref(self._w)), "dpow_worker_new")
        self.device = device

    def set_board(self, board: Optional[Board]):
        """Node mode (dpow_worker_set_board): tasks with 1 <= workerBits <= 6 search on the board."""
        check(lib().dpow_worker_set_board(self._w, board.handle if board is not None else None),
              "dpow_worker_set_board")

    def close(self):
        if self._w:
            lib().dpow_worker_free(self._w)
            self._w = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- RPCs ------------------------------------------------------------------
    def mine(self, nonce, num_trailing_zeros, worker_byte, worker_bits, token=0):
        n = bytes(nonce)
        check(lib().dpow_worker_mine(self._w, n, len(n), num_trailing_zeros, worker_byte, worker_bits, token),
              "WorkerRPCHandler.Mine")

    def found(self, nonce, num_trailing_zeros, worker_byte, secret, token=0):
        n, s = bytes(nonce), bytes(secret)
        check(lib().dpow_worker_found(self._w, n, len(n), num_trailing_zeros, worker_byte, s, len(s), token),
              "WorkerRPCHandler.Found")

    def cancel(self, nonce, num_trailing_zeros, worker_byte):
        n = bytes(nonce)
        return check(lib().dpow_worker_cancel(self._w, n, len(n), num_trailing_zeros, worker_byte),
                     "WorkerRPCHandler.Cancel")

    # -- ResultChannel -----------------------------------------------------------
    def next_result(self, timeout_ms: int = -1) -> Optional[WorkerResultWithToken]:
        r = WorkerResult()
        code = lib().dpow_worker_next_result(self._w, ctypes.byref(r), timeout_ms)
        if code == ETIMEOUT:
            return None
        check(code, "dpow_worker_next_result")
        return WorkerResultWithToken(bytes(r.nonce[:r.nonce_len]), r.num_trailing_zeros, r.worker_byte,
                                     bytes(r.secret[:r.secret_len]) if r.has_secret else None, r.token,
                                     r.error)

    # -- introspection -------------------------------------------------------------
    def trace(self) -> List[dict]:
        n = lib().dpow_worker_trace(self._w, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        lib().dpow_worker_trace(self._w, buf, n + 1)
        return [json.loads(l) for l in buf.value.decode().splitlines() if l]

    def active_tasks(self) -> int:
        return lib().dpow_worker_active_tasks(self._w)


__all__ = ["Board", "Worker", "WorkerResultWithToken", "DpowError"]
