"""A native worker in a process of its own, driven over pipes: the reference's topology
(cmd/worker/main.go: one worker process per machine, here per GPU, which the coordinator
reaches over net/rpc, coordinator.go:179-230) without the network, which is out of scope.

The child process holds one `distpow.worker.Worker` (the native mirror of worker.go) and, for
node mode, opens the node board by name (dpow_board_open of a POSIX shared-memory object), as
every worker process of a node does with DPOW_NODE_BOARD in INTEGRATION.md's Go binding.  The
parent's `ProcessWorker` has the Worker's methods, so `distpow.coordinator.Coordinator(workers=...)`
drives W worker processes exactly as it drives in-process workers.  Used by the GPU tests of the
cross-process node board (tests/test_coordinator.py).
"""
import multiprocessing as mp
import os
import threading
from typing import Optional

from .worker import WorkerResultWithToken

__all__ = ["ProcessWorker"]


def _child(device: int, board_name: Optional[str], env: dict, cmd_conn, res_conn):
    os.environ.update(env)
    from .worker import Board, Worker
    w = Worker(device)
    board = Board(board_name) if board_name else None
    if board is not None:
        w.set_board(board)
    stop = threading.Event()

    def forward():  # the worker's ResultChannel -> the coordinator (cmd/worker/main.go:27-36)
        while not stop.is_set():
            r = w.next_result(timeout_ms=50)
            if r is not None:
                res_conn.send(("result", r))

    fwd = threading.Thread(target=forward, daemon=True)
    fwd.start()
    try:
        while True:
            op, args = cmd_conn.recv()
            try:
                if op == "mine":
                    out = w.mine(*args)
                elif op == "found":
                    out = w.found(*args)
                elif op == "cancel":
                    out = w.cancel(*args)
                elif op == "trace":
                    out = w.trace()
                elif op == "active_tasks":
                    out = w.active_tasks()
                elif op == "close":
                    break
                else:
                    raise ValueError(f"unknown op {op!r}")
                cmd_conn.send(("ok", out))
            except Exception as e:  # reported to the caller, which re-raises it
                cmd_conn.send(("error", repr(e)))
    finally:
        w.close()  # every miner ends at its kill (dpow_worker_free)
        stop.set()
        fwd.join()
        if board is not None:
            board.close()
        cmd_conn.send(("ok", None))


class ProcessWorker:
    """The Worker interface over a child process (spawned: a fresh HIP runtime).  board_name: the
    node board every worker process of the node opens ("/name"); env: extra environment of the
    child (e.g. DPOW_DIAG_BOARD_SPLIT)."""

    def __init__(self, device: int = 0, board_name: Optional[str] = None, env: Optional[dict] = None):
        ctx = mp.get_context("spawn")
        self._cmd, child_cmd = ctx.Pipe()
        self._res, child_res = ctx.Pipe(duplex=False)
        self._lock = threading.Lock()
        self.device = device
        self._proc = ctx.Process(target=_child, args=(device, board_name, dict(env or {}), child_cmd, child_res),
                                 daemon=True)
        self._proc.start()
        child_cmd.close()
        child_res.close()

    def _call(self, op, *args):
        with self._lock:
            self._cmd.send((op, args))
            status, out = self._cmd.recv()
        if status != "ok":
            raise RuntimeError(f"worker process {self._proc.pid}: {op}: {out}")
        return out

    def mine(self, nonce, num_trailing_zeros, worker_byte, worker_bits, token=0):
        return self._call("mine", bytes(nonce), num_trailing_zeros, worker_byte, worker_bits, token)

    def found(self, nonce, num_trailing_zeros, worker_byte, secret, token=0):
        return self._call("found", bytes(nonce), num_trailing_zeros, worker_byte, bytes(secret), token)

    def cancel(self, nonce, num_trailing_zeros, worker_byte):
        return self._call("cancel", bytes(nonce), num_trailing_zeros, worker_byte)

    def trace(self):
        return self._call("trace")

    def active_tasks(self) -> int:
        return self._call("active_tasks")

    def next_result(self, timeout_ms: int = -1) -> Optional[WorkerResultWithToken]:
        if not self._res.poll(None if timeout_ms < 0 else timeout_ms / 1e3):
            return None
        try:
            kind, r = self._res.recv()
        except EOFError:  # the child has exited
            return None
        return r

    def close(self):
        if self._proc.is_alive():
            try:
                self._call("close")
            except (EOFError, OSError, RuntimeError):
                pass
        self._proc.join(timeout=30)
        if self._proc.is_alive():
            self._proc.kill()
            self._proc.join()
