"""In-process mirror of the reference coordinator (coordinator.go) over native GPU workers.

The reference coordinator talks net/rpc to W worker processes; here the same
protocol drives W native workers (dpow_worker, one per logical worker) placed
round-robin on the node's GPUs, so the coordinator's workerBits fan-out
(coordinator.go:122-129, 179-199, 326) lands on GPU partitions:

  CoordRPCHandler.Mine   coordinator.go:139-298  -> Coordinator.mine
  CoordRPCHandler.Result coordinator.go:302-320  -> Coordinator._result (fed by one forwarder per
                                                   worker, as cmd/worker/main.go:27-36 does)
  CoordinatorResultCache coordinator.go:391-473  -> Coordinator._cache_get / _cache_add

Protocol kept: cache check; Mine fan-out; the first result wins (it must carry a
secret); Found fan-out; wait for 2W messages in total; one extra Found round (W
cache ACKs) per additional result; reply with the first result's secret.

Node mode (the default for W a power of two in [2, 64]): the W workers share one node board
(distpow.worker.Board, include/dpow.h dpow_board_*), so each task runs as one node search over
the W partitions and only the owner of its minimum index reports it.  The first result is then
the deterministic answer -- the reference enumeration's workerBits = 0 first hit -- instead of
whichever worker happened to finish first; the messages are the reference's (2 per worker).
The coordinator code below is the same in both modes: the change is entirely on the workers'
side, as on a real node where each worker process opens the same board.  W = 1 and non-power-
of-two W (coordinator.go:326 leaves overlapping partitions) keep first-arrived.
Trace actions carry the reference's type names (CoordinatorMine,
CoordinatorWorkerMine, CoordinatorWorkerResult, CoordinatorWorkerCancel,
CoordinatorSuccess, CacheHit/Miss/Add/Remove).
"""
import math
import queue
import threading
import time
from typing import Dict, List, Optional, Sequence

from .worker import Board, Worker

__all__ = ["Coordinator", "CoordinatorProtocolError"]


class CoordinatorProtocolError(RuntimeError):
    """What the reference log.Fatal's on (coordinator.go:205)."""


def _task_key(nonce: bytes, ntz: int) -> str:  # coordinator.go:475-477
    return f"{nonce.hex()}|{ntz}"


def _bytes_greater(a: bytes, b: bytes) -> bool:  # bytes.Compare(a, b) > 0
    return a > b


class Coordinator:
    def __init__(self, n_workers: int, devices: Sequence[int] = (0,), timeout_s: float = 600.0,
                 node: Optional[bool] = None, workers: Optional[Sequence] = None):
        """workers: the W workers to drive instead of in-process ones -- anything with the Worker
        methods, e.g. distpow.procworker.ProcessWorker (one worker process each, which opens the
        node's named board itself); the coordinator then owns their lifetime but no board."""
        if workers is not None:
            n_workers = len(workers)
        if n_workers < 1:
            raise ValueError("need at least one worker")
        pow2 = 2 <= n_workers <= 64 and n_workers & (n_workers - 1) == 0
        if node and not pow2:
            raise ValueError("node mode needs W a power of two in [2, 64] (coordinator.go:326 partitions)")
        self.board: Optional[Board] = None
        if workers is not None:
            self.workers = list(workers)
        else:
            self.workers: List[Worker] = [Worker(devices[i % len(devices)]) for i in range(n_workers)]
            self.board = Board() if (pow2 if node is None else node) else None
            if self.board is not None:
                for w in self.workers:
                    w.set_board(self.board)
        self.worker_bytes = [i & 0xFF for i in range(n_workers)]  # workerByte = uint8(i), coordinator.go:127
        self.worker_bits = int(math.log2(n_workers))              # uint(math.Log2(float64(W))), coordinator.go:326
        self.timeout_s = timeout_s
        self._tasks: Dict[str, queue.Queue] = {}
        self._tasks_mu = threading.Lock()
        self._cache: Dict[bytes, tuple] = {}
        self._cache_mu = threading.Lock()
        self._trace: List[dict] = []
        self._trace_mu = threading.Lock()
        self._token = 0
        self._stop = False
        self._fwd = [threading.Thread(target=self._forward, args=(w,), daemon=True) for w in self.workers]
        for t in self._fwd:
            t.start()

    # -- tracing ---------------------------------------------------------------------
    def _record(self, token, action, **fields):
        with self._trace_mu:
            self._trace.append(dict(trace=token, action=action, **fields))

    def trace(self) -> List[dict]:
        with self._trace_mu:
            return list(self._trace)

    # -- cache (coordinator.go:391-473) -------------------------------------------------
    def _cache_get(self, nonce: bytes, ntz: int, token) -> Optional[bytes]:
        with self._cache_mu:
            e = self._cache.get(nonce)
            if e is not None and e[0] >= ntz:
                self._record(token, "CacheHit", Nonce=list(nonce), NumTrailingZeros=ntz, Secret=list(e[1]))
                return e[1]
            self._record(token, "CacheMiss", Nonce=list(nonce), NumTrailingZeros=ntz)
            return None

    def _cache_add(self, nonce: bytes, ntz: int, secret: bytes, token):
        with self._cache_mu:
            e = self._cache.get(nonce)
            if e is None:
                self._cache[nonce] = (ntz, secret)
                self._record(token, "CacheAdd", Nonce=list(nonce), NumTrailingZeros=ntz, Secret=list(secret))
            elif ntz > e[0] or (ntz == e[0] and _bytes_greater(secret, e[1])):
                self._record(token, "CacheRemove", Nonce=list(nonce), NumTrailingZeros=e[0], Secret=list(e[1]))
                self._record(token, "CacheAdd", Nonce=list(nonce), NumTrailingZeros=ntz, Secret=list(secret))
                self._cache[nonce] = (ntz, secret)

    def cache_entry(self, nonce) -> Optional[tuple]:
        with self._cache_mu:
            return self._cache.get(bytes(nonce))

    # -- CoordRPCHandler.Result (coordinator.go:302-320) ----------------------------------
    def _forward(self, w: Worker):
        while not self._stop:
            r = w.next_result(timeout_ms=100)
            if r is not None:
                self._result(r)

    def _result(self, r):
        if r.error:
            self._record(r.token, "CoordinatorWorkerError", Nonce=list(r.nonce), NumTrailingZeros=r.num_trailing_zeros,
                         WorkerByte=r.worker_byte, Code=r.error)
        if r.secret is not None:
            self._record(r.token, "CoordinatorWorkerResult", Nonce=list(r.nonce), NumTrailingZeros=r.num_trailing_zeros,
                         WorkerByte=r.worker_byte, Secret=list(r.secret))
            self._cache_add(r.nonce, r.num_trailing_zeros, r.secret, r.token)
        with self._tasks_mu:
            q = self._tasks.get(_task_key(r.nonce, r.num_trailing_zeros))
        if q is None:  # the reference sends on a nil channel here and blocks forever (coordinator.go:318)
            self._record(r.token, "CoordinatorDroppedResult", Nonce=list(r.nonce), NumTrailingZeros=r.num_trailing_zeros,
                         WorkerByte=r.worker_byte)
            return
        q.put(r)

    def _get(self, q, ack_phase: bool = False):
        try:
            r = q.get(timeout=self.timeout_s)
        except queue.Empty:
            raise CoordinatorProtocolError("timed out waiting for worker messages")
        if r.error and ack_phase:
            # The request already holds a verified secret: another worker's failed search
            # is that worker's final message (recorded by _result), not a reason to fail it.
            return r
        if r.error:
            # A failed GPU search (no counterpart in the Go reference, whose miner cannot
            # fail): surface it now rather than after timeout_s of waiting for ACKs.
            raise CoordinatorProtocolError(
                f"worker {r.worker_byte} search failed with code {r.error} "
                f"(nonce {r.nonce.hex()}, {r.num_trailing_zeros} zeros)")
        return r

    # -- CoordRPCHandler.Mine (coordinator.go:139-298) ---------------------------------------
    def mine(self, nonce, num_trailing_zeros: int, token: Optional[int] = None) -> bytes:
        nonce = bytes(nonce)
        ntz = num_trailing_zeros
        with self._tasks_mu:
            self._token += 1
            tok = self._token if token is None else token
        self._record(tok, "CoordinatorMine", Nonce=list(nonce), NumTrailingZeros=ntz)
        cached = self._cache_get(nonce, ntz, tok)
        if cached is not None:
            self._record(tok, "CoordinatorSuccess", Nonce=list(nonce), NumTrailingZeros=ntz, Secret=list(cached))
            return cached
        W = len(self.workers)
        q: queue.Queue = queue.Queue(maxsize=2 * W)
        key = _task_key(nonce, ntz)
        with self._tasks_mu:
            self._tasks[key] = q
        for w, wb in zip(self.workers, self.worker_bytes):
            self._record(tok, "CoordinatorWorkerMine", Nonce=list(nonce), NumTrailingZeros=ntz, WorkerByte=wb)
            w.mine(nonce, ntz, wb, self.worker_bits, tok)
        try:
            result = self._get(q)
        except CoordinatorProtocolError:
            self._abort(key, nonce, ntz)
            raise
        if result.secret is None:
            self._abort(key, nonce, ntz)
            raise CoordinatorProtocolError(
                f"First worker result appears to be cancellation ACK, from workerByte = {result.worker_byte}")
        for w, wb in zip(self.workers, self.worker_bytes):
            self._record(tok, "CoordinatorWorkerCancel", Nonce=list(nonce), NumTrailingZeros=ntz, WorkerByte=wb)
            w.found(nonce, ntz, wb, result.secret, tok)
        try:
            received = 1
            extra = []
            while received < 2 * W:
                ack = self._get(q, ack_phase=True)
                if ack.secret is not None:
                    extra.append(ack)
                received += 1
            for ack in extra:
                for w, wb in zip(self.workers, self.worker_bytes):
                    self._record(tok, "CoordinatorWorkerCancel", Nonce=list(nonce), NumTrailingZeros=ntz, WorkerByte=wb)
                    w.found(nonce, ntz, wb, ack.secret, tok)
                for _ in range(W):
                    self._get(q, ack_phase=True)
        finally:
            with self._tasks_mu:
                self._tasks.pop(key, None)
        self._record(tok, "CoordinatorSuccess", Nonce=list(nonce), NumTrailingZeros=ntz, Secret=list(result.secret))
        return result.secret

    def _abort(self, key, nonce, ntz):
        """A failed request: drop the task and stop the other workers' miners (their
        ACKs are then dropped results).  The reference log.Fatal's instead."""
        with self._tasks_mu:
            self._tasks.pop(key, None)
        for w, wb in zip(self.workers, self.worker_bytes):
            try:
                w.cancel(nonce, ntz, wb)
            except Exception:  # the failed worker's task is gone already
                pass

    def close(self):
        self._stop = True
        for t in self._fwd:
            t.join(timeout=5)
        for w in self.workers:
            w.close()
        if self.board is not None:  # every miner has returned (Worker.close joins them)
            self.board.close()
            self.board = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
