"""Multi-GPU search on one node: the coordinator's workerBits prefix fan-out
(coordinator.go:122-129, 179-199, 326) mapped onto G GPUs, one process per GPU.

Rank r of G = 2^b owns the reference worker partition (WorkerByte = r,
WorkerBits = b): threadBytes [r * 2^(8-b), (r+1) * 2^(8-b)) (worker.go:302-316).
All ranks scan the same k-window per batch.  At each batch boundary the ranks take
one MIN of three int64 values, [best global index, running, healthy] (24 bytes): it
picks the globally lowest index and votes on cancellation and on failure.  When every
rank shares one host the MIN goes through the node board's shared memory
(NodeBoard.vote, dpow_node_vote: a few microseconds); across hosts it is one
torch.distributed all-reduce, RCCL over xGMI with the "nccl" backend (bench.py's
per-step reduce of the sweep is RCCL too).  The minimum over partitions of each
partition's first hit is the workerBits = 0 answer, so the result is deterministic and
equals the single-worker enumeration's first hit.

This replaces the reference's first-message-wins gather (coordinator.go:202) by
a deterministic reduction; the owner of the winning index is rank
(threadByte >> (8 - b)), the worker that would have reported WorkerResult.
"""
import math
import threading
import time
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

from ._lib import CANCELLED, DPOW_K_LIMIT, DPOW_NO_HIT, EPROTO, EXHAUSTED, FOUND

__all__ = ["NodeResult", "NodeError", "NodeBoard", "auto_batch_candidates", "node_mine", "node_mine_async",
           "partition_of_rank", "owner_rank", "first_window_k"]


@dataclass
class NodeResult:
    status: int
    global_idx: int = DPOW_NO_HIT
    secret: Optional[bytes] = None
    owner: int = -1      # rank whose partition holds the winning index
    batches: int = 0


def partition_of_rank(rank: int, world: int):
    """(worker_byte, worker_bits) of a rank: coordinator.go:127 workerByte = i,
    coordinator.go:326 workerBits = floor(log2(W))."""
    if world < 1 or world & (world - 1):
        raise ValueError("world size must be a power of two (non-power-of-two W leaves holes/overlaps "
                         "in the reference's prefix partition, coordinator.go:326 / worker.go:315)")
    return rank, int(math.log2(world))


def owner_rank(global_idx: int, world: int) -> int:
    b = int(math.log2(world))
    return (global_idx & 0xFF) >> (8 - b) if b else 0


RANK_RATE = 2.17e11        # candidates/s of one MI355X on the one-block layouts (bench `value`)
# node_mine's fixed cost per batch c: the window's search call (launch, drain,
# completion record) plus the batch boundary (pinned copy in, all-reduce MIN, copy out,
# synchronize).  Measured on an MI355X over a world-1 RCCL group (tests/test_gpu_rccl.py,
# bench.py `collective`): boundary 31-33 us, a whole batch of 2^16 candidates 74-80 us.
BATCH_OVERHEAD_S = 8e-5


def auto_batch_candidates(num_trailing_zeros: int, world: int, rate: float = RANK_RATE,
                          overhead_s: float = BATCH_OVERHEAD_S, lo: int = 1 << 16, hi: int = 1 << 31) -> int:
    """Per-rank batch (candidates) that minimises the node's expected time to its first hit.

    A candidate passes the suffix test (worker.go:246-256) with p = 16^-N: MD5's output
    nibbles are uniform.  So the node's first hit is geometric and the search is
    memoryless: every batch faces the same problem and the best batch is one constant
    size.  With the node's hit rate lam = world * rate * p per second and a fixed cost c
    per batch (every rank hashes its whole batch, then the all-reduce), the expected time
    (c + t) / (1 - exp(-lam t)) ~ (1 / lam)(1 + c / t)(1 + lam t / 2) is smallest at
    t = sqrt(2 c / lam): B = rate * t = sqrt(2 c rate / (world p)).  At 8 GPUs that is
    0.15 M candidates per rank at N = 3, 2.4 M at N = 5, 9.5 M at N = 6, 38 M at N = 7,
    152 M at N = 8 and 610 M at N = 9 (clamped to [2^16, 2^31]).  Growing from 2^8 k instead
    (round 2's first schedule) spends 4-7 batch costs before a batch holds 0.1 ms of
    hashing: more than the search itself at N <= 7.
    """
    p = 16.0 ** -min(max(num_trailing_zeros, 0), 32)
    b = math.sqrt(2.0 * overhead_s * rate / (max(1, world) * p))
    return int(min(hi, max(lo, b)))


class NodeError(RuntimeError):
    """Another rank's search failed: the node's search ends on every rank (the reference
    log.Fatal's on a missing or malformed result, coordinator.go:202-206)."""


class NodeBoard:
    """The node's Found fan-out in shared memory (dpow_node_slot, include/dpow.h).

    The ranks of one node map one small POSIX shared-memory segment of SLOTS 64-byte
    slots.  node_mine uses slot (call index mod SLOTS) for one node search and attaches
    it to the rank's GPU context: a rank's verified hit is posted to the slot at once,
    and every other rank's running search takes it as its bound while it waits for its
    kernels, so the node stops at its lowest hit without waiting for a batch boundary.
    A cancelled or failed rank raises the slot's stop, which ends every rank's search.
    The batch boundary still decides the answer (the minimum over the ranks, the
    workerBits = 0 first hit): on a shared board it is the node vote (dpow_node_vote, a
    MIN over the ranks' entries in the same shared memory: microseconds, where an RCCL
    all-reduce of the 24 bytes plus its host copies costs ~33 us at world 1), else the
    RCCL all-reduce.  The slot of call c + 2 is reset at the end of call c: every rank
    has passed call c + 1's last boundary before any rank uses it, so no reset can race
    a post.

    Created collectively (every rank of `group`); None from create() when the ranks do
    not share one host (then node_mine runs on RCCL batch boundaries alone).
    """
    SLOTS = 4
    SLOT_BYTES = 64
    VOTE_BYTES = 64  # dpow_node_vote_entry; two per rank
    VOTE_TIMEOUT_NS = 120 * 10**9  # a rank that never votes (dead): NodeError after 2 minutes

    def __init__(self, shm=None, world: int = 0, rank: int = 0):
        import ctypes
        self._shm = shm  # an mmap.mmap of the node's /dev/shm segment (create())
        self.world, self.rank = world, rank
        if shm is not None:
            self._base = ctypes.addressof(ctypes.c_char.from_buffer(shm))
        else:  # local(): one process's own slots (single-rank use, tools/node_probe.py)
            self._mem = (ctypes.c_uint64 * (self.SLOTS * self.SLOT_BYTES // 8))()
            self._base = ctypes.addressof(self._mem)
        self._votes = self._base + self.SLOTS * self.SLOT_BYTES
        self._epoch = 0
        self._calls = 0
        self._native = None  # node_mine's dpow_node_mine call state (_NativeCall), built at first use

    @property
    def shared(self) -> bool:
        """The board is mapped by every rank of the node (create()): node_mine votes through it."""
        return self._shm is not None and self.world > 0

    @classmethod
    def nbytes(cls, world: int) -> int:
        return cls.SLOTS * cls.SLOT_BYTES + 2 * world * cls.VOTE_BYTES

    def vote(self, values):
        """MIN over the node's ranks of three int64 (dpow_node_vote); every rank calls it at
        the same boundaries, with the same values' meaning, and gets the same result."""
        import ctypes

        from ._lib import check, lib
        self._epoch += 1
        vin = (ctypes.c_int64 * 3)(*values)
        vout = (ctypes.c_int64 * 3)()
        rc = lib().dpow_node_vote(self._votes, self.rank, self.world, self._epoch, vin, vout, self.VOTE_TIMEOUT_NS)
        if rc < 0:
            raise NodeError(f"rank {self.rank}: node vote failed ({rc}): {lib().dpow_last_error().decode()}")
        return [int(x) for x in vout]

    @classmethod
    def local(cls) -> "NodeBoard":
        """A board in this process's memory (no other rank can map it)."""
        from ._lib import lib
        board = cls()
        for i in range(cls.SLOTS):
            lib().dpow_node_slot_reset(board.slot(i))
        return board

    @classmethod
    def create(cls, group=None) -> Optional["NodeBoard"]:
        """The segment is a file of /dev/shm that rank 0 creates and unlinks once every rank has
        mapped it, opened with os.open + mmap: multiprocessing.shared_memory would register it
        with a resource tracker that ranks spawned from one parent share, whose cleanup then
        printed a KeyError traceback into every GPU log."""
        import mmap
        import os
        import socket
        import uuid

        import torch.distributed as dist

        from ._lib import lib
        me = (socket.gethostname(), open("/proc/sys/kernel/random/boot_id").read().strip())
        world = dist.get_world_size(group)
        hosts = [None] * world
        dist.all_gather_object(hosts, me, group=group)
        if any(h != me for h in hosts):
            return None
        rank = dist.get_rank(group)
        name = [None]
        size = cls.nbytes(world)
        shm = None
        if rank == 0:
            path = f"/dev/shm/dpow_node_{os.getpid()}_{uuid.uuid4().hex[:12]}"
            try:
                fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
                try:
                    os.ftruncate(fd, size)
                    shm = mmap.mmap(fd, size)
                finally:
                    os.close(fd)
                name[0] = path
            except OSError:  # e.g. /dev/shm full: every rank goes on without a board (name None)
                try:
                    os.unlink(path)
                except OSError:
                    pass
                name[0] = None
        dist.broadcast_object_list(name, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if name[0] is None:
            return None
        ok = [True]
        if rank != 0:
            try:
                fd = os.open(name[0], os.O_RDWR)
                try:
                    shm = mmap.mmap(fd, size)
                finally:
                    os.close(fd)
            except (OSError, ValueError):
                ok[0], shm = False, None
        # every rank must have it mapped, or none uses it
        oks = [None] * world
        dist.all_gather_object(oks, ok[0], group=group)
        if rank == 0:  # mapped by every rank that could: nothing is left in /dev/shm, whatever happens next
            try:
                os.unlink(name[0])
            except OSError:
                pass
        if not all(oks):
            if shm is not None:
                shm.close()
            return None
        board = cls(shm, world, rank)
        if rank == 0:
            for i in range(cls.SLOTS):
                lib().dpow_node_slot_reset(board.slot(i))
            shm[cls.SLOTS * cls.SLOT_BYTES:size] = bytes(2 * world * cls.VOTE_BYTES)
        dist.barrier(group=group)
        return board

    def slot(self, i: int) -> int:
        return self._base + (i % self.SLOTS) * self.SLOT_BYTES

    def begin(self) -> int:
        return self.slot(self._calls)

    def end(self):
        from ._lib import lib
        lib().dpow_node_slot_reset(self.slot(self._calls + 2))
        self._calls += 1

    def best(self, slot: int) -> int:
        import ctypes
        return ctypes.c_uint64.from_address(slot).value

    def stop(self, slot: int):
        from ._lib import lib
        lib().dpow_node_stop(slot)

    def post(self, slot: int, global_idx: int):
        from ._lib import lib
        lib().dpow_node_post(slot, global_idx)

    def close(self):
        """Unmap the board (every rank's context detached first: node_mine detaches at its
        end); the library drops its HIP registration of the pages (dpow_node_release), so a
        later board mapped at the same address is registered afresh.  A local() board
        releases its pages the same way before its memory goes (dpow.h: mandatory for any
        slot memory)."""
        if self._shm is None and self._base:
            from ._lib import check, lib
            check(lib().dpow_node_release(self._base, self.nbytes(self.world)), "dpow_node_release")
            self._base = 0
            self._mem = None
            return
        if self._shm is not None:
            from ._lib import DpowError, check, lib
            err = None
            try:
                check(lib().dpow_node_release(self._base, self.nbytes(self.world)), "dpow_node_release")
            except DpowError as e:
                # A context still attached (a failed search skipped its detach): the pages stay
                # registered, so the mapping is left to the process -- unmapping it under a
                # registration would let a later mapping at the same address match it.  The
                # error is raised after the cleanup, so it never hides the one that led here.
                err = e
            self._base = 0
            if err is None:
                try:
                    self._shm.close()
                except BufferError:  # a ctypes view still alive; the mapping goes with the process
                    pass
            self._shm = None
            if err is not None:
                raise err


# With a node board, hits end every rank's batch at once, so a batch costs its boundary
# (the search call and the all-reduce) only when it holds no hit: batches can be long.
BOARD_BATCH_CANDIDATES = 1 << 33


def first_window_k(num_trailing_zeros: int, world: int, factor: float) -> int:
    """The first window of a node search on a board, in k: `factor` times the candidates this
    rank's partition expects before its first hit (16^N R / 256 of R = 256 / world per k), at
    least one k; 0 when factor is 0 (the first window is a whole board batch)."""
    if factor <= 0:
        return 0
    rbits = 8 - int(math.log2(world)) % 9
    expect = (16.0 ** min(max(num_trailing_zeros, 0), 32)) * (1 << rbits) / 256.0
    return max(1, int(factor * expect) >> rbits)


# A/B knob of the first window (multiples of the per-rank expected first hit; 0 = off)
NODE_FIRST_FACTOR = float(__import__("os").environ.get("DPOW_NODE_FIRST", "0") or 0)


def _miner_class():
    from .search import Miner
    return Miner


class _NativeCall:
    """The ctypes state of one board's dpow_node_mine calls, built once: the bound entry
    point, the out-parameters and their pointers, the slot-reset entry point.  A node search
    of tens of microseconds paid ~5 us of Python (imports, ctypes objects, lookups) around the
    call, each time (tools/search_timeline.py)."""

    def __init__(self):
        import ctypes

        from ._lib import DPOW_MAX_SECRET, lib
        L = lib()
        self.fn = L.dpow_node_mine
        self.reset = L.dpow_node_slot_reset
        self.last_error = L.dpow_last_error
        self.epoch = ctypes.c_uint64(0)
        self.best = ctypes.c_uint64(DPOW_NO_HIT)
        self.sec = (ctypes.c_uint8 * DPOW_MAX_SECRET)()
        self.slen = ctypes.c_size_t()
        self.batches = ctypes.c_uint32()
        self.p_epoch = ctypes.pointer(self.epoch)
        self.p_best = ctypes.pointer(self.best)
        self.p_slen = ctypes.pointer(self.slen)
        self.p_batches = ctypes.pointer(self.batches)


def _node_mine_native(miner, board: "NodeBoard", nonce: Sequence[int], num_trailing_zeros: int, rank: int,
                      world: int, k_start: int, k_limit: int, batch_k: int, first_k: int) -> NodeResult:
    """node_mine over a board in one call of dpow_node_mine (include/dpow.h, ABI 4): the batch
    loop, the Found fan-out and the node vote in C, no Python round per batch."""
    nc = board._native
    if nc is None:
        nc = board._native = _NativeCall()
    calls = board._calls
    slot = board._base + (calls % board.SLOTS) * board.SLOT_BYTES
    n = bytes(nonce)
    nc.epoch.value = board._epoch
    votes = board._votes if (board.shared and board.world == world) else None
    try:
        rc = nc.fn(miner._ctx, slot, votes, rank, world, nc.p_epoch, board.VOTE_TIMEOUT_NS, n, len(n),
                   num_trailing_zeros, k_start, k_limit, first_k, batch_k, nc.p_best, nc.sec, nc.p_slen,
                   nc.p_batches)
    finally:
        board._epoch = nc.epoch.value
        # board.end(): the slot two calls ahead is reset for its next user
        nc.reset(board._base + ((calls + 2) % board.SLOTS) * board.SLOT_BYTES)
        board._calls = calls + 1
    if rc == FOUND:
        best = nc.best.value
        return NodeResult(FOUND, best, bytes(nc.sec[:nc.slen.value]), owner_rank(best, world), nc.batches.value)
    if rc == EPROTO:
        raise NodeError(f"rank {rank}: {nc.last_error().decode()}")
    if rc < 0:
        from ._lib import DpowError
        raise DpowError(rc, f"rank {rank}: dpow_node_mine: {nc.last_error().decode()}")
    return NodeResult(rc, batches=nc.batches.value)


def _never() -> bool:
    return False


def _native_applies(board: "NodeBoard", world: int) -> bool:
    """dpow_node_mine decides the node's answer from the board's votes alone: when the board is
    shared by exactly `world` ranks, or when no process group runs (then the rank's values alone
    decide, as node_mine's local_only path: one rank, or the one-GPU emulation of
    tools/node_probe.py).  A local board, or a shared board of another size, under an initialised
    group would let every rank vote alone and return its own partition's first hit: that case
    takes the Python loop, whose boundary is the group's all-reduce."""
    if board.shared and board.world == world:
        return True
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized())


def node_mine(search_fn: Callable, nonce: Sequence[int], num_trailing_zeros: int, rank: int, world: int,
              batch_k: Optional[int] = None, k_start: int = 0, k_limit: int = DPOW_K_LIMIT, group=None,
              device=None, cancelled: Callable[[], bool] = _never, growth: int = 4,
              batch_k_max: Optional[int] = None, batch_candidates_max: int = 1 << 29,
              board: Optional[NodeBoard] = None, attach_fn: Optional[Callable[[Optional[int]], None]] = None,
              miner=None) -> NodeResult:
    """Search until the first hit of the whole node (deterministic) or a cancel vote.

    search_fn(nonce, ntz, worker_byte, worker_bits, k_begin, k_end, bound) -> SearchResult
    is this rank's one-window search (Miner.search for the GPU product).

    Every rank must finish a batch before the all-reduce, so a batch bounds the
    overshoot past the hit, and each batch costs a fixed c on top of its hashing.
    - batch_k None (default): one constant batch per rank sized for N and the node
      (auto_batch_candidates, the expected-time optimum of the geometric first hit);
      with a board, BOARD_BATCH_CANDIDATES (the board ends a batch at its first hit).
    - batch_k given: batches start at batch_k chunks and grow by `growth` up to
      batch_k_max (default: batch_candidates_max = 2^29 candidates per rank, 2.5 ms of
      hashing; 2^24 k at 8 GPUs).  For T ms of hashing per rank, c T / B + B / 2 is
      smallest near B = sqrt(2 c T), 2.3 ms for N = 9 at 8 GPUs.

    The batch boundary is a MIN over [best index, running, healthy] across the ranks: the
    node vote of a shared board (NodeBoard.vote, every rank on one host), else the
    all-reduce over the process group whenever one is initialised (also at world = 1).  A
    rank whose search raises votes healthy = 0 at the same boundary, so no rank is left
    waiting for a vote the failed rank never casts: the failing rank re-raises its error,
    the others raise NodeError (coordinator.go:202-206: a missing result is fatal, not
    silent).

    board / attach_fn: the node's shared-memory Found fan-out (NodeBoard); attach_fn(slot)
    attaches a slot address to this rank's search context (Miner.attach_node), None
    detaches.  Without attach_fn the board still carries the vote and the posted hits
    between batches, but no running kernel sees another rank's hit, so the batch stays the
    expected-time one (not BOARD_BATCH_CANDIDATES, which relies on the kernels stopping).

    miner: a distpow.Miner with a board and no explicit batch_k: the whole loop runs in C
    (dpow_node_mine, round 5) -- the same windows, votes and answers, without a Python round
    per batch (4-5 us per node search).  search_fn and attach_fn are then unused.  Only when the
    board's votes decide the node (_native_applies) and no `cancelled` callback is given (the C
    loop sees the context's cancel flag, not a Python predicate); otherwise the Python loop runs.
    """
    if (miner is not None and board is not None and batch_k is None and cancelled is _never and
            isinstance(miner, _miner_class()) and _native_applies(board, world)):
        wbits = world.bit_length() - 1
        if world < 1 or world & (world - 1):
            partition_of_rank(rank, world)  # raises
        bk = max(1, BOARD_BATCH_CANDIDATES >> (8 - wbits % 9))
        return _node_mine_native(miner, board, nonce, num_trailing_zeros, rank, world, k_start, k_limit, bk,
                                 first_window_k(num_trailing_zeros, world, NODE_FIRST_FACTOR))
    import torch
    import torch.distributed as dist

    wb, wbits = partition_of_rank(rank, world)
    if batch_k is None:
        cand = (BOARD_BATCH_CANDIDATES if board is not None and attach_fn is not None
                else auto_batch_candidates(num_trailing_zeros, world))
        batch_k = max(1, cand >> (8 - wbits % 9))
        growth = 1
    if batch_k_max is None:
        batch_k_max = max(1, batch_candidates_max >> (8 - wbits % 9))
    dist_on = dist.is_available() and dist.is_initialized()
    # The batch boundary: the node vote on a shared board (all ranks on one host), else the
    # all-reduce over the process group (RCCL with the "nccl" backend).
    board_vote = board is not None and board.shared and board.world == world
    # no process group and no shared board (one rank alone, tools/node_probe.py): the
    # boundary is this rank's own values
    local_only = not board_vote and not dist_on
    if not board_vote and not local_only:
        if device is None:
            backend = dist.get_backend(group) if dist_on else "gloo"
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        buf = torch.empty(3, dtype=torch.int64, device=device)
        # With a device buffer (RCCL), a pinned host twin carries the values in and out:
        # stream-ordered copies around the all-reduce and one stream synchronize per batch.
        on_gpu = buf.device.type == "cuda"
        hbuf = torch.empty(3, dtype=torch.int64, pin_memory=True) if on_gpu else buf
    slot = board.begin() if board is not None else None
    if attach_fn is None:
        attach_fn = lambda s: None  # noqa: E731
    bound = DPOW_NO_HIT
    secret = None
    k = k_start
    batches = 0
    attached = False
    try:
        # A rank that cannot attach its slot (e.g. the shared page refused by its GPU) fails its
        # first batch: it stops the slot, so the other ranks' searches end at once, and votes
        # healthy = 0 at the first boundary, so nobody waits out the vote's timeout.
        attach_err = None
        if slot is not None:
            try:
                attach_fn(slot)
                attached = True
            except Exception as e:
                attach_err = e
                board.stop(slot)
        while k < k_limit:
            ke = min(k_limit, k + batch_k)
            batch_k = min(batch_k * growth, max(batch_k, batch_k_max))
            err = attach_err
            r = None
            try:
                if err is None:
                    r = search_fn(nonce, num_trailing_zeros, wb, wbits, k, ke, bound)
            except Exception as e:  # voted below; re-raised after the all-reduce
                err, r = e, None
                if slot is not None:
                    board.stop(slot)
            found = r is not None and r.status == FOUND
            mine = r.global_idx if found else DPOW_NO_HIT
            if found:
                secret = r.secret
            running = 0 if (err is not None or r.status == CANCELLED or cancelled()) else 1
            # The board's best is another rank's verified hit in this same batch (one slot per
            # node search): voting it too ends the batch for a rank that was bounded by it even
            # without a process group, and the all-reduce's minimum is unchanged.
            vote = min(mine, board.best(slot)) if slot is not None else mine
            if board_vote:
                best, all_running, healthy = board.vote([vote, running, 0 if err is not None else 1])
            elif local_only:
                best, all_running, healthy = vote, running, 0 if err is not None else 1
            else:
                hbuf[0], hbuf[1], hbuf[2] = vote, running, 0 if err is not None else 1
                if on_gpu:
                    buf.copy_(hbuf, non_blocking=True)
                if dist_on:
                    dist.all_reduce(buf, op=dist.ReduceOp.MIN, group=group)
                if on_gpu:
                    hbuf.copy_(buf, non_blocking=True)
                    torch.cuda.current_stream(buf.device).synchronize()
                best, all_running, healthy = (int(x) for x in hbuf.tolist())
            batches += 1
            if not healthy:
                if err is not None:
                    raise err
                raise NodeError(f"rank {rank}: another rank's search failed in batch {batches} "
                                f"(k window [{k}, {ke}))")
            if best != DPOW_NO_HIT:
                own = owner_rank(best, world)
                if best != mine:
                    secret = None  # another rank's partition won; its owner holds the secret bytes
                from .search import secret_from_index
                return NodeResult(FOUND, best, secret if secret is not None else secret_from_index(best), own, batches)
            if not all_running:
                return NodeResult(CANCELLED, batches=batches)
            k = ke
        return NodeResult(EXHAUSTED, batches=batches)
    finally:
        if slot is not None:
            if attached:
                try:
                    attach_fn(None)
                except Exception:  # never hides the error that brought us here
                    pass
            board.end()


def node_mine_async(search_fn: Callable, nonce: Sequence[int], num_trailing_zeros: int, rank: int, world: int,
                    bound_fn: Callable[[int], None] = lambda g: None, cancel_fn: Callable[[], None] = lambda: None,
                    clear_fn: Callable[[], None] = lambda: None, batch_k: Optional[int] = None,
                    k_start: int = 0, k_limit: int = DPOW_K_LIMIT, group=None, device=None,
                    cancelled: Callable[[], bool] = lambda: False, growth: int = 4,
                    batch_candidates_max: int = 1 << 31, tick_s: float = 1e-4,
                    sync_candidates: int = 1 << 27, tick_group=None, tick_device=None) -> NodeResult:
    """node_mine without batch boundaries on the search path: the same answer (the node's
    minimum global index, i.e. the workerBits = 0 first hit), found sooner.

    Each rank searches its partition in a thread, window after window (growing from
    batch_k chunks by `growth` up to batch_candidates_max per window), never waiting for
    the other ranks.  The calling thread ticks every tick_s: one all-reduce MIN of
    [best hit, coverage, running] over the node (RCCL over xGMI with the "nccl" backend),
    where a rank's coverage is the global index below which it has searched all of its
    candidates (its window frontier, or everything once it holds a hit).  When a best hit
    is known, every rank lowers the bound of its in-flight search to it (bound_fn ->
    Miner.bound, dpow_search_bound: the kernel stops claiming work above it at its next
    group), and the node is done as soon as every rank's coverage reaches the best hit:
    no rank hashes a whole batch past the answer, and no rank idles at a batch
    boundary.  Every rank sees the same reduced values, so all take the same decision on
    the same tick (the all-reduces stay matched).  cancel_fn / clear_fn raise and clear
    the pinned cancel flag to end the in-flight search at the end.

    The first sync_candidates per rank (2^27: 0.6 ms of hashing) run as node_mine's
    synchronous batches (batch_k None: its constant expected-time batch; else growing from
    batch_k): a small N ends there without a thread or a tick (the ticked
    loop costs a few hundred microseconds of latency, which only pays on longer searches).

    tick_group / tick_device: where the ticks' all-reduce runs (default: group / device).
    With the nccl backend a gloo group on the host keeps the 24-byte control message off
    the GPUs, whose CUs the persistent search grids occupy while the ticks run.

    search_fn(nonce, ntz, worker_byte, worker_bits, k_begin, k_end, bound) -> SearchResult.
    """
    import torch
    import torch.distributed as dist

    wb, wbits = partition_of_rank(rank, world)
    rbits = 8 - wbits % 9
    k_switch = min(k_limit, k_start + (sync_candidates >> rbits))
    if k_switch > k_start:
        r = node_mine(search_fn, nonce, num_trailing_zeros, rank, world, batch_k=batch_k, k_start=k_start,
                      k_limit=k_switch, group=group, device=device, cancelled=cancelled, growth=growth)
        if r.status != EXHAUSTED or k_switch >= k_limit:
            return r
        # continue with windows about the size of the synchronous phase's last batches
        batch_k = max(batch_k or 1, (k_switch - k_start) >> 1)
        k_start = k_switch
    if batch_k is None:
        batch_k = max(1, auto_batch_candidates(num_trailing_zeros, world) >> rbits)
    batch_k_max = max(1, batch_candidates_max >> rbits)
    dist_on = dist.is_available() and dist.is_initialized()
    if device is None:
        backend = dist.get_backend(group) if dist_on else "gloo"
        device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    if tick_group is None:
        tick_group = group
    if tick_device is None:
        if tick_group is not None and dist_on:
            tick_device = torch.device("cpu") if dist.get_backend(tick_group) == "gloo" else device
        else:
            tick_device = device
    INF = DPOW_NO_HIT
    mu = threading.Lock()
    st = {"best": INF, "secret": None, "cover": k_start << 8, "cancelled": False, "seen": INF, "error": None}
    stop = threading.Event()
    changed = threading.Event()  # the searcher's state moved: tick now rather than at the next period

    def searcher():
        k, bk = k_start, batch_k
        try:
            while not stop.is_set():
                with mu:
                    bound = min(st["best"], st["seen"])
                if k >= k_limit or (k << 8) >= bound:  # nothing of ours below the bound is left
                    with mu:
                        st["cover"] = INF if (k << 8) >= bound else max(st["cover"], k_limit << 8)
                    return
                ke = min(k_limit, k + bk)
                bk = min(bk * growth, max(bk, batch_k_max))
                r = search_fn(nonce, num_trailing_zeros, wb, wbits, k, ke, bound)
                with mu:
                    if r.status == FOUND:
                        if r.global_idx < st["best"]:
                            st["best"], st["secret"] = r.global_idx, r.secret
                        st["cover"] = INF  # every candidate of ours below our first hit is searched
                        return
                    if r.status == CANCELLED:
                        st["cancelled"] = True
                        return
                    st["cover"] = ke << 8
                changed.set()
                k = ke
        except BaseException as e:  # surfaced by the tick loop as a cancel vote + re-raise
            with mu:
                st["error"] = e
                st["cancelled"] = True
        finally:
            changed.set()

    th = threading.Thread(target=searcher, daemon=True)
    th.start()
    buf = torch.empty(3, dtype=torch.int64, device=tick_device)
    ticks = 0
    try:
        while True:
            with mu:
                vals = [st["best"], st["cover"], 0 if (st["cancelled"] or cancelled()) else 1]
            buf.copy_(torch.tensor(vals, dtype=torch.int64))
            if dist_on:
                dist.all_reduce(buf, op=dist.ReduceOp.MIN, group=tick_group)
            ticks += 1
            gbest, gcover, grun = (int(x) for x in buf.tolist())
            if gbest != INF and gcover >= gbest:
                status = FOUND
                break
            if not grun:
                status = CANCELLED
                break
            if gbest == INF and gcover >= (k_limit << 8):
                status = EXHAUSTED
                break
            if gbest != INF:
                with mu:
                    lower = gbest < st["seen"]
                    st["seen"] = min(st["seen"], gbest)
                if lower:
                    bound_fn(gbest)  # the in-flight search stops at the node's best hit
            changed.wait(tick_s)
            changed.clear()
    finally:
        stop.set()
        cancel_fn()
        th.join()
        clear_fn()
    if st["error"] is not None:
        raise st["error"]
    if status != FOUND:
        return NodeResult(status, batches=ticks)
    secret = st["secret"] if st["best"] == gbest else None
    if secret is None:  # another rank's partition won; its owner holds the secret bytes
        from .search import secret_from_index
        secret = secret_from_index(gbest)
    return NodeResult(FOUND, gbest, secret, owner_rank(gbest, world), ticks)
