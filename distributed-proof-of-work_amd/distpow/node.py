"""Multi-GPU search on one node: the coordinator's workerBits prefix fan-out
(coordinator.go:122-129, 179-199, 326) mapped onto G GPUs, one process per GPU.

Rank r of G = 2^b owns the reference worker partition (WorkerByte = r,
WorkerBits = b): threadBytes [r * 2^(8-b), (r+1) * 2^(8-b)) (worker.go:302-316).
All ranks scan the same k-window per batch.  At each batch boundary one
all-reduce MIN over [best global index, -running] (16 bytes; torch.distributed,
i.e. RCCL over xGMI with the "nccl" backend) picks the globally lowest index and
votes on cancellation.  The minimum over partitions of each partition's first
hit is the workerBits = 0 answer, so the result is deterministic and equals the
single-worker enumeration's first hit.

This replaces the reference's first-message-wins gather (coordinator.go:202) by
a deterministic reduction; the owner of the winning index is rank
(threadByte >> (8 - b)), the worker that would have reported WorkerResult.
"""
import math
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

from ._lib import CANCELLED, DPOW_K_LIMIT, DPOW_NO_HIT, EXHAUSTED, FOUND

__all__ = ["NodeResult", "node_mine", "partition_of_rank", "owner_rank"]


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


def node_mine(search_fn: Callable, nonce: Sequence[int], num_trailing_zeros: int, rank: int, world: int,
              batch_k: int = 1 << 8, k_start: int = 0, k_limit: int = DPOW_K_LIMIT, group=None,
              device=None, cancelled: Callable[[], bool] = lambda: False, growth: int = 4,
              batch_k_max: Optional[int] = None, batch_candidates_max: int = 1 << 29) -> NodeResult:
    """Search until the first hit of the whole node (deterministic) or a cancel vote.

    search_fn(nonce, ntz, worker_byte, worker_bits, k_begin, k_end, bound) -> SearchResult
    is this rank's one-window search (Miner.search for the GPU product).

    Batches start at batch_k chunks and grow by `growth` up to batch_k_max (default:
    batch_candidates_max = 2^29 candidates per rank, 2.5 ms of hashing; 2^24 k at 8
    GPUs).  Every rank must finish a batch before the all-reduce, so a batch bounds the
    overshoot past the hit: small first batches keep small N at a few short batches.
    The cap trades the per-batch cost c (the window's launch and drain, the all-reduce
    and the host round trip, ~0.1 ms) against the overshoot (about half the last batch):
    for T ms of hashing per rank the sum c T / B + B / 2 is smallest near B = sqrt(2 c T),
    2.3 ms for N = 9 at 8 GPUs (~26 ms per rank).  (Round 1 capped at 2^22 k, 0.6 ms.)
    """
    import torch
    import torch.distributed as dist

    wb, wbits = partition_of_rank(rank, world)
    if batch_k_max is None:
        batch_k_max = max(1, batch_candidates_max >> (8 - wbits % 9))
    dist_on = world > 1 and dist.is_available() and dist.is_initialized()
    if device is None:
        backend = dist.get_backend(group) if dist_on else "gloo"
        device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    buf = torch.empty(2, dtype=torch.int64, device=device)
    bound = DPOW_NO_HIT
    secret = None
    k = k_start
    batches = 0
    while k < k_limit:
        ke = min(k_limit, k + batch_k)
        batch_k = min(batch_k * growth, max(batch_k, batch_k_max))
        r = search_fn(nonce, num_trailing_zeros, wb, wbits, k, ke, bound)
        mine = r.global_idx if r.status == FOUND else DPOW_NO_HIT
        if r.status == FOUND:
            secret = r.secret
        running = 0 if (r.status == CANCELLED or cancelled()) else 1
        # one host->device copy in and one device->host copy out per batch (each is a
        # synchronous round trip of tens of microseconds with RCCL's device tensors)
        buf.copy_(torch.tensor([mine, running], dtype=torch.int64))
        if dist_on:
            dist.all_reduce(buf, op=dist.ReduceOp.MIN, group=group)
        batches += 1
        best, all_running = (int(x) for x in buf.tolist())
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
