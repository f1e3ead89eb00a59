"""Shard a chunk batch across the GPUs of one node.

Chunks verify independently, so there is no data-path collective: each rank
takes a contiguous, byte-balanced slice of the batch, runs the engine on its own
GPU, and only the per-chunk results (4-byte value + ok flag) are gathered —
the storage analogue of ResyncWorker / ReliableForwarding scrubbing
(src/storage/sync/ResyncWorker.cc:252, src/storage/service/ReliableForwarding.cc:158-212).
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np


def partition(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) index ranges, one per rank, balanced by payload bytes.

    Boundaries sit where the byte prefix sum crosses k/world of the total, so a
    rank's share differs from the mean by at most one chunk."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = len(lengths)
    if n == 0:
        return [(0, 0)] * world
    prefix = np.concatenate([[0], np.cumsum(np.asarray(lengths, dtype=np.float64))])
    total = prefix[-1]
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        c = int(np.searchsorted(prefix, target, side="left"))
        c = min(max(c, cuts[-1]), n)
        cuts.append(c)
    cuts.append(n)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def run_sharded(items: Sequence, expected: Sequence[int], verify_fn: Callable, rank: int, world: int,
                lengths: Sequence[int] = None, group=None):
    """Verify this rank's slice with ``verify_fn(items, expected) -> (raw, ok)`` and
    gather every rank's results (control-plane gather of 5 B per chunk).

    Returns (raw uint32[n], ok bool[n]) for the whole batch on every rank."""
    import torch.distributed as dist

    if lengths is None:
        lengths = [getattr(it, "nbytes", None) or len(it) for it in items]
    lo, hi = partition(lengths, world)[rank]
    raw, ok = verify_fn(items[lo:hi], list(expected[lo:hi]))
    mine = (lo, np.asarray(raw, dtype=np.uint32), np.asarray(ok, dtype=bool))
    if world == 1:
        parts = [mine]
    else:
        parts = [None] * world
        dist.all_gather_object(parts, mine, group=group)
    n = len(items)
    out_raw = np.zeros(n, dtype=np.uint32)
    out_ok = np.zeros(n, dtype=bool)
    for lo_k, raw_k, ok_k in parts:
        out_raw[lo_k: lo_k + raw_k.size] = raw_k
        out_ok[lo_k: lo_k + ok_k.size] = ok_k
    return out_raw, out_ok


def partition_updates(op_chunk: Sequence[int], chunk_bytes: Sequence[int], world: int) -> List[np.ndarray]:
    """Shard a sequence of update ops by chunk: chunks are split
    into byte-balanced contiguous ranges and every op goes to the rank owning its chunk,
    so all writes to a chunk stay on one GPU in sequence order.  Returns, per rank, the op
    indices in their original order.  Ops naming a chunk outside the table go to rank 0
    (which reports them invalid)."""
    ranges = partition(chunk_bytes, world)
    owner = np.zeros(len(chunk_bytes), dtype=np.int64)
    for r, (lo, hi) in enumerate(ranges):
        owner[lo:hi] = r
    oc = np.asarray(op_chunk, dtype=np.int64)
    valid = (oc >= 0) & (oc < len(chunk_bytes))
    op_owner = np.where(valid, owner[np.clip(oc, 0, max(len(chunk_bytes) - 1, 0))] if len(chunk_bytes) else 0, 0)
    return [np.nonzero(op_owner == r)[0] for r in range(world)]


def run_sharded_updates(op_chunk: Sequence[int], chunk_bytes: Sequence[int], apply_fn: Callable, rank: int,
                        world: int, group=None):
    """Apply this rank's ops with ``apply_fn(op_indices) -> per-op result records`` (numpy
    structured or 1-D array, one entry per index) and gather every rank's results in the
    original op order (control-plane gather of the small per-op records)."""
    import torch.distributed as dist

    mine_idx = partition_updates(op_chunk, chunk_bytes, world)[rank]
    mine = (mine_idx, np.asarray(apply_fn(mine_idx)))
    if world == 1:
        parts = [mine]
    else:
        parts = [None] * world
        dist.all_gather_object(parts, mine, group=group)
    n = len(op_chunk)
    proto = next(p[1] for p in parts if p[1].size) if any(p[1].size for p in parts) else np.zeros(0)
    out = np.zeros(n, dtype=proto.dtype)
    for idx, res in parts:
        out[idx] = res
    return out
