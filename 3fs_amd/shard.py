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


def _gather_bytes(mine: np.ndarray, sizes: Sequence[int], group=None) -> List[np.ndarray]:
    """Every rank's byte array (rank k's has sizes[k] bytes, known to all ranks from the partition): one
    all_gather of equal-length uint8 tensors (padded to the largest), no pickling."""
    import torch
    import torch.distributed as dist

    width = max(max(sizes), 1)
    buf = torch.zeros(width, dtype=torch.uint8)
    if mine.size:
        buf[: mine.size] = torch.from_numpy(np.ascontiguousarray(mine).view(np.uint8).reshape(-1))
    outs = [torch.empty(width, dtype=torch.uint8) for _ in sizes]
    dist.all_gather(outs, buf, group=group)
    return [o.numpy()[:k] for o, k in zip(outs, sizes)]


def run_sharded(items: Sequence, expected: Sequence[int], verify_fn: Callable, rank: int, world: int,
                lengths: Sequence[int] = None, group=None):
    """Verify this rank's slice with ``verify_fn(items, expected) -> (raw, ok)`` and
    gather every rank's results (control-plane gather of 5 B per chunk: one all_gather of
    fixed-size byte tensors, each rank's slice length known to all from the partition).

    Returns (raw uint32[n], ok bool[n]) for the whole batch on every rank."""
    if lengths is None:
        lengths = [getattr(it, "nbytes", None) or len(it) for it in items]
    parts = partition(lengths, world)
    lo, hi = parts[rank]
    raw, ok = verify_fn(items[lo:hi], list(expected[lo:hi]))
    n = len(items)
    out_raw = np.zeros(n, dtype=np.uint32)
    out_ok = np.zeros(n, dtype=bool)
    rec = np.zeros(hi - lo, dtype=[("raw", "<u4"), ("ok", "u1")])
    rec["raw"] = np.asarray(raw, dtype=np.uint32)
    rec["ok"] = np.asarray(ok, dtype=bool)
    if world == 1:
        got = [rec.view(np.uint8)]
    else:
        got = _gather_bytes(rec.view(np.uint8), [(b - a) * rec.dtype.itemsize for a, b in parts], group)
    for (a, b), g in zip(parts, got):
        r = g.view(rec.dtype)
        out_raw[a:b] = r["raw"]
        out_ok[a:b] = r["ok"].astype(bool)
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
    original op order (control-plane gather of the small per-op records: one all_gather of fixed-size
    byte tensors, no pickling; every rank's records share one dtype)."""
    owners = partition_updates(op_chunk, chunk_bytes, world)
    mine = np.ascontiguousarray(np.asarray(apply_fn(owners[rank])))
    n = len(op_chunk)
    out = np.zeros(n, dtype=mine.dtype)
    if world == 1:
        out[owners[0]] = mine
        return out
    # every rank knows every rank's op indices (the partition) and the record type (its own results')
    got = _gather_bytes(mine.view(np.uint8), [len(ix) * mine.dtype.itemsize for ix in owners], group)
    for ix, g in zip(owners, got):
        out[ix] = g.view(mine.dtype)
    return out
