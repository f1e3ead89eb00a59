"""Bulk recalculated verify of stored chunks and checksum diffing.

* ``Scrubber``  -- the resync / scrub consumer of the recalculate path: every chunk is
  re-checksummed with its stored type and compared with its stored value, as
  ``AioReadJob::setResult`` does with ``recalculateChecksum`` set
  (src/storage/aio/BatchReadJob.cc:43-54; set for full-chunk syncing reads at
  src/storage/service/ReliableForwarding.cc:179-180).  Chunks stay in HBM; the plan's
  descriptors are uploaded once and re-run on every pass.
* ``diff_checksums`` -- the checksum comparison ResyncWorker makes between the local
  and the remote chunk metadata (src/storage/sync/ResyncWorker.cc:252,
  ``meta.checksum() != remoteMeta.checksum``).
"""
from __future__ import annotations

from typing import Dict, Hashable, List, Sequence, Tuple

import numpy as np

from .engine import DESC_DTYPE, ChecksumInfo, ChecksumType, MemKind, Plan

kChecksumMismatch = 4080  # StorageCode::kChecksumMismatch


class Scrubber:
    """chunks[i] = (device address, length, stored ChecksumInfo).  NONE-typed chunks are
    not verified (their recomputed value is {NONE, 0}, equal to what they store)."""

    def __init__(self, chunks: Sequence[Tuple[int, int, ChecksumInfo]], device: int = 0):
        import torch

        self.n = len(chunks)
        descs = np.zeros(self.n, dtype=DESC_DTYPE)
        expected = np.zeros(self.n, dtype=np.uint32)
        for i, (ptr, length, ck) in enumerate(chunks):
            descs[i] = (ptr, length, 0xFFFFFFFF, int(ck.type), int(MemKind.DEVICE), 0)
            expected[i] = ck.value & 0xFFFFFFFF if ck.type != ChecksumType.NONE else 0
        self.plan = Plan(descs, device)
        dev = torch.device("cuda", device)
        self.expected = torch.from_numpy(expected.view(np.int32)).to(dev)
        self.out = torch.zeros(self.n, dtype=torch.int32, device=dev)
        self.ok = torch.zeros(self.n, dtype=torch.uint8, device=dev)
        self.mismatch = torch.zeros(1, dtype=torch.int32, device=dev)

    def run_async(self, stream=None) -> None:
        """Enqueue one verify pass (nothing is synchronised)."""
        self.mismatch.zero_()
        self.plan.run(self.out, self.expected, self.ok, self.mismatch, stream)

    def run(self, stream=None) -> List[int]:
        """One pass; returns the indices whose recomputed checksum differs from the stored one."""
        self.run_async(stream)
        if int(self.mismatch.item()) == 0:
            return []
        return np.nonzero(self.ok.cpu().numpy() == 0)[0].tolist()

    def recomputed(self) -> np.ndarray:
        return self.out.cpu().numpy().view(np.uint32)

    def close(self) -> None:
        self.plan.close()


def diff_checksums(local: Dict[Hashable, ChecksumInfo], remote: Dict[Hashable, ChecksumInfo]):
    """(ids whose checksums differ, ids only local, ids only remote)."""
    differ = sorted((k for k in local.keys() & remote.keys() if local[k] != remote[k]), key=repr)
    return differ, sorted(local.keys() - remote.keys(), key=repr), sorted(remote.keys() - local.keys(), key=repr)
