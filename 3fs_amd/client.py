"""Client-side checksum work of ``StorageClientImpl`` batched on the GPU.

* write path  (src/client/storage/StorageClientImpl.cc:1878-1883): every write IO carries
  ``ChecksumInfo::create(config_.chunk_checksum_type(), data, length)``.
* read verify (StorageClientImpl.cc:1720-1737): with ``verifyChecksum()``, every read IO
  with a non-zero result length is re-checksummed with the server's checksum type and a
  difference fails the IO with ``StorageClientCode::kChecksumMismatch`` (7015,
  src/common/utils/StatusCodeDetails.h:236).
* split reads (StorageClientImpl.cc:1607-1633): a large read split into pieces gets the
  first piece's checksum, combined with every further piece's (``ChecksumInfo::combine``).

The checksum switches are the reference's (src/client/storage/StorageClient.h:161-221, 418):
``ReadOptions.enableChecksum`` (default off) and ``WriteOptions.enableChecksum`` (default on),
both forced on in debug builds (``#ifndef NDEBUG``) and off under the ``bypass_disk_io`` /
``bypass_rdma_xmit`` debug options; ``IoOptions::Config.chunk_checksum_type`` (CRC32C).

Payloads may be torch CUDA tensors (read in place) or host buffers (staged by the engine).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .engine import ChecksumInfo, ChecksumType, _check, batch_create, lib

kChecksumMismatch = 7015  # StorageClientCode::kChecksumMismatch


@dataclass
class DebugOptions:
    """StorageClient.h:161-163."""
    bypass_disk_io: bool = False
    bypass_rdma_xmit: bool = False


@dataclass
class _ChecksumOptions:
    enable_checksum: bool
    debug: DebugOptions = field(default_factory=DebugOptions)
    ndebug: bool = True  # a release build (NDEBUG); debug builds always checksum

    def verify_checksum(self) -> bool:
        """StorageClient.h:196-204 / 214-222."""
        enabled = self.enable_checksum if self.ndebug else True
        return enabled and not self.debug.bypass_disk_io and not self.debug.bypass_rdma_xmit


@dataclass
class ReadOptions(_ChecksumOptions):
    enable_checksum: bool = False  # CONFIG_HOT_UPDATED_ITEM(enableChecksum, false), StorageClient.h:192


@dataclass
class WriteOptions(_ChecksumOptions):
    enable_checksum: bool = True  # CONFIG_HOT_UPDATED_ITEM(enableChecksum, true), StorageClient.h:211


@dataclass
class ClientConfig:
    chunk_checksum_type: int = ChecksumType.CRC32C  # CONFIG_ITEM(chunk_checksum_type, CRC32C), StorageClient.h:418


def read_checksum_type(config: Optional[ClientConfig] = None, options: Optional[ReadOptions] = None) -> int:
    """The checksum type a read request asks the server for (StorageClientImpl.cc:703):
    chunk_checksum_type when the read verifies, else NONE."""
    config = config or ClientConfig()
    options = options or ReadOptions()
    return int(config.chunk_checksum_type) if options.verify_checksum() else int(ChecksumType.NONE)


def write_checksums(payloads: Sequence, checksum_type: Optional[int] = None, stream=None,
                    config: Optional[ClientConfig] = None, options: Optional[WriteOptions] = None) -> List[ChecksumInfo]:
    """One ChecksumInfo per write IO payload (StorageClientImpl.cc:1878-1883): created with the
    client's chunk_checksum_type when ``options.verify_checksum()``, else the default {NONE, 0}.
    ``checksum_type`` (if given) overrides ``config.chunk_checksum_type``."""
    options = options or WriteOptions()
    if not options.verify_checksum():
        return [ChecksumInfo(ChecksumType.NONE, 0) for _ in payloads]
    ctype = checksum_type if checksum_type is not None else (config or ClientConfig()).chunk_checksum_type
    t, v = batch_create(payloads, int(ctype), stream=stream)
    return [ChecksumInfo(ChecksumType(int(a)), int(b)) for a, b in zip(t, v)]


def verify_read_checksums(results: Sequence[Tuple[object, int, ChecksumInfo]], stream=None,
                          options: Optional[ReadOptions] = None) -> np.ndarray:
    """results[i] = (data, result length, server checksum).  Returns per-IO status:
    0, or kChecksumMismatch when the local checksum differs (IOs of length 0 are skipped).
    With ``options`` given, nothing is checked unless ``options.verify_checksum()``
    (StorageClientImpl.cc:1720); without, every IO is checked."""
    status = np.zeros(len(results), dtype=np.uint32)
    if options is not None and not options.verify_checksum():
        return status
    idx = [i for i, (_, n, _) in enumerate(results) if n > 0]
    if not idx:
        return status
    items = [(results[i][0], results[i][1], 0xFFFFFFFF, int(results[i][2].type)) for i in idx]
    t, v = batch_create(items, stream=stream)
    for k, i in enumerate(idx):
        server = results[i][2]
        if int(t[k]) != int(server.type) or int(v[k]) != (server.value & 0xFFFFFFFF):
            status[i] = kChecksumMismatch
    return status


def fold_split_reads(groups: Sequence[Sequence[Tuple[ChecksumInfo, int]]]):
    """groups[g] = [(piece checksum, piece length), ...] in piece order.  Returns
    (ChecksumInfo per parent IO, status per parent: 0 or 4080 on a type mismatch)."""
    types, values, lens, begin = [], [], [], [0]
    for g in groups:
        for ck, n in g:
            types.append(int(ck.type))
            values.append(ck.value & 0xFFFFFFFF)
            lens.append(n)
        begin.append(len(types))
    ng = len(groups)
    t = np.asarray(types, dtype=np.uint8)
    v = np.asarray(values, dtype=np.uint32)
    ln = np.asarray(lens, dtype=np.uint64)
    b = np.asarray(begin, dtype=np.uint64)
    ot = np.zeros(ng, dtype=np.uint8)
    ov = np.zeros(ng, dtype=np.uint32)
    st = np.zeros(ng, dtype=np.uint32)
    ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
    _check(lib.h3c_combine_fold(ptr(t), ptr(v), ptr(ln), ptr(b), ng, ptr(ot), ptr(ov), ptr(st)))
    return [ChecksumInfo(ChecksumType(int(a)), int(c)) for a, c in zip(ot, ov)], st
