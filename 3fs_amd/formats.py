"""Adjacent checksum formats on the same GPU kernels.

* ``Checksum.calc_serde``  -- RPC message checksum, ``Checksum::calcSerde``
  (src/common/net/MessageHeader.h:32-37): ``folly::crc32c(data, size, 0)`` with the low
  byte replaced by ``kSerdeMessageMagicNum`` (0x86) | compressed; verified on receipt by
  ``Processor::unpackSerdeMsg`` (src/common/net/Processor.h:113-117).
* ``rust_crc32c``          -- the crc32c crate 0.6.8 API the Rust chunk engine calls
  (std domain: std = ~raw; chunk_engine/src/alloc/chunk.rs:152-269).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from .engine import ChecksumType, _check, _desc_array, _stream_handle, _u64, lib

SERDE_MAGIC = 0x86  # kSerdeMessageMagicNum, MessageHeader.h:14


def is_serde_message(checksum: int) -> bool:
    """MessageHeader::isSerdeMessage (MessageHeader.h:24)."""
    return (checksum & 0xFE) == SERDE_MAGIC


def is_compressed(checksum: int) -> bool:
    """MessageHeader::isCompressed (MessageHeader.h:26)."""
    return bool(checksum & 1)


class Checksum:
    """``hf3fs::net::Checksum`` (MessageHeader.h:32-37)."""

    @staticmethod
    def calc_serde(data, compressed: bool = False, stream=None) -> int:
        return int(batch_serde_checksum([data], [compressed], stream=stream)[0])


def batch_serde_checksum(messages: Sequence, compressed: Optional[Sequence[bool]] = None, stream=None) -> np.ndarray:
    descs, keep = _desc_array(messages, ChecksumType.CRC32C, 0)
    n = len(descs)
    out = np.zeros(n, dtype=np.uint32)
    comp = None if compressed is None else np.ascontiguousarray(np.asarray(compressed, dtype=np.uint8))
    _check(lib.h3c_batch_serde_checksum(descs.ctypes.data, n, comp.ctypes.data if comp is not None else None,
                                        out.ctypes.data, _stream_handle(stream)))
    del keep
    return out


def batch_serde_verify(messages: Sequence, received: Sequence[int], stream=None):
    """Returns (ok bool[n], n_bad): the receive-side check of every message."""
    descs, keep = _desc_array(messages, ChecksumType.CRC32C, 0)
    n = len(descs)
    rec = np.ascontiguousarray(np.asarray(received, dtype=np.uint32))
    ok = np.zeros(n, dtype=np.uint8)
    bad = _u64(0)
    _check(lib.h3c_batch_serde_verify(descs.ctypes.data, n, rec.ctypes.data, ok.ctypes.data, ctypes.byref(bad),
                                      _stream_handle(stream)))
    del keep
    return ok.astype(bool), int(bad.value)


class rust_crc32c:  # noqa: N801 -- mirrors the crate path crc32c::*
    """crc32c crate 0.6.8 (Cargo.lock:399-402), std-domain values."""

    @staticmethod
    def crc32c(data, stream=None) -> int:
        return int(rust_crc32c.batch([data], stream=stream)[0])

    @staticmethod
    def crc32c_append(crc: int, data, stream=None) -> int:
        return int(rust_crc32c.batch([data], append_to=[crc], stream=stream)[0])

    @staticmethod
    def crc32c_combine(crc1: int, crc2: int, len2: int) -> int:
        return int(lib.h3c_std_crc32c_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, len2))

    @staticmethod
    def batch(items: Sequence, append_to: Optional[Sequence[int]] = None, stream=None) -> np.ndarray:
        descs, keep = _desc_array(items, ChecksumType.CRC32C, 0xFFFFFFFF)
        n = len(descs)
        out = np.zeros(n, dtype=np.uint32)
        app = None if append_to is None else np.ascontiguousarray(np.asarray(append_to, dtype=np.uint32))
        _check(lib.h3c_batch_std_crc32c(descs.ctypes.data, n, app.ctypes.data if app is not None else None,
                                        out.ctypes.data, _stream_handle(stream)))
        del keep
        return out
