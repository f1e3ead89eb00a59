"""MI355X-native batched CRC32C / CRC32 chunk-checksum engine for 3FS.

Host-side mirror of the reference's checksum surface
(``hf3fs::storage::ChecksumInfo``, src/fbs/storage/Common.h:113-201) over the
C ABI in ``include/h3c_crc.h``.  Every checksum of payload bytes is computed by
the HIP kernels in ``csrc/h3c_engine.hip`` (``_lib/libh3c_crc.so``); there is no
CPU fallback — importing this package without the built library raises.

The package directory starts with a digit, so import it with
``importlib.import_module("3fs_amd")``.
"""
from __future__ import annotations

from .engine import (  # noqa: F401
    ChecksumInfo,
    ChecksumType,
    EngineError,
    HostBuffer,
    HostFed,
    device_numa_node,
    Plan,
    StatusCode,
    batch_create,
    batch_verify,
    crc32,
    crc32_combine,
    crc32c,
    crc32c_combine,
    crc32c_shift,
    device_batch_combine,
    device_count,
    fill_splitmix,
    lib,
    lib_path,
    profile_enable,
    profile_read,
    read_results,
    update_blocks,
    update_ios,
    update_ios_dev,
    update_workspace_bytes,
    CHUNK_STATE_DTYPE,
    UPDATE_IO_DTYPE,
    UPDATE_RESULT_DTYPE,
    UPD_WRITE,
    UPD_REMOVE,
    UPD_TRUNCATE,
    UPD_EXTEND,
    UPD_COMMIT,
    UPD_EXACT,
    IO_SYNCING,
    UpdateCounters,
)

__all__ = [
    "ChecksumInfo",
    "ChecksumType",
    "EngineError",
    "HostBuffer",
    "HostFed",
    "device_numa_node",
    "Plan",
    "StatusCode",
    "batch_create",
    "batch_verify",
    "crc32",
    "crc32_combine",
    "crc32c",
    "crc32c_combine",
    "crc32c_shift",
    "device_batch_combine",
    "device_count",
    "fill_splitmix",
    "lib",
    "lib_path",
    "profile_enable",
    "profile_read",
    "read_results",
    "update_blocks",
    "update_ios",
    "update_ios_dev",
    "update_workspace_bytes",
    "CHUNK_STATE_DTYPE",
    "UPDATE_IO_DTYPE",
    "UPDATE_RESULT_DTYPE",
    "UPD_WRITE",
    "UPD_REMOVE",
    "UPD_TRUNCATE",
    "UPD_EXTEND",
    "UPD_COMMIT",
    "UPD_EXACT",
    "IO_SYNCING",
    "UpdateCounters",
]
