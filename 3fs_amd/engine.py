"""ctypes binding of ``include/h3c_crc.h`` plus the ``ChecksumInfo`` mirror.

Reference interface mirrored here (paths relative to the 3FS checkout):

* ``ChecksumType``            src/fbs/storage/Common.h:66-70
* ``ChecksumInfo::create``    src/fbs/storage/Common.h:146-177 (buffer and DataIterator forms)
* ``ChecksumInfo::combine``   src/fbs/storage/Common.h:179-198 (error 4080 on type mismatch)
* ``operator==``              src/fbs/storage/Common.h:200
* fmt formatter (``TYPE#~value``)  src/fbs/storage/Common.h:768-773
* ``folly::crc32c_combine``   called at src/fbs/storage/Common.h:191

Payload checksums always run on the GPU through ``libh3c_crc.so``.  The only
host arithmetic is the scalar GF(2) combine, which the reference also does on
the host (it touches no payload bytes).
"""
from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
lib_path = os.environ.get("H3C_LIB_PATH") or os.path.join(_HERE, "_lib", "libh3c_crc.so")  # env: test hook

if not os.path.exists(lib_path):
    raise ImportError(
        f"{lib_path} is missing: the HIP engine is not built (run `python -c 'import __graft_entry__ as g; g.build()'`). "
        "There is no CPU fallback."
    )

# One HIP runtime per process: torch ships its own libamdhip64.so.7 (same soname as
# /opt/rocm's).  Whichever is loaded first serves everyone, and two copies in one
# process fight over the device ("no ROCm-capable device").  Load torch's first
# when torch is present so tensors, streams and this library share it.
try:  # pragma: no cover - import side effect only
    import torch as _torch  # noqa: F401
except ImportError:
    _torch = None

lib = ctypes.CDLL(lib_path)

_u8, _u16, _u32, _u64 = ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64
_vp, _sz, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


class _Desc(ctypes.Structure):
    _fields_ = [("ptr", _vp), ("len", _u64), ("start_raw", _u32), ("type", _u8), ("mem", _u8), ("reserved", _u16)]


assert ctypes.sizeof(_Desc) == 24

DESC_DTYPE = np.dtype(
    [("ptr", "<u8"), ("len", "<u8"), ("start_raw", "<u4"), ("type", "u1"), ("mem", "u1"), ("reserved", "<u2")]
)
assert DESC_DTYPE.itemsize == 24


def _proto(name, restype, *argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


_proto("h3c_crc32c_combine", _u32, _u32, _u32, _u64)
_proto("h3c_crc32_combine", _u32, _u32, _u32, _u64)
_proto("h3c_crc32c_shift", _u32, _u32, _u64)
_proto("h3c_device_count", _int)
_proto("h3c_init", _int, _int)
_proto("h3c_last_error", ctypes.c_char_p)
_proto("h3c_batch_create", _int, _vp, _sz, _vp, _vp, _vp)
_proto("h3c_batch_verify", _int, _vp, _vp, _sz, _vp, _vp, _vp, _vp)
_proto("h3c_plan_create", _int, _vp, _sz, _int, ctypes.POINTER(_vp))
_proto("h3c_plan_run", _int, _vp, _vp, _vp, _vp, _vp, _vp)
_proto("h3c_plan_bytes", _u64, _vp)
_proto("h3c_plan_destroy", None, _vp)
_proto("h3c_batch_combine", _int, _u8, _vp, _vp, _vp, _sz, _vp, _vp)
_proto("h3c_fill_splitmix", _int, _vp, _u64, _u64, _u64, _u64, _u64, _vp)
_proto("h3c_update_workspace_bytes", _sz, _u32, _u32, _u64, _u32)
_proto("h3c_stream_release", _int, _vp)
_proto("h3c_update_blocks", _int, _u8, _vp, _u32, _u64, _u32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _sz, _vp, _vp)
_proto("h3c_update_ios", _int, _u8, _vp, _u32, _vp, _u32, _vp, _u32, _vp)
_proto("h3c_update_ios_ex", _int, _u8, _vp, _u32, _vp, _u32, _vp, _u32, _vp, _vp)
_proto("h3c_update_blocks_ex", _int, _u8, _vp, _u32, _u64, _u32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _sz, _vp,
       _u32, _vp, _vp)
_proto("h3c_test_hook", _int, _int, _u64)
_proto("h3c_set_coalescing", _int, _int)
_proto("h3c_diag_counter", _u64, _int)
_proto("h3c_diag_last_graph", _int, _vp)
_proto("h3c_diag_last_graph_audit", _int, _vp)
_proto("h3c_diag_host_trace", _int, _vp, _int)
_proto("h3c_diag_sync_bench", _int, _int, _u64, _int, _int, _vp, _vp)
_proto("h3c_update_ios_dev", _int, _u8, _vp, _u32, _vp, _u32, _vp, _u32, _vp, _vp)
_proto("h3c_serde_checksum_mark", _u32, _u32, _int)
_proto("h3c_batch_serde_checksum", _int, _vp, _sz, _vp, _vp, _vp)
_proto("h3c_batch_serde_verify", _int, _vp, _sz, _vp, _vp, _vp, _vp)
_proto("h3c_std_crc32c_combine", _u32, _u32, _u32, _u64)
_proto("h3c_batch_std_crc32c", _int, _vp, _sz, _vp, _vp, _vp)
_proto("h3c_checksum_combine", _int, ctypes.POINTER(_u8), ctypes.POINTER(_u32), _u8, _u32, _u64)
_proto("h3c_combine_fold", _int, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp)
_proto("h3c_batch_read_result", _int, _u8, _vp, _sz, _vp, _vp, _vp, _vp)
_proto("h3c_batch_read_result_ex", _int, _u8, _vp, _sz, _vp, _vp, _vp, _vp, _vp)
_proto("h3c_crc32c", _int, _vp, _sz, _u32, ctypes.POINTER(_u32), _vp)
_proto("h3c_folly_crc32c", _u32, _vp, _sz, _u32)
_proto("h3c_folly_crc32", _u32, _vp, _sz, _u32)
_proto("h3c_crc32", _int, _vp, _sz, _u32, ctypes.POINTER(_u32), _vp)
_proto("h3c_hostfed_create", _int, _int, _u64, ctypes.POINTER(_vp))
_proto("h3c_hostfed_run", _int, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp)
_proto("h3c_hostfed_destroy", None, _vp)
_proto("h3c_host_alloc", _int, _int, _u64, ctypes.POINTER(_vp), ctypes.POINTER(_int))
_proto("h3c_host_free", _int, _vp)
_proto("h3c_device_numa_node", _int, _int)
_proto("h3c_multi_partition", _int, _vp, _sz, _int, _vp)
_proto("h3c_multi_create", _int, _vp, _int, _u64, ctypes.POINTER(_vp))
_proto("h3c_multi_destroy", None, _vp)
_proto("h3c_multi_workers", _int, _vp)
_proto("h3c_multi_batch_create", _int, _vp, _vp, _sz, _vp, _vp)
_proto("h3c_multi_verify", _int, _vp, _vp, _sz, _vp, _vp, _vp, _vp)
_proto("h3c_multi_update_ios", _int, _vp, _u8, _vp, _u32, _vp, _u32, _vp, _u32, _vp)
_proto("h3c_multi_plan_create", _int, _vp, _vp, _sz, ctypes.POINTER(_vp))
_proto("h3c_multi_plan_verify", _int, _vp, _vp, _vp, _vp, _vp)
_proto("h3c_multi_plan_destroy", None, _vp)
_proto("h3c_multi_last_stats", _int, _vp, _vp, _vp, _vp)
_proto("h3c_profile_enable", None, _int)
_proto("h3c_profile_read", _int, _int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_u64), ctypes.POINTER(_u64),
       _int)

PROF_SEG, PROF_UPDATE, PROF_HOSTFED, PROF_UPDIO = 0, 1, 2, 3


class ChecksumType(enum.IntEnum):
    """``enum class ChecksumType : uint8_t`` (Common.h:66-70)."""

    NONE = 0
    CRC32C = 1
    CRC32 = 2


class StatusCode(enum.IntEnum):
    OK = 0
    kInvalidArg = 3
    kChunkReadFailed = 4010  # StatusCodeDetails.h:160
    kChunkSizeMismatch = 4015  # StatusCodeDetails.h:165
    kChecksumMismatch = 4080  # StatusCodeDetails.h:186
    kHipError = 9001
    kNoDevice = 9002


class MemKind(enum.IntEnum):
    DEVICE = 0
    HOST_PINNED = 1
    HOST_PAGEABLE = 2


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = int(code)
        detail = msg or (lib.h3c_last_error() or b"").decode(errors="replace")
        try:
            name = StatusCode(self.code).name
        except ValueError:
            name = str(self.code)
        super().__init__(f"h3c error {name}: {detail}")


def _check(rc: int) -> None:
    if rc != 0:
        raise EngineError(rc)


def _stream_handle(stream) -> int:
    if stream is None:
        try:
            import torch

            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except ImportError:  # pragma: no cover
            pass
        return 0
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


# ---------------------------------------------------------------- scalar host arithmetic


def crc32c_combine(c1: int, c2: int, len2: int) -> int:
    """``folly::crc32c_combine`` (Common.h:191)."""
    return lib.h3c_crc32c_combine(c1 & 0xFFFFFFFF, c2 & 0xFFFFFFFF, len2)


def crc32_combine(c1: int, c2: int, len2: int) -> int:
    """``folly::crc32_combine`` (Common.h:195)."""
    return lib.h3c_crc32_combine(c1 & 0xFFFFFFFF, c2 & 0xFFFFFFFF, len2)


def crc32c(data, start: int = 0xFFFFFFFF, stream=None) -> int:
    """``folly::crc32c(data, n, start)`` (raw register) computed on the GPU (h3c_crc32c)."""
    ptr, nbytes, _, keep = _payload(data, None)
    out = _u32(0)
    _check(lib.h3c_crc32c(ptr or None, nbytes, start & 0xFFFFFFFF, ctypes.byref(out), _stream_handle(stream)))
    del keep
    return int(out.value)


def crc32(data, start: int = 0xFFFFFFFF, stream=None) -> int:
    """``folly::crc32(data, n, start)`` (raw register, IEEE polynomial) on the GPU."""
    ptr, nbytes, _, keep = _payload(data, None)
    out = _u32(0)
    _check(lib.h3c_crc32(ptr or None, nbytes, start & 0xFFFFFFFF, ctypes.byref(out), _stream_handle(stream)))
    del keep
    return int(out.value)


def crc32c_shift(crc: int, nbytes: int) -> int:
    return lib.h3c_crc32c_shift(crc & 0xFFFFFFFF, nbytes)


def device_count() -> int:
    return lib.h3c_device_count()


# ---------------------------------------------------------------- payload adapters


def _payload(data, length: Optional[int]):
    """Return (ptr, nbytes, mem, keepalive) for a payload object."""
    if data is None:
        return 0, (length or 0), MemKind.HOST_PAGEABLE, None
    try:
        import torch
    except ImportError:  # pragma: no cover
        torch = None
    if torch is not None and isinstance(data, torch.Tensor):
        if not data.is_contiguous():
            raise ValueError("payload tensor must be contiguous")
        nbytes = data.numel() * data.element_size()
        if data.is_cuda:
            mem = MemKind.DEVICE
        else:
            mem = MemKind.HOST_PINNED if data.is_pinned() else MemKind.HOST_PAGEABLE
        return data.data_ptr(), nbytes, mem, data
    if isinstance(data, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(data, dtype=np.uint8)
        return arr.ctypes.data if arr.size else 0, arr.size, MemKind.HOST_PAGEABLE, (data, arr)
    if isinstance(data, np.ndarray):
        arr = np.ascontiguousarray(data)
        ptr = arr.ctypes.data if arr.size else 0
        mem = MemKind.HOST_PINNED if _in_host_buffer(ptr, arr.nbytes) else MemKind.HOST_PAGEABLE
        return ptr, arr.nbytes, mem, arr
    raise TypeError(f"unsupported payload type {type(data)!r}")


def _desc_array(items: Sequence, type_: int, start: int):
    descs = np.zeros(len(items), dtype=DESC_DTYPE)
    keep = []
    for i, it in enumerate(items):
        if isinstance(it, tuple):
            data, length = it[0], it[1]
            st = it[2] if len(it) > 2 else start
            ty = it[3] if len(it) > 3 else type_
        else:
            data, length, st, ty = it, None, start, type_
        ptr, nbytes, mem, ka = _payload(data, length)
        if length is not None:
            if data is not None and length > nbytes:
                raise ValueError(f"length {length} exceeds payload size {nbytes}")
            nbytes = length
        keep.append(ka)
        descs[i] = (ptr, nbytes, st & 0xFFFFFFFF, int(ty), int(mem), 0)
    return descs, keep


# ---------------------------------------------------------------- batch API


def batch_create(items: Sequence, type_: int = ChecksumType.CRC32C, start: int = 0xFFFFFFFF, stream=None):
    """ChecksumInfo::create over every item; returns (types uint8[n], raw uint32[n])."""
    descs, keep = _desc_array(items, type_, start)
    n = len(descs)
    out_t = np.zeros(n, dtype=np.uint8)
    out_v = np.zeros(n, dtype=np.uint32)
    _check(lib.h3c_batch_create(descs.ctypes.data, n, out_t.ctypes.data, out_v.ctypes.data, _stream_handle(stream)))
    del keep
    return out_t, out_v


def batch_verify(items: Sequence, expected: Sequence[int], type_: int = ChecksumType.CRC32C,
                 start: int = 0xFFFFFFFF, stream=None):
    """Recompute and compare; returns (raw uint32[n], ok bool[n], n_mismatch)."""
    descs, keep = _desc_array(items, type_, start)
    n = len(descs)
    exp = np.ascontiguousarray(np.asarray(expected, dtype=np.uint32))
    if exp.size != n:
        raise ValueError("expected must have one entry per item")
    out_v = np.zeros(n, dtype=np.uint32)
    ok = np.zeros(n, dtype=np.uint8)
    mis = _u64(0)
    _check(lib.h3c_batch_verify(descs.ctypes.data, exp.ctypes.data, n, out_v.ctypes.data, ok.ctypes.data,
                                ctypes.addressof(mis), _stream_handle(stream)))
    del keep
    return out_v, ok.astype(bool), int(mis.value)


def device_batch_combine(c1, c2, len2, out, type_: int = ChecksumType.CRC32C, stream=None) -> None:
    """out[i] = folly::crc32c_combine(c1[i], c2[i], len2[i]) on device (torch cuda tensors)."""
    n = c1.numel()
    _check(lib.h3c_batch_combine(int(type_), c1.data_ptr(), c2.data_ptr(), len2.data_ptr(), n, out.data_ptr(),
                                 _stream_handle(stream)))


def fill_splitmix(base, chunk_len: int, nchunks: int, stride: int, seed: int, first_chunk: int = 0,
                  stream=None) -> None:
    """Bench/test utility: the same splitmix64 chunk generator as the oracle, written in HBM."""
    ptr = base if isinstance(base, int) else base.data_ptr()
    _check(lib.h3c_fill_splitmix(ptr, chunk_len, nchunks, stride, seed, first_chunk, _stream_handle(stream)))


def update_workspace_bytes(n_blocks: int, nchunks: int, chunk_len: int, block_bytes: int = 4096) -> int:
    return int(lib.h3c_update_workspace_bytes(n_blocks, nchunks, chunk_len, block_bytes))


def update_blocks(chunk_bases, chunk_len: int, raw_in, blk_chunk, blk_index, payload, out_raw, raw_out,
                  block_bytes: int = 4096, workspace=None, n_invalid=None, type_: int = ChecksumType.CRC32C,
                  stream=None, exact: bool = False, counters=None) -> None:
    """Batched ChunkReplica::update + updateChecksum for block-aligned overwrites (h3c_update_blocks).

    All tensors are on the GPU: chunk_bases int64[nchunks] (device addresses), raw_in /
    raw_out int32[nchunks], blk_chunk / blk_index int32[n], payload uint8[n*block_bytes],
    out_raw int32[n] (chunk checksum right after each block write).  `exact` recomputes the
    chunks' checksums from their bytes first (H3C_UPD_EXACT); `counters` (int64[8] on the GPU,
    UpdateCounters order) receives the batch's case counts (h3c_update_blocks_ex)."""
    import torch

    n, nchunks = blk_chunk.numel(), chunk_bases.numel()
    ws_bytes = update_workspace_bytes(n, nchunks, chunk_len, block_bytes)
    if workspace is None:
        workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=payload.device)
    if counters is not None and (not counters.is_cuda or counters.numel() * counters.element_size() != 64):
        raise ValueError("counters must be a GPU tensor of 8 x 64-bit")
    _check(lib.h3c_update_blocks_ex(int(type_), chunk_bases.data_ptr(), nchunks, chunk_len, block_bytes,
                                    raw_in.data_ptr(), blk_chunk.data_ptr(), blk_index.data_ptr(), payload.data_ptr(),
                                    n, out_raw.data_ptr(), raw_out.data_ptr(), workspace.data_ptr(),
                                    workspace.numel() * workspace.element_size(),
                                    n_invalid.data_ptr() if n_invalid is not None else None,
                                    UPD_EXACT if exact else 0,
                                    counters.data_ptr() if counters is not None else None, _stream_handle(stream)))


def stream_release(stream) -> None:
    """h3c_stream_release: free the update scratch the library keeps for `stream` (call before the stream
    is destroyed; its handle value may be reused by a new stream)."""
    _check(lib.h3c_stream_release(_stream_handle(stream)))


def set_coalescing(on: bool) -> None:
    """h3c_set_coalescing: merge concurrent synchronous default-stream calls into one launch."""
    _check(lib.h3c_set_coalescing(1 if on else 0))


def sync_bench(threads: int, nbytes: int, calls: int, api: str = "verify"):
    """h3c_diag_sync_bench: per-call latencies (us, threads x calls) and the wall time (s) of
    `threads` host threads each calling the synchronous API on their own pinned buffer."""
    lat = np.zeros(threads * calls, dtype=np.float64)
    wall = ctypes.c_double(0)
    _check(lib.h3c_diag_sync_bench(threads, nbytes, calls, 0 if api == "verify" else 1, lat.ctypes.data,
                                   ctypes.byref(wall)))
    return lat, wall.value


HOOK_SEG_BYTES, HOOK_DEBUG_FLAGS, HOOK_UPD_SCAN, HOOK_UPD_GRAPHS, HOOK_UPD_LOOKBACK, HOOK_UPD_FRONT = 1, 2, 3, 4, 5, 6
HOOK_UPD_FAST, HOOK_UPD_GIVEUP, HOOK_FAST_POLL_US, HOOK_UPD_ALIGNED = 7, 8, 9, 10
UPD_SCAN_PATHS = {"default": 0, "fused": 1, "tiles": 2, "sort": 3}

# h3c_diag_counter indices (include/h3c_crc.h): process-wide, monotonic
DIAG_NAMES = ("graph_replays", "graph_captures", "graph_capture_failures", "redo_front_void", "rerun_phase_b_void",
              "redo_failed_a6", "redo_short_fragment_guess", "fast_batches", "fast_abandoned", "fast_recovered",
              "graph_topology_refused", "graph_pointer_refused", "aligned_batches", "aligned_abandoned",
              "aligned_recovered")


def diag_counter(which: int) -> int:
    """h3c_diag_counter(which): see DIAG_NAMES (0 UpdateIO graph replays, 1 captures, ...)."""
    return int(lib.h3c_diag_counter(int(which)))


def diag_last_graph() -> dict:
    """h3c_diag_last_graph: the shape of the last UpdateIO graph this thread captured."""
    out = (ctypes.c_uint64 * 7)()
    _check(lib.h3c_diag_last_graph(ctypes.cast(out, ctypes.c_void_p)))
    return dict(zip(("nodes", "roots", "copies", "kernels", "reachable", "edges", "max_out"), map(int, out)))


def diag_last_graph_audit() -> dict:
    """h3c_diag_last_graph_audit: the pointer audit of the last UpdateIO graph this thread captured."""
    out = (ctypes.c_uint64 * 4)()
    _check(lib.h3c_diag_last_graph_audit(ctypes.cast(out, ctypes.c_void_p)))
    return dict(zip(("kernels", "pointers", "outside", "unknown"), map(int, out)))


def diag_host_trace(reset: bool = False) -> dict:
    """h3c_diag_host_trace: this thread's mean host microseconds per h3c_update_ios_dev call, by phase."""
    out = (ctypes.c_uint64 * 6)()
    _check(lib.h3c_diag_host_trace(ctypes.cast(out, ctypes.c_void_p), int(reset)))
    n = max(int(out[5]), 1)
    names = ("caller", "to_launch", "launches", "to_outcome", "to_return")
    return {**{k: round(int(v) / n / 1e3, 2) for k, v in zip(names, out)}, "calls": int(out[5])}


def diag_counters() -> dict:
    """Every h3c_diag_counter by name."""
    return {name: diag_counter(k) for k, name in enumerate(DIAG_NAMES)}


def set_test_hook(key: int, value: int) -> None:
    """h3c_test_hook: force an internal path for tests (0 restores the default)."""
    _check(lib.h3c_test_hook(int(key), int(value)))


# ---------------------------------------------------------------- general updates (h3c_update_ios)

UPD_WRITE, UPD_REMOVE, UPD_TRUNCATE, UPD_EXTEND, UPD_COMMIT = 1, 2, 4, 8, 16  # UpdateType (Common.h:51-58)
UPD_STD_DOMAIN = 1  # flag: Rust chunk engine semantics (std-domain values)
UPD_EXACT = 2  # flag: stored checksums are not trusted (each chunk CRC'd once first)
UPD_GRAPHS = 4  # flag: a repeated batch shape may run as one captured HIP graph (caller: no concurrent
#                 legacy-default-stream launches in the process during the call)
IO_SYNCING = 1  # per-op flag: UpdateOptions.isSyncing full-chunk replace
IO_CHUNK_SIZE = 2  # per-op flag: `chunk_size` carries UpdateIO.chunkSize (range check, kChunkSizeMismatch)

CHUNK_STATE_DTYPE = np.dtype([("base", "<u8"), ("chunk_size", "<u4"), ("size", "<u4"), ("value", "<u4"),
                              ("type", "u1"), ("reserved", "u1", 3)])
UPDATE_IO_DTYPE = np.dtype([("payload", "<u8"), ("chunk", "<u4"), ("offset", "<u4"), ("length", "<u4"),
                            ("checksum_value", "<u4"), ("checksum_type", "u1"), ("kind", "u1"), ("flags", "u1"),
                            ("reserved", "u1"), ("chunk_size", "<u4")])
UPDATE_RESULT_DTYPE = np.dtype([("status", "<u4"), ("size", "<u4"), ("value", "<u4"), ("type", "u1"),
                                ("reserved", "u1", 3)])
assert CHUNK_STATE_DTYPE.itemsize == 24 and UPDATE_IO_DTYPE.itemsize == 32 and UPDATE_RESULT_DTYPE.itemsize == 16


class UpdateCounters(ctypes.Structure):
    """h3c_update_counters: the reference's checksum case counters for one batch
    (ChunkReplica.cc:25-28, StorageTarget.cc:331-332; Rust metrics.rs:12-14)."""

    _fields_ = [(f, _u64) for f in ("none", "reuse", "combine", "read_chunk", "recalculate", "checksum_mismatch",
                                    "invalid", "stale_chunks")]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


def update_ios(chunks: np.ndarray, ios: np.ndarray, type_: int = ChecksumType.CRC32C, std_domain: bool = False,
               exact: bool = False, counters: Optional[UpdateCounters] = None, stream=None,
               out: Optional[np.ndarray] = None, graphs: bool = False) -> np.ndarray:
    """Batched ChunkReplica::update + updateChecksum for any mix of WRITE / REMOVE / TRUNCATE /
    EXTEND / COMMIT (h3c_update_ios_ex).  `chunks` (CHUNK_STATE_DTYPE, updated in place: size /
    type / value) and `ios` (UPDATE_IO_DTYPE) are host arrays whose `base` / `payload` fields are
    device addresses.  Returns one UPDATE_RESULT_DTYPE record per op: status 0 / 3 kInvalidArg /
    4080 kChecksumMismatch, chunk size after, and result.checksum (type, value).  `exact` does not
    trust stored checksums (H3C_UPD_EXACT); `counters` receives the batch's case counts; `out`
    (UPDATE_RESULT_DTYPE, len(ios)) receives the results instead of a new array (pass a pinned
    one to skip the runtime's staging copy).  `graphs` (H3C_UPD_GRAPHS): a repeated batch shape
    may replay as one HIP graph -- only when no other thread launches on the legacy default
    stream meanwhile."""
    if chunks.dtype != CHUNK_STATE_DTYPE or ios.dtype != UPDATE_IO_DTYPE:
        raise TypeError("chunks / ios must use CHUNK_STATE_DTYPE / UPDATE_IO_DTYPE")
    if not (chunks.flags.c_contiguous and ios.flags.c_contiguous):
        raise ValueError("chunks / ios must be contiguous")
    if out is not None:
        if out.dtype != UPDATE_RESULT_DTYPE or len(out) != len(ios) or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous UPDATE_RESULT_DTYPE array with one record per op")
        res = out
    else:
        res = np.zeros(len(ios), dtype=UPDATE_RESULT_DTYPE)
    flags = (UPD_STD_DOMAIN if std_domain else 0) | (UPD_EXACT if exact else 0) | (UPD_GRAPHS if graphs else 0)
    _check(lib.h3c_update_ios_ex(int(type_), chunks.ctypes.data, len(chunks), ios.ctypes.data, len(ios),
                                 res.ctypes.data, flags, ctypes.byref(counters) if counters is not None else None,
                                 _stream_handle(stream)))
    return res


def update_ios_dev(chunks, ios, results, type_: int = ChecksumType.CRC32C, std_domain: bool = False,
                   exact: bool = False, counters=None, stream=None, graphs: bool = False) -> None:
    """update_ios with every table on the GPU (h3c_update_ios_dev): `chunks` uint8 tensor of
    nchunks x 24 bytes (CHUNK_STATE_DTYPE records, updated in place), `ios` uint8 tensor of
    n x 32 bytes (UPDATE_IO_DTYPE), `results` uint8 tensor of n x 16 bytes (UPDATE_RESULT_DTYPE),
    `counters` an int64 tensor of 8 (UpdateCounters order) or None.  No PCIe traffic; synchronous
    on `stream`."""
    for t, rec in ((chunks, CHUNK_STATE_DTYPE), (ios, UPDATE_IO_DTYPE), (results, UPDATE_RESULT_DTYPE)):
        if not t.is_cuda or not t.is_contiguous() or (t.numel() * t.element_size()) % rec.itemsize:
            raise ValueError("chunks / ios / results must be contiguous GPU tensors of whole records")
    nchunks = chunks.numel() * chunks.element_size() // CHUNK_STATE_DTYPE.itemsize
    n = ios.numel() * ios.element_size() // UPDATE_IO_DTYPE.itemsize
    if results.numel() * results.element_size() != n * UPDATE_RESULT_DTYPE.itemsize:
        raise ValueError("results must hold one record per op")
    if counters is not None and (not counters.is_cuda or counters.numel() * counters.element_size() != 64):
        raise ValueError("counters must be a GPU tensor of 8 x 64-bit")
    flags = (UPD_STD_DOMAIN if std_domain else 0) | (UPD_EXACT if exact else 0) | (UPD_GRAPHS if graphs else 0)
    _check(lib.h3c_update_ios_dev(int(type_), chunks.data_ptr(), nchunks, ios.data_ptr(), n, results.data_ptr(),
                                  flags, counters.data_ptr() if counters is not None else None,
                                  _stream_handle(stream)))


class UpdateIosDev:
    """update_ios_dev bound once to its tables: the checks and pointers of the first call are kept and
    run() makes only the C call (h3c_update_ios_dev), as a C++ caller repeating a batch on the same
    buffers does.  The tensors must stay alive and in place while the object is used."""

    def __init__(self, chunks, ios, results, type_: int = ChecksumType.CRC32C, std_domain: bool = False,
                 exact: bool = False, counters=None, stream=None, graphs: bool = False):
        for t, rec in ((chunks, CHUNK_STATE_DTYPE), (ios, UPDATE_IO_DTYPE), (results, UPDATE_RESULT_DTYPE)):
            if not t.is_cuda or not t.is_contiguous() or (t.numel() * t.element_size()) % rec.itemsize:
                raise ValueError("chunks / ios / results must be contiguous GPU tensors of whole records")
        n = ios.numel() * ios.element_size() // UPDATE_IO_DTYPE.itemsize
        if results.numel() * results.element_size() != n * UPDATE_RESULT_DTYPE.itemsize:
            raise ValueError("results must hold one record per op")
        if counters is not None and (not counters.is_cuda or counters.numel() * counters.element_size() != 64):
            raise ValueError("counters must be a GPU tensor of 8 x 64-bit")
        flags = (UPD_STD_DOMAIN if std_domain else 0) | (UPD_EXACT if exact else 0) | (UPD_GRAPHS if graphs else 0)
        self._keep = (chunks, ios, results, counters)
        self._args = (int(type_), chunks.data_ptr(), chunks.numel() * chunks.element_size() // CHUNK_STATE_DTYPE.itemsize,
                      ios.data_ptr(), n, results.data_ptr(), flags,
                      counters.data_ptr() if counters is not None else None, _stream_handle(stream))

    def run(self) -> None:
        _check(lib.h3c_update_ios_dev(*self._args))


READ_JOB_DTYPE = np.dtype([("data", "<u8"), ("length", "<u8"), ("chunk_len", "<u8"), ("offset", "<u4"),
                           ("chunk_value", "<u4"), ("chunk_type", "u1"), ("mem", "u1"), ("recalculate", "u1"),
                           ("reserved", "u1", 5)])
assert READ_JOB_DTYPE.itemsize == 40


def read_results(batch_type: int, jobs: Sequence, stream=None, counters: Optional[dict] = None):
    """AioReadJob::setResult (BatchReadJob.cc:24-55) for a batch of completed reads.

    jobs[i] = (data, length, chunk_len, offset, stored ChecksumInfo, recalculate).  Returns
    (list of result ChecksumInfo, status uint32[n]: 0 or 4080 from the recalculate check).
    `counters` (a dict) receives "checksum_mismatch": the reference's
    storage.aio.checksum_mismatch count for the batch (BatchReadJob.cc:14)."""
    arr = np.zeros(len(jobs), dtype=READ_JOB_DTYPE)
    keep = []
    for i, (data, length, chunk_len, offset, ck, recalc) in enumerate(jobs):
        ptr, nbytes, mem, ka = _payload(data, length)
        if data is not None and length > nbytes:
            raise ValueError("length exceeds the read buffer")
        keep.append(ka)
        arr[i] = (ptr, length, chunk_len, offset, ck.value & 0xFFFFFFFF, int(ck.type), int(mem), int(bool(recalc)), 0)
    n = len(arr)
    ot = np.zeros(n, dtype=np.uint8)
    ov = np.zeros(n, dtype=np.uint32)
    st = np.zeros(n, dtype=np.uint32)
    mis = _u64(0)
    _check(lib.h3c_batch_read_result_ex(int(batch_type), arr.ctypes.data, n, ot.ctypes.data, ov.ctypes.data,
                                        st.ctypes.data, ctypes.byref(mis), _stream_handle(stream)))
    if counters is not None:
        counters["checksum_mismatch"] = int(mis.value)
    del keep
    return [ChecksumInfo(ChecksumType(int(a)), int(b)) for a, b in zip(ot, ov)], st


def profile_enable(on: bool = True) -> None:
    lib.h3c_profile_enable(1 if on else 0)


def profile_read(reset: bool = False, kind: int = PROF_SEG) -> Tuple[float, int, int]:
    """(summed ms, launches, algorithmic bytes) of the profiled launches of `kind`."""
    ms, launches, nbytes = ctypes.c_double(0), _u64(0), _u64(0)
    _check(lib.h3c_profile_read(kind, ctypes.byref(ms), ctypes.byref(launches), ctypes.byref(nbytes),
                                1 if reset else 0))
    return ms.value, int(launches.value), int(nbytes.value)


class Plan:
    """Device-resident descriptor set reused across create/verify runs (scrub, resync)."""

    def __init__(self, descs: np.ndarray, device: int):
        self._h = _vp()
        self.n = len(descs)
        self.device = device
        self._descs = descs
        _check(lib.h3c_plan_create(descs.ctypes.data, self.n, device, ctypes.byref(self._h)))
        self.bytes = int(lib.h3c_plan_bytes(self._h))

    @classmethod
    def uniform(cls, base_ptr, chunk_len: int, nchunks: int, stride: Optional[int] = None,
                start: int = 0xFFFFFFFF, type_: int = ChecksumType.CRC32C, device: int = 0,
                extent: Optional[int] = None) -> "Plan":
        """Chunk i = [base + i*stride, + chunk_len).  `base_ptr` is a device address or a GPU
        tensor; the bytes the plan may read end at base + `extent` (default: the tensor's size
        when a tensor is given).  A layout that runs past it, stride*(n-1) + chunk_len > extent,
        is rejected with kInvalidArg before anything is uploaded or launched; the library also
        rejects descriptors that run past their HIP allocation (h3c_plan_create)."""
        if not isinstance(base_ptr, int):  # a tensor: its own extent bounds the plan
            if extent is None:
                extent = base_ptr.numel() * base_ptr.element_size()
            base_ptr = base_ptr.data_ptr()
        stride = chunk_len if stride is None else stride
        if chunk_len < 0 or stride < 0 or nchunks < 0:
            raise EngineError(StatusCode.kInvalidArg, "negative plan geometry")
        need = stride * (nchunks - 1) + chunk_len if nchunks else 0
        if extent is not None and need > extent:
            raise EngineError(StatusCode.kInvalidArg,
                              f"uniform plan reads {need} bytes (stride {stride} x {nchunks - 1} + {chunk_len}) "
                              f"past an extent of {extent}")
        d = np.zeros(nchunks, dtype=DESC_DTYPE)
        d["ptr"] = base_ptr + np.arange(nchunks, dtype=np.uint64) * np.uint64(stride)
        d["len"] = chunk_len
        d["start_raw"] = start & 0xFFFFFFFF
        d["type"] = int(type_)
        d["mem"] = int(MemKind.DEVICE)
        return cls(d, device)

    def run(self, out_raw, expected=None, ok=None, mismatch=None, stream=None) -> None:
        _check(lib.h3c_plan_run(
            self._h,
            expected.data_ptr() if expected is not None else None,
            out_raw.data_ptr(),
            ok.data_ptr() if ok is not None else None,
            mismatch.data_ptr() if mismatch is not None else None,
            _stream_handle(stream),
        ))

    def close(self) -> None:
        if self._h:
            lib.h3c_plan_destroy(self._h)
            self._h = _vp()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_host_ranges = {}  # HostBuffer address -> size (numpy views into them are pinned payloads)


def _in_host_buffer(ptr: int, nbytes: int) -> bool:
    return any(a <= ptr and ptr + nbytes <= a + n for a, n in _host_ranges.items())


def device_numa_node(device: int = 0) -> int:
    """NUMA node of the GPU's PCIe root (h3c_device_numa_node), -1 when unknown."""
    return lib.h3c_device_numa_node(device)


class HostBuffer:
    """Pinned host memory on the GPU's NUMA node (h3c_host_alloc): the host-fed analogue
    of the storage service's RDMA BufferPool.  `array` is a uint8 numpy view; slices of it
    are passed as pinned payloads."""

    def __init__(self, device: int, nbytes: int):
        p, node = _vp(), _int(-1)
        _check(lib.h3c_host_alloc(device, nbytes, ctypes.byref(p), ctypes.byref(node)))
        self.ptr, self.nbytes, self.node = int(p.value), int(nbytes), int(node.value)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.ptr))
        _host_ranges[self.ptr] = self.nbytes

    def close(self) -> None:
        if self.ptr:
            _host_ranges.pop(self.ptr, None)
            self.array = None
            _check(lib.h3c_host_free(self.ptr))
            self.ptr = 0


class HostFed:
    """Host-fed pipeline (h3c_hostfed_*): payloads in (pinned) host memory, H2D copies
    double-buffered against the CRC kernels."""

    def __init__(self, device: int = 0, window_bytes: int = 64 << 20):
        self._h = _vp()
        self.device = device
        _check(lib.h3c_hostfed_create(device, window_bytes, ctypes.byref(self._h)))

    def run(self, items: Sequence, expected: Optional[Sequence[int]] = None, type_: int = ChecksumType.CRC32C,
            start: int = 0xFFFFFFFF, stream=None):
        """Returns raw uint32[n] (create), or (raw, ok bool[n], n_mismatch) with `expected`."""
        descs, keep = _desc_array(items, type_, start)
        n = len(descs)
        out = np.zeros(n, dtype=np.uint32)
        if expected is None:
            _check(lib.h3c_hostfed_run(self._h, descs.ctypes.data, n, None, out.ctypes.data, None, None,
                                       _stream_handle(stream)))
            return out
        exp = np.ascontiguousarray(np.asarray(expected, dtype=np.uint32))
        ok = np.zeros(n, dtype=np.uint8)
        mis = _u64(0)
        _check(lib.h3c_hostfed_run(self._h, descs.ctypes.data, n, exp.ctypes.data, out.ctypes.data, ok.ctypes.data,
                                   ctypes.addressof(mis), _stream_handle(stream)))
        del keep
        return out, ok.astype(bool), int(mis.value)

    def close(self) -> None:
        if self._h:
            lib.h3c_hostfed_destroy(self._h)
            self._h = _vp()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- several GPUs, one process (h3c_multi_*)


def multi_partition(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """h3c_multi_partition: the C++ byte-balanced split the multi-GPU engine uses, as [lo, hi) ranges
    (identical to 3fs_amd/shard.py::partition).  Host arithmetic only: needs no GPU."""
    ln = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint64))
    cuts = np.zeros(world + 1 if world >= 1 else 1, dtype=np.uint64)
    _check(lib.h3c_multi_partition(ln.ctypes.data if ln.size else None, ln.size, int(world), cuts.ctypes.data))
    return [(int(cuts[k]), int(cuts[k + 1])) for k in range(world)]


class Multi:
    """One engine over several GPUs of this process (h3c_multi_*): a host worker thread per entry of
    `devices` (a device may repeat), each batch split byte-balanced (updates by chunk) and run on every
    worker at once, results in the caller's arrays.  Device payloads must live on a listed device."""

    def __init__(self, devices: Sequence[int], hostfed_window: int = 0):
        devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
        self._h = _vp()
        self.devices = [int(d) for d in devs]
        _check(lib.h3c_multi_create(devs.ctypes.data, len(devs), int(hostfed_window), ctypes.byref(self._h)))

    def _descs(self, items, type_, start):
        if isinstance(items, np.ndarray) and items.dtype == DESC_DTYPE:
            return np.ascontiguousarray(items), None
        return _desc_array(items, type_, start)

    def batch_create(self, items, type_: int = ChecksumType.CRC32C, start: int = 0xFFFFFFFF):
        """ChecksumInfo::create over every item (or a DESC_DTYPE array): (types uint8[n], raw uint32[n])."""
        descs, keep = self._descs(items, type_, start)
        n = len(descs)
        out_t, out_v = np.zeros(n, dtype=np.uint8), np.zeros(n, dtype=np.uint32)
        _check(lib.h3c_multi_batch_create(self._h, descs.ctypes.data, n, out_t.ctypes.data, out_v.ctypes.data))
        del keep
        return out_t, out_v

    def verify(self, items, expected, type_: int = ChecksumType.CRC32C, start: int = 0xFFFFFFFF):
        """(raw uint32[n], ok bool[n], n_mismatch) as batch_verify, over every worker."""
        descs, keep = self._descs(items, type_, start)
        n = len(descs)
        exp = np.ascontiguousarray(np.asarray(expected, dtype=np.uint32))
        if exp.size != n:
            raise ValueError("expected must have one entry per item")
        out_v, ok, mis = np.zeros(n, dtype=np.uint32), np.zeros(n, dtype=np.uint8), _u64(0)
        _check(lib.h3c_multi_verify(self._h, descs.ctypes.data, n, exp.ctypes.data, out_v.ctypes.data,
                                    ok.ctypes.data, ctypes.byref(mis)))
        del keep
        return out_v, ok.astype(bool), int(mis.value)

    def update_ios(self, chunks: np.ndarray, ios: np.ndarray, type_: int = ChecksumType.CRC32C,
                   std_domain: bool = False, exact: bool = False, counters: Optional[UpdateCounters] = None,
                   graphs: bool = False) -> np.ndarray:
        """update_ios over every worker (h3c_multi_update_ios): chunks sharded by chunk, ops in sequence
        order per chunk; `chunks` is updated in place, one UPDATE_RESULT_DTYPE record per op returned."""
        if chunks.dtype != CHUNK_STATE_DTYPE or ios.dtype != UPDATE_IO_DTYPE:
            raise TypeError("chunks / ios must use CHUNK_STATE_DTYPE / UPDATE_IO_DTYPE")
        if not (chunks.flags.c_contiguous and ios.flags.c_contiguous):
            raise ValueError("chunks / ios must be contiguous")
        res = np.zeros(len(ios), dtype=UPDATE_RESULT_DTYPE)
        flags = (UPD_STD_DOMAIN if std_domain else 0) | (UPD_EXACT if exact else 0) | (UPD_GRAPHS if graphs else 0)
        _check(lib.h3c_multi_update_ios(self._h, int(type_), chunks.ctypes.data, len(chunks), ios.ctypes.data,
                                        len(ios), res.ctypes.data, flags,
                                        ctypes.byref(counters) if counters is not None else None))
        return res

    def plan(self, descs: np.ndarray) -> "MultiPlan":
        return MultiPlan(self, descs)

    def last_stats(self):
        """The last call's share per worker: [(units, algorithmic bytes, wall ms)]."""
        k = len(self.devices)
        u, b, ms = np.zeros(k, dtype=np.uint64), np.zeros(k, dtype=np.uint64), np.zeros(k, dtype=np.float64)
        _check(lib.h3c_multi_last_stats(self._h, u.ctypes.data, b.ctypes.data, ms.ctypes.data))
        return [(int(u[i]), int(b[i]), float(ms[i])) for i in range(k)]

    def close(self) -> None:
        if self._h:
            lib.h3c_multi_destroy(self._h)
            self._h = _vp()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class MultiPlan:
    """A resident chunk set (DESC_DTYPE, device memory on the engine's devices) verified repeatedly over
    every worker (h3c_multi_plan_*): per run only expected values and results cross PCIe, read and
    written in place by the kernels through each worker's pinned mirror."""

    def __init__(self, multi: Multi, descs: np.ndarray):
        if descs.dtype != DESC_DTYPE:
            raise TypeError("descs must use DESC_DTYPE")
        self._m = multi
        self._descs = np.ascontiguousarray(descs)
        self.n = len(descs)
        self._h = _vp()
        _check(lib.h3c_multi_plan_create(multi._h, self._descs.ctypes.data, self.n, ctypes.byref(self._h)))
        self.out = np.zeros(self.n, dtype=np.uint32)
        self.ok = np.zeros(self.n, dtype=np.uint8)

    def verify(self, expected) -> int:
        """Runs one verify; results in self.out / self.ok; returns the mismatch count."""
        exp = np.ascontiguousarray(np.asarray(expected, dtype=np.uint32))
        if exp.size != self.n:
            raise ValueError("expected must have one entry per descriptor")
        mis = _u64(0)
        _check(lib.h3c_multi_plan_verify(self._h, exp.ctypes.data, self.out.ctypes.data, self.ok.ctypes.data,
                                         ctypes.byref(mis)))
        return int(mis.value)

    def close(self) -> None:
        if self._h:
            lib.h3c_multi_plan_destroy(self._h)
            self._h = _vp()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- ChecksumInfo mirror


@dataclass
class ChecksumInfo:
    """``hf3fs::storage::ChecksumInfo`` (Common.h:113-201): {type u8, value u32 raw}."""

    type: ChecksumType = ChecksumType.NONE
    value: int = 0

    kChunkSize = 1 << 20  # Common.h:118

    @staticmethod
    def create(type_: int, data, length: Optional[int] = None, starting_checksum: int = 0xFFFFFFFF,
               stream=None) -> "ChecksumInfo":
        """Common.h:146-177: NONE -> {NONE,0}; empty -> {type, start}; null with length>0 -> {NONE,0}."""
        t, v = batch_create([(data, length, starting_checksum, int(type_))], int(type_), starting_checksum, stream)
        return ChecksumInfo(ChecksumType(int(t[0])), int(v[0]))

    @staticmethod
    def memory_data_iterator(buffer, length: int):
        """MemoryDataIterator (Common.h:126-144): (piece, size) slices of at most kChunkSize,
        then (None, 0)."""
        off = 0
        while off < length:
            size = min(length - off, ChecksumInfo.kChunkSize)
            yield buffer[off: off + size], size
            off += size
        yield None, 0

    @staticmethod
    def create_from_iterator(type_: int, pieces, length: int, starting_checksum: int = 0xFFFFFFFF,
                             stream=None) -> "ChecksumInfo":
        """ChecksumInfo::create(type, DataIterator*, length, start) (Common.h:146-172): pieces
        (data, size) are taken while data is not None and fewer than `length` bytes were taken
        (a piece is taken whole); a byte count other than `length` gives {NONE, 0}.  The
        pieces are checksummed in one GPU batch -- the first from `starting_checksum`, the
        others from 0 -- and chained with the combine shift (crc32c_combine), which equals
        the reference's sequential chain."""
        if int(type_) == ChecksumType.NONE:
            return ChecksumInfo(ChecksumType.NONE, 0)
        items, total = [], 0
        for data, size in pieces:
            if data is None or total >= length:
                break
            total += size
            if size:
                items.append((data, size, starting_checksum if not items else 0, int(type_)))
        if total != length:
            return ChecksumInfo(ChecksumType.NONE, 0)
        if not items:
            return ChecksumInfo(ChecksumType(int(type_)), starting_checksum & 0xFFFFFFFF)
        _, v = batch_create(items, int(type_), starting_checksum, stream)
        comb = lib.h3c_crc32c_combine if int(type_) == ChecksumType.CRC32C else lib.h3c_crc32_combine
        acc = int(v[0])
        for k in range(1, len(items)):
            acc = int(comb(acc, int(v[k]), items[k][1]))
        return ChecksumInfo(ChecksumType(int(type_)), acc)

    def combine(self, o: "ChecksumInfo", length: int) -> None:
        """Common.h:179-198 (h3c_checksum_combine).  Raises EngineError(kChecksumMismatch)
        on a type mismatch; length 0 is a no-op; a NONE receiver copies `o`."""
        t, v = _u8(int(self.type)), _u32(self.value & 0xFFFFFFFF)
        rc = lib.h3c_checksum_combine(ctypes.byref(t), ctypes.byref(v), int(o.type), o.value & 0xFFFFFFFF, length)
        if rc:
            raise EngineError(rc, f"different type {self} != {o}")
        self.type, self.value = ChecksumType(t.value), int(v.value)

    def serialize(self) -> bytes:
        """serde binary form (src/common/serde/Serde.h:267-290, DownwardBytes): Varint32 table
        length, then type (1 byte) and value (4 bytes, little endian); TestCommonStruct.cc:46-56
        pins the size (6) and the round trip."""
        return bytes([5, int(self.type)]) + int(self.value & 0xFFFFFFFF).to_bytes(4, "little")

    @staticmethod
    def deserialize(data: bytes) -> "ChecksumInfo":
        """Inverse of serialize; fields missing at the end of the table keep their defaults
        (Serde.h:499-507).  Raises EngineError(kInvalidArg) on a short or malformed buffer."""
        tlen, k, shift = 0, 0, 0
        while True:
            if k >= len(data) or shift > 28:
                raise EngineError(StatusCode.kInvalidArg, "serde: short varint")
            tlen |= (data[k] & 0x7F) << shift
            k += 1
            if not data[k - 1] & 0x80:
                break
            shift += 7
        if tlen > len(data) - k or 1 < tlen < 5:
            raise EngineError(StatusCode.kInvalidArg, "serde: short table")
        t = data[k: k + tlen]
        o = ChecksumInfo()
        if tlen >= 1:
            o.type = ChecksumType(t[0])
        if tlen >= 5:
            o.value = int.from_bytes(t[1:5], "little")
        return o

    def __str__(self) -> str:  # Common.h:768-773
        return f"{ChecksumType(self.type).name}#{(~self.value) & 0xFFFFFFFF:08X}"
