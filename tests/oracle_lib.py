"""ctypes access to the CPU oracle (oracle/crc_oracle.c) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load the
oracle; it is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")

NONE, CRC32C, CRC32 = 0, 1, 2
POLY_CRC32C = 0x82F63B78
POLY_CRC32 = 0xEDB88320


def load():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    L = ctypes.CDLL(ORACLE_SO)
    u8, u32, u64, vp, sz = ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t
    for f in ("orc_crc32c_bitwise", "orc_crc32c_table", "orc_crc32c_sse42", "orc_crc32c_sse42_3way",
              "orc_crc32_table"):
        getattr(L, f).restype = u32
        getattr(L, f).argtypes = [vp, sz, u32]
    L.orc_gf_mul.restype = u32
    L.orc_gf_mul.argtypes = [u32, u32, u32]
    L.orc_xpow8n.restype = u32
    L.orc_xpow8n.argtypes = [u64, u32]
    L.orc_shift.restype = u32
    L.orc_shift.argtypes = [u32, u64, u32]
    L.orc_crc32c_combine.restype = u32
    L.orc_crc32c_combine.argtypes = [u32, u32, u64]
    L.orc_crc32_combine.restype = u32
    L.orc_crc32_combine.argtypes = [u32, u32, u64]
    L.orc_checksum_create.restype = None
    L.orc_checksum_create.argtypes = [u8, vp, u64, u32, ctypes.POINTER(u8), ctypes.POINTER(u32)]
    L.orc_checksum_combine.restype = ctypes.c_int
    L.orc_checksum_combine.argtypes = [ctypes.POINTER(u8), ctypes.POINTER(u32), u8, u32, u64]
    L.orc_splitmix64.restype = u64
    L.orc_splitmix64.argtypes = [u64]
    L.orc_fill_splitmix.restype = None
    L.orc_fill_splitmix.argtypes = [vp, u64, u64, u64]
    L.orc_batch_crc32c.restype = None
    L.orc_batch_crc32c.argtypes = [vp, u64, u64, u32, ctypes.c_int, ctypes.c_int, vp]
    return L


class ChunkMeta(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("checksum_type", ctypes.c_uint8), ("checksum_value", ctypes.c_uint32)]


class WriteIO(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint32), ("length", ctypes.c_uint32), ("checksum_type", ctypes.c_uint8),
                ("checksum_value", ctypes.c_uint32), ("is_truncate_or_extend", ctypes.c_uint8)]


_L = None


def lib():
    global _L
    if _L is None:
        _L = load()
        _L.orc_update_checksum.restype = ctypes.c_int
        _L.orc_update_checksum.argtypes = [ctypes.POINTER(ChunkMeta), WriteIO, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_void_p]
    return _L


def _ptr(a: np.ndarray):
    return a.ctypes.data if a.size else None


def crc32c(data, start=0xFFFFFFFF, mech="sse42"):
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return getattr(lib(), f"orc_crc32c_{mech}")(_ptr(a), a.size, start & 0xFFFFFFFF)


def crc32(data, start=0xFFFFFFFF):
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return lib().orc_crc32_table(_ptr(a), a.size, start & 0xFFFFFFFF)


def create(type_, data, length=None, start=0xFFFFFFFF):
    """ChecksumInfo::create restatement -> (type, value)."""
    t, v = ctypes.c_uint8(0), ctypes.c_uint32(0)
    if data is None:
        lib().orc_checksum_create(type_, None, length or 0, start & 0xFFFFFFFF, ctypes.byref(t), ctypes.byref(v))
    else:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        n = a.size if length is None else length
        lib().orc_checksum_create(type_, _ptr(a), n, start & 0xFFFFFFFF, ctypes.byref(t), ctypes.byref(v))
    return t.value, v.value


def combine(t, v, ot, ov, length):
    """ChecksumInfo::combine restatement -> (rc, type, value)."""
    tt, vv = ctypes.c_uint8(t), ctypes.c_uint32(v)
    rc = lib().orc_checksum_combine(ctypes.byref(tt), ctypes.byref(vv), ot, ov & 0xFFFFFFFF, length)
    return rc, tt.value, vv.value


def splitmix_bytes(length, seed, chunk_idx):
    out = np.empty(length, dtype=np.uint8)
    lib().orc_fill_splitmix(_ptr(out), length, seed, chunk_idx)
    return out


def update_checksum(meta: dict, wio: dict, size_before: int, is_append: bool, chunk_after: np.ndarray):
    m = ChunkMeta(meta["size"], meta["type"], meta["value"])
    w = WriteIO(wio["offset"], wio["length"], wio["type"], wio["value"] & 0xFFFFFFFF, int(wio.get("trunc_ext", 0)))
    rc = lib().orc_update_checksum(ctypes.byref(m), w, size_before, int(is_append), _ptr(chunk_after))
    return rc, {"size": m.size, "type": m.checksum_type, "value": m.checksum_value}


UPD_WRITE, UPD_REMOVE, UPD_TRUNCATE, UPD_EXTEND, UPD_COMMIT = 1, 2, 4, 8, 16  # UpdateType (Common.h:51-58)
# updateChecksum branch taken (ChunkReplica.cc:25-28 counters); KEEP: Rust engine left the checksum alone
CASE_NOT_RUN, CASE_NONE, CASE_REUSE, CASE_COMBINE, CASE_READ_CHUNK, CASE_KEEP = range(6)


class UpdateIO(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint8), ("offset", ctypes.c_uint32), ("length", ctypes.c_uint32),
                ("checksum_type", ctypes.c_uint8), ("checksum_value", ctypes.c_uint32), ("syncing", ctypes.c_uint8)]


class UpdateResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int), ("size", ctypes.c_uint32), ("type", ctypes.c_uint8),
                ("value", ctypes.c_uint32), ("ucase", ctypes.c_int)]


class EngineCounters(ctypes.Structure):
    _fields_ = [("reuse", ctypes.c_uint64), ("combine", ctypes.c_uint64), ("recalculate", ctypes.c_uint64)]


def _bind_update(L):
    if not hasattr(L, "_replica_update_bound"):
        L.orc_chunk_replica_update.restype = ctypes.c_int
        L.orc_chunk_replica_update.argtypes = [ctypes.POINTER(ChunkMeta), ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.POINTER(UpdateIO), ctypes.c_void_p,
                                               ctypes.POINTER(UpdateResult)]
        L.orc_chunk_replica_update_cs.restype = ctypes.c_int
        L.orc_chunk_replica_update_cs.argtypes = [ctypes.POINTER(ChunkMeta), ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_uint32, ctypes.POINTER(UpdateIO), ctypes.c_void_p,
                                                  ctypes.POINTER(UpdateResult)]
        L.orc_chunk_engine_update.restype = ctypes.c_int
        L.orc_chunk_engine_update.argtypes = [ctypes.POINTER(ChunkMeta), ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.POINTER(UpdateIO), ctypes.c_void_p, ctypes.c_int,
                                              ctypes.POINTER(UpdateResult), ctypes.POINTER(EngineCounters)]
        L._replica_update_bound = True


def _update_args(meta, io, payload):
    m = ChunkMeta(meta["size"], meta["type"], meta["value"] & 0xFFFFFFFF)
    u = UpdateIO(io["kind"], io["offset"], io["length"], io["type"], io["value"] & 0xFFFFFFFF,
                 int(bool(io.get("syncing", 0))))
    pay = None
    if payload is not None and len(payload):
        pay = np.ascontiguousarray(payload, dtype=np.uint8)
    return m, u, pay


def replica_update(meta: dict, chunk: np.ndarray, chunk_size: int, io: dict, payload=None):
    """ChunkReplica::update restatement (A6 + A8): applies one UpdateIO to `chunk` in place.

    io = {kind, offset, length, type, value[, syncing][, chunk_size]}: `chunk_size` is the op's
    UpdateIO.chunkSize (default: the chunk's own, `chunk_size` here).  Returns (result dict with
    the updateChecksum branch in "ucase", new meta dict)."""
    L = lib()
    _bind_update(L)
    m, u, pay = _update_args(meta, io, payload)
    r = UpdateResult()
    L.orc_chunk_replica_update_cs(ctypes.byref(m), chunk.ctypes.data, chunk_size, io.get("chunk_size", chunk_size),
                                  ctypes.byref(u), pay.ctypes.data if pay is not None else None, ctypes.byref(r))
    return ({"status": r.status, "size": r.size, "type": r.type, "value": r.value, "ucase": r.ucase},
            {"size": m.size, "type": m.checksum_type, "value": m.checksum_value})


def engine_update(meta: dict, chunk: np.ndarray, chunk_size: int, io: dict, payload=None, payload_aligned=False,
                  counters: EngineCounters = None):
    """Rust chunk engine restatement (ChunkEngine.cc:15-80, engine.rs:288-429, chunk.rs:89-281):
    meta["value"] is the std-domain crc32c; results are {CRC32C, ~std} as ChunkEngine.cc:66
    reports them.  `counters` (EngineCounters) accumulates metrics.rs's checksum counters."""
    L = lib()
    _bind_update(L)
    m, u, pay = _update_args(meta, io, payload)
    r = UpdateResult()
    L.orc_chunk_engine_update(ctypes.byref(m), chunk.ctypes.data, chunk_size, ctypes.byref(u),
                              pay.ctypes.data if pay is not None else None, int(bool(payload_aligned)),
                              ctypes.byref(r), ctypes.byref(counters) if counters is not None else None)
    return ({"status": r.status, "size": r.size, "type": r.type, "value": r.value, "ucase": r.ucase},
            {"size": m.size, "type": m.checksum_type, "value": m.checksum_value})


def read_result_checksum(batch_type, chunk_type, chunk_value, chunk_len, offset, length, data, recalculate, full):
    """AioReadJob::setResult restatement -> (status, type, value)."""
    L = lib()
    if not hasattr(L, "_read_result_bound"):
        u8, u32 = ctypes.c_uint8, ctypes.c_uint32
        L.orc_read_result_checksum.restype = ctypes.c_int
        L.orc_read_result_checksum.argtypes = [u8, u8, u32, u32, u32, u32, ctypes.c_void_p, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.POINTER(u8), ctypes.POINTER(u32)]
        L._read_result_bound = True
    t, v = ctypes.c_uint8(0), ctypes.c_uint32(0)
    d = np.ascontiguousarray(data, dtype=np.uint8)
    f = np.ascontiguousarray(full, dtype=np.uint8)
    rc = L.orc_read_result_checksum(batch_type, chunk_type, chunk_value & 0xFFFFFFFF, chunk_len, offset, length,
                                    _ptr(d), int(recalculate), _ptr(f), ctypes.byref(t), ctypes.byref(v))
    return rc, t.value, v.value
