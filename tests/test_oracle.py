"""The CPU oracle, pinned before anything is checked against it (CPU only).

Pins: standard CRC-32C / CRC-32 check values, the constants logged at
tests/common/utils/TestFolly.cc:20-21 of the reference, the combine identity of
TestFolly.cc:9-18, three independent CRC mechanisms agreeing, and the
whole-chunk CRC after partial writes (TestStorageClientInterface.cc:435).
"""
import json
import os
import zlib

import numpy as np
import pytest

import oracle_lib as orc
from golden.gen_golden import materialize

HERE = os.path.dirname(os.path.abspath(__file__))
CRC_VECTORS = json.load(open(os.path.join(HERE, "golden", "crc_vectors.json")))
COMBINE_VECTORS = json.load(open(os.path.join(HERE, "golden", "combine_vectors.json")))
UPDATE_TRACES = json.load(open(os.path.join(HERE, "golden", "update_traces.json")))
MASK = 0xFFFFFFFF


def test_standard_check_values():
    assert orc.crc32c(b"123456789") == 0x1CF96D7C  # raw
    assert (~orc.crc32c(b"123456789")) & MASK == 0xE3069283  # std
    assert (~orc.crc32(b"123456789")) & MASK == 0xCBF43926


def test_testfolly_constants():
    # TestFolly.cc:20-21 log ~0x14298C12 (1 MiB of zeros) and ~0x527D5351 (one zero byte).
    assert orc.crc32c(bytes(1 << 20)) == (~0x14298C12) & MASK
    assert orc.crc32c(bytes(1)) == (~0x527D5351) & MASK
    # ...and combine them the way the test does: crc32c_combine(~crc1, crc2, 1)
    out = orc.lib().orc_crc32c_combine(0x14298C12, (~0x527D5351) & MASK, 1)
    assert out == orc.crc32c(bytes((1 << 20) + 1), 0xFFFFFFFF) ^ 0  # raw of 1 MiB + 1 zero bytes


def test_testfolly_combine_identity():
    # TestFolly.cc:9-18: combine(crc32c(a,0), crc32c(b,0), |b|) == crc32c(b, start=crc32c(a,0))
    a, b = b"hello", b"world"
    c1, c2 = orc.crc32c(a, 0), orc.crc32c(b, 0)
    assert orc.lib().orc_crc32c_combine(c1, c2, len(b)) == orc.crc32c(b, c1)


@pytest.mark.parametrize("case", CRC_VECTORS, ids=lambda c: c["name"])
def test_golden_crc_vectors_all_mechanisms(case):
    data = materialize(case)
    start = case["start"]
    want = case["crc32c_raw"]
    assert orc.crc32c(data, start, "table") == want
    assert orc.crc32c(data, start, "sse42") == want
    assert orc.crc32c(data, start, "sse42_3way") == want
    if data.size <= (64 << 10):
        assert orc.crc32c(data, start, "bitwise") == want
    assert orc.crc32(data, start) == case["crc32_raw"]
    if start == 0xFFFFFFFF and data.size <= (4 << 20):
        assert (~case["crc32_raw"]) & MASK == zlib.crc32(data.tobytes())  # independent IEEE oracle
    if "kat_crc32c_std" in case:
        assert (~want) & MASK == case["kat_crc32c_std"]


@pytest.mark.parametrize("v", COMBINE_VECTORS)
def test_golden_combine_vectors(v):
    assert orc.lib().orc_crc32c_combine(v["c1"], v["c2"], v["len2"]) == v["crc32c"]
    assert orc.lib().orc_crc32_combine(v["c1"], v["c2"], v["len2"]) == v["crc32"]


def test_combine_matches_concatenation_random():
    rng = np.random.default_rng(1)
    for _ in range(50):
        na, nb = int(rng.integers(0, 5000)), int(rng.integers(0, 5000))
        a = rng.integers(0, 256, na, dtype=np.uint8)
        b = rng.integers(0, 256, nb, dtype=np.uint8)
        s = int(rng.integers(0, 1 << 32))
        ab = np.concatenate([a, b])
        # raw(init s, A||B) == combine(raw(init s, A), crc0(B), |B|)
        assert orc.lib().orc_crc32c_combine(orc.crc32c(a, s), orc.crc32c(b, 0), nb) == orc.crc32c(ab, s)
        # ChecksumInfo::combine on ~0-start values yields raw(A||B) (Common.h:191)
        rc, t, v = orc.combine(orc.CRC32C, orc.crc32c(a), orc.CRC32C, orc.crc32c(b), nb)
        if nb:
            assert rc == 0 and t == orc.CRC32C and v == orc.crc32c(ab)


def test_checksum_info_create_semantics():
    assert orc.create(orc.NONE, b"abc") == (orc.NONE, 0)  # Common.h:150
    assert orc.create(orc.CRC32C, b"") == (orc.CRC32C, 0xFFFFFFFF)  # empty: {type, start}
    assert orc.create(orc.CRC32C, b"", start=0x1234) == (orc.CRC32C, 0x1234)
    assert orc.create(orc.CRC32C, None, 10) == (orc.NONE, 0)  # iterBytes != length (Common.h:166-169)
    big = orc.splitmix_bytes((3 << 20) + 5, 7, 0)  # chained over 1 MiB iterator pieces
    assert orc.create(orc.CRC32C, big) == (orc.CRC32C, orc.crc32c(big))
    assert orc.create(orc.CRC32, big)[1] == orc.crc32(big)


def test_checksum_info_combine_semantics():
    assert orc.combine(orc.CRC32C, 5, orc.CRC32, 7, 10)[0] == 4080  # type mismatch (Common.h:180-183)
    assert orc.combine(orc.CRC32C, 5, orc.CRC32C, 7, 0) == (0, orc.CRC32C, 5)  # length 0 no-op
    assert orc.combine(orc.NONE, 0, orc.CRC32C, 7, 10) == (0, orc.CRC32C, 7)  # NONE receiver copies
    assert orc.combine(orc.NONE, 0, orc.CRC32, 9, 0) == (0, orc.NONE, 0)  # length 0 first


@pytest.mark.parametrize("trace", UPDATE_TRACES, ids=lambda t: f"{t['pattern']}_{t['chunk_size']}")
def test_update_checksum_traces(trace):
    """ChunkReplica::updateChecksum restated, replayed over the reference test's write shapes.

    After every write the stored chunk checksum must equal crc32c(whole chunk)
    (TestStorageClientInterface.cc:435)."""
    chunk = np.zeros(0, dtype=np.uint8)
    meta = {"size": 0, "type": orc.NONE, "value": 0}
    for op in trace["ops"]:
        off, ln = op["offset"], op["length"]
        data = orc.splitmix_bytes(ln, op["seed"], op["widx"])
        wt, wv = orc.create(orc.CRC32C, data)
        assert wv == op["write_crc32c"]
        size_before = chunk.size
        is_append = off == size_before  # ChunkReplica.cc:246
        if off + ln > chunk.size:
            grown = np.zeros(off + ln, dtype=np.uint8)
            grown[: chunk.size] = chunk
            chunk = grown
        chunk[off: off + ln] = data
        meta["size"] = chunk.size
        rc, meta = orc.update_checksum(meta, {"offset": off, "length": ln, "type": wt, "value": wv},
                                       size_before, is_append, chunk)
        assert rc == 0
        assert meta["value"] == op["chunk_crc32c"] == orc.crc32c(chunk)


def test_splitmix_generator_matches_python():
    def sm(x):
        x = (x + 0x9E3779B97F4A7C15) & ((1 << 64) - 1)
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
        return x ^ (x >> 31)

    seed, chunk = 20250629, 5
    got = orc.splitmix_bytes(45, seed, chunk)
    words = [sm(seed ^ (chunk << 40) ^ k) for k in range(6)]
    want = b"".join(w.to_bytes(8, "little") for w in words)[:45]
    assert got.tobytes() == want


def test_std_domain_combine():
    """Rust crc32c-crate domain (std = ~raw, ChunkEngine.cc:42,66): combine is the same shift-XOR."""
    rng = np.random.default_rng(8)
    for _ in range(30):
        a = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)
        b = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)
        std = lambda x: (~orc.crc32c(x)) & MASK
        assert orc.lib().orc_crc32c_combine(std(a), std(b), b.size) == std(np.concatenate([a, b]))


@pytest.mark.parametrize("seed", [21, 22])
def test_replica_update_restatement_relational_pin(seed):
    """The reference pins chunk checksums only relationally: after every write the stored
    checksum equals crc32c of the whole chunk (TestStorageClientInterface.cc:431-459).
    Replay random WRITE / TRUNCATE / EXTEND sequences through the ChunkReplica::update
    restatement and check that relation, the zero of updateChecksum case (i), the
    kInvalidArg range check and the client-checksum verify."""
    rng = np.random.default_rng(seed)
    cs = 20000
    chunk = np.zeros(cs, dtype=np.uint8)
    model = np.zeros(0, dtype=np.uint8)
    meta = {"size": 0, "type": orc.NONE, "value": 0}
    for _ in range(300):
        u = rng.random()
        if u < 0.6:
            off = int(rng.integers(0, cs))
            ln = int(rng.integers(0, min(cs - off, 3000) + 1))
            p = rng.integers(0, 256, ln, dtype=np.uint8)
            ty = orc.CRC32C if rng.random() > 0.15 else orc.NONE
            val = orc.create(ty, p, ln)[1] if ty else 0
            good = rng.random() > 0.1 or ty == orc.NONE or ln == 0
            io = {"kind": orc.UPD_WRITE, "offset": off, "length": ln, "type": ty, "value": val if good else val ^ 4}
            res, meta2 = orc.replica_update(meta, chunk, cs, io, p)
            if not good:
                assert res["status"] == 4080 and meta2 == meta
                continue
            assert res["status"] == 0
            if off > model.size:
                model = np.concatenate([model, np.zeros(off - model.size, dtype=np.uint8)])
            if off + ln > model.size:
                model = np.concatenate([model, np.zeros(off + ln - model.size, dtype=np.uint8)])
            model[off:off + ln] = p
        elif u < 0.8:
            kind = orc.UPD_TRUNCATE if rng.random() < 0.5 else orc.UPD_EXTEND
            t = int(rng.integers(0, cs + 1))
            res, meta2 = orc.replica_update(meta, chunk, cs, {"kind": kind, "offset": 0, "length": t, "type": 0,
                                                              "value": 0})
            assert res["status"] == 0
            if t > model.size:
                model = np.concatenate([model, np.zeros(t - model.size, dtype=np.uint8)])
            elif kind == orc.UPD_TRUNCATE:
                model = model[:t].copy()
        else:
            res, meta2 = orc.replica_update(meta, chunk, cs, {"kind": orc.UPD_WRITE, "offset": cs - 5, "length": 9,
                                                              "type": 1, "value": 0},
                                            np.zeros(9, dtype=np.uint8))
            assert res["status"] == 3 and meta2 == meta
            continue
        meta = meta2
        assert meta["size"] == model.size == res["size"]
        assert np.array_equal(chunk[:model.size], model)
        if meta["type"] == orc.NONE or model.size == 0:
            assert meta["value"] == 0
        else:
            assert meta["value"] == orc.crc32c(model)
        assert (res["type"], res["value"]) == (meta["type"], meta["value"])


def test_vpclmul_best_case_cpu_variant_matches():
    """The best-case CPU variant (VPCLMULQDQ folding, not the reference's path) is bit-exact
    with the table restatement at every length around its 512 B / 256 B / 16 B boundaries."""
    import ctypes

    L = orc.lib()
    L.orc_crc32c_vpclmul.restype = ctypes.c_uint32
    L.orc_crc32c_vpclmul.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    rng = np.random.default_rng(31)
    sizes = list(range(0, 40)) + [255, 256, 257, 511, 512, 513, 767, 768, 1023, 1024, 1040, 4096 + 7,
                                  (1 << 20) + 13]
    for n in sizes:
        a = rng.integers(0, 256, n, dtype=np.uint8)
        for st in (0xFFFFFFFF, 0, 0xDEADBEEF):
            assert L.orc_crc32c_vpclmul(a.ctypes.data if n else None, n, st) == orc.crc32c(a, st, mech="table")


def _std(crc_raw):
    return (~crc_raw) & 0xFFFFFFFF


def test_replica_remove_commit_and_syncing_restatement():
    """REMOVE (doRemove builds {offset 0, length 0, NONE}, StorageOperator.cc:808-815) runs
    updateChecksum case (i): {NONE, 0}, size and bytes unchanged.  COMMIT sets no checksum
    (ChunkReplica::commit, :397-467).  A syncing full-chunk write (ReliableForwarding.cc:203-207)
    sets meta.size = length (:289) and takes the reuse branch (:337-339)."""
    rng = np.random.default_rng(1)
    cs = 16384
    chunk = np.zeros(cs, dtype=np.uint8)
    chunk[:9000] = rng.integers(0, 256, 9000, dtype=np.uint8)
    meta = {"size": 9000, "type": orc.CRC32C, "value": orc.crc32c(chunk[:9000])}
    res, m2 = orc.replica_update(dict(meta), chunk, cs, {"kind": orc.UPD_COMMIT, "offset": 0, "length": 0,
                                                         "type": 0, "value": 0})
    assert res == {"status": 0, "size": 9000, "type": 0, "value": 0, "ucase": orc.CASE_NOT_RUN} and m2 == meta
    p = rng.integers(0, 256, 5000, dtype=np.uint8)
    res, m3 = orc.replica_update(dict(meta), chunk, cs, {"kind": orc.UPD_WRITE, "offset": 0, "length": 5000,
                                                         "type": orc.CRC32C, "value": orc.crc32c(p),
                                                         "syncing": 1}, p)
    assert res["status"] == 0 and res["ucase"] == orc.CASE_REUSE
    assert m3 == {"size": 5000, "type": orc.CRC32C, "value": orc.crc32c(p)}
    res, m4 = orc.replica_update(dict(m3), chunk, cs, {"kind": orc.UPD_REMOVE, "offset": 0, "length": 0,
                                                       "type": 0, "value": 0})
    assert res == {"status": 0, "size": 5000, "type": 0, "value": 0, "ucase": orc.CASE_NONE}
    assert m4 == {"size": 5000, "type": 0, "value": 0}


def test_replica_stale_stored_checksum_semantics():
    """What the reference stores when meta.checksumValue disagrees with the bytes: an append
    combines with the stale value (:340-355, the error is carried, shifted), the prefix /
    suffix case re-reads the bytes (:356-390, the error is gone), and a truncate whose
    offset equals the size keeps the stale value (combine of length 0)."""
    rng = np.random.default_rng(2)
    cs = 1 << 16
    chunk = np.zeros(cs, dtype=np.uint8)
    chunk[:8192] = rng.integers(0, 256, 8192, dtype=np.uint8)
    good = orc.crc32c(chunk[:8192])
    err = 0x00400001
    meta = {"size": 8192, "type": orc.CRC32C, "value": good ^ err}
    p = rng.integers(0, 256, 100, dtype=np.uint8)
    res, meta = orc.replica_update(meta, chunk, cs, {"kind": orc.UPD_WRITE, "offset": 8192, "length": 100,
                                                     "type": orc.CRC32C, "value": orc.crc32c(p)}, p)
    assert res["ucase"] == orc.CASE_COMBINE
    assert meta["value"] == orc.crc32c(chunk[:8292]) ^ orc.lib().orc_shift(err, 100, orc.POLY_CRC32C)
    res, meta2 = orc.replica_update(dict(meta), chunk.copy(), cs, {"kind": orc.UPD_TRUNCATE, "offset": 8292,
                                                                   "length": 50, "type": 0, "value": 0})
    assert res["ucase"] == orc.CASE_COMBINE and meta2["size"] == 50 and meta2["value"] == meta["value"]
    q = rng.integers(0, 256, 10, dtype=np.uint8)
    res, meta = orc.replica_update(meta, chunk, cs, {"kind": orc.UPD_WRITE, "offset": 20, "length": 10,
                                                     "type": orc.CRC32C, "value": orc.crc32c(q)}, q)
    assert res["ucase"] == orc.CASE_READ_CHUNK and meta["value"] == orc.crc32c(chunk[:8292])


def test_engine_restatement_relational_pin():
    """engine.rs's own assertion (test_engine_checksum :1229-1253 and :789-818): after every
    update the stored std checksum is crc32c of the chunk content; the "etc" + "zzz" at offset
    3 trace; and the checksum counters add up to the ops that reached copy_on_write /
    safe_write."""
    cs = 1 << 16
    chunk = np.zeros(cs, dtype=np.uint8)
    meta = {"size": 0, "type": orc.CRC32C, "value": 0}
    cnt = orc.EngineCounters()
    for off, data in ((0, b"etc"), (3, b"zzz")):
        p = np.frombuffer(data, dtype=np.uint8)
        res, meta = orc.engine_update(meta, chunk, cs, {"kind": orc.UPD_WRITE, "offset": off, "length": 3,
                                                        "type": orc.CRC32C, "value": orc.crc32c(p)}, p,
                                      counters=cnt)
        assert res["status"] == 0
    assert bytes(chunk[:6]) == b"etczzz" and meta["value"] == _std(orc.crc32c(b"etczzz"))
    rng = np.random.default_rng(3)
    host = np.zeros(cs, dtype=np.uint8)
    size, applied = 6, 2
    host[:6] = chunk[:6]
    for _ in range(300):
        u = rng.random()
        if u < 0.6:
            off = int(rng.integers(0, cs))
            if rng.random() < 0.5:
                off -= off % 4096
            ln = int(rng.integers(0, min(cs - off, 9000) + 1))
            if rng.random() < 0.3:
                ln -= ln % 4096
            p = rng.integers(0, 256, ln, dtype=np.uint8)
            io = {"kind": orc.UPD_WRITE, "offset": off, "length": ln, "type": orc.CRC32C, "value": orc.crc32c(p)}
            res, meta = orc.engine_update(meta, chunk, cs, io, p, payload_aligned=rng.random() < 0.5, counters=cnt)
            if off > size:
                host[size:off] = 0
            host[off:off + ln] = p
            size = max(size, off + ln)
        else:
            t = int(rng.integers(0, cs + 1))
            kind = orc.UPD_TRUNCATE if u < 0.85 else orc.UPD_EXTEND
            res, meta = orc.engine_update(meta, chunk, cs, {"kind": kind, "offset": 0, "length": t, "type": 0,
                                                            "value": 0}, None, counters=cnt)
            if t > size:
                host[size:t] = 0
            if kind == orc.UPD_TRUNCATE or t > size:
                size = t
        assert res["status"] == 0 and res["size"] == size == meta["size"]
        assert meta["value"] == _std(orc.crc32c(host[:size])), _
        assert res["type"] == orc.CRC32C and res["value"] == orc.crc32c(host[:size])
        if res["ucase"] != orc.CASE_KEEP:
            applied += 1
    assert cnt.reuse + cnt.recalculate + cnt.combine >= applied - 2


def test_replica_update_chunk_size_semantics():
    """UpdateIO.chunkSize restated (ChunkReplica.cc:141-145, 171-180): the range check uses the
    op's chunkSize (kInvalidArg, before result.checksum is set); a WRITE / TRUNCATE whose chunkSize
    differs from the chunk's fails with kChunkSizeMismatch (4015) after :174 set result.checksum =
    meta.checksum(), leaving bytes and metadata alone; REMOVE takes the chunk's own chunkSize."""
    cs = 8192
    rng = np.random.default_rng(15)
    chunk = rng.integers(0, 256, cs, dtype=np.uint8)
    meta = {"size": 6000, "type": orc.CRC32C, "value": orc.crc32c(chunk[:6000])}
    before = chunk.copy()
    pay = rng.integers(0, 256, 10, dtype=np.uint8)
    w = {"kind": orc.UPD_WRITE, "offset": 100, "length": 10, "type": orc.CRC32C,
         "value": orc.create(orc.CRC32C, pay, 10)[1]}
    res, m2 = orc.replica_update(dict(meta), chunk, cs, dict(w, chunk_size=4096), pay)
    assert res["status"] == 4015 and (res["type"], res["value"]) == (orc.CRC32C, meta["value"])
    assert m2 == meta and np.array_equal(chunk, before)
    res, m2 = orc.replica_update(dict(meta), chunk, cs, dict(w, offset=5000, chunk_size=4096), pay)
    assert res["status"] == 3 and res["type"] == 0 and res["value"] == 0  # range check first
    res, m2 = orc.replica_update(dict(meta), chunk, cs, dict(w, offset=8190, chunk_size=16384), pay)
    assert res["status"] == 4015
    res, _ = orc.replica_update(dict(meta), chunk, cs, {"kind": orc.UPD_TRUNCATE, "offset": 0, "length": 10,
                                                        "type": 0, "value": 0, "chunk_size": 4096})
    assert res["status"] == 4015
    res, m2 = orc.replica_update(dict(meta), chunk, cs, {"kind": orc.UPD_REMOVE, "offset": 0, "length": 0,
                                                         "type": 0, "value": 0, "chunk_size": 7})
    assert res["status"] == 0 and m2["type"] == orc.NONE
    res, m2 = orc.replica_update(dict(meta), chunk, cs, dict(w, chunk_size=cs), pay)  # equal: applied
    assert res["status"] == 0 and m2["value"] == orc.crc32c(chunk[:6000])
