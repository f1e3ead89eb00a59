#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

The reference holds no asserted literal CRC outputs; its
tests pin the path relationally against folly / the crc32c crate.  So:

* ``kat`` cases carry expected values taken from the reference itself (the
  constants at tests/common/utils/TestFolly.cc:20-21) and the published
  CRC-32C / CRC-32 check values.  These pin the oracle.
* every other case is input (a generator recipe) plus the oracle's output; the
  oracle is pinned beforehand by the KATs and by three independent CRC
  mechanisms (bitwise, byte table, x86 SSE4.2 ``crc32``) agreeing.
* the update traces replay the reference's VerifyChecksum test shape
  (tests/storage/client/TestStorageClientInterface.cc:357-463: SEQ/JUMP/RAND
  writes into 128 KiB and 512 B chunks) and record the whole-chunk CRC after
  every write, which is exactly what that test asserts (:435).

Patterns mirror the reference tests: 0xFF fill (TestStorageClientInterface.cc:363),
'A'+i fill (src/client/cli/admin/Bench.cc:96-97), constant ``i as u8`` chunks
(src/storage/chunk_engine/src/core/engine.rs:1004), "etc"+"zzz" at offset 3
(engine.rs:1243-1253), "hello"/"world" (tests/common/utils/TestFolly.cc:10-18).

Run:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as orc  # noqa: E402

SEED = 20250629


def materialize(case) -> np.ndarray:
    """Rebuild a case's payload from its recipe (shared with the tests)."""
    p = case["pattern"]
    n = case["len"]
    if p == "splitmix":
        return orc.splitmix_bytes(n, case["seed"], case.get("chunk", 0))
    if p == "fill":
        return np.full(n, case["byte"], dtype=np.uint8)
    if p == "ascii":
        return np.frombuffer(case["text"].encode(), dtype=np.uint8).copy()
    if p == "ramp":
        return (np.arange(n, dtype=np.uint64) % 251).astype(np.uint8)
    raise ValueError(p)


def crc_case(**kw):
    c = dict(kw)
    c.setdefault("start", 0xFFFFFFFF)
    data = materialize(c)
    assert data.size == c["len"]
    c["crc32c_raw"] = orc.crc32c(data, c["start"], "table")
    c["crc32_raw"] = orc.crc32(data, c["start"])
    return c


def gen_crc_vectors():
    cases = []
    # Known answers (expected values NOT from the oracle).
    cases.append({"name": "kat_check_123456789", "pattern": "ascii", "text": "123456789", "len": 9,
                  "start": 0xFFFFFFFF, "kat_crc32c_std": 0xE3069283, "kat_crc32_std": 0xCBF43926})
    cases.append({"name": "kat_testfolly_1MiB_zero", "pattern": "fill", "byte": 0, "len": 1 << 20,
                  "start": 0xFFFFFFFF, "kat_crc32c_std": 0x14298C12})  # TestFolly.cc:20
    cases.append({"name": "kat_testfolly_one_zero", "pattern": "fill", "byte": 0, "len": 1,
                  "start": 0xFFFFFFFF, "kat_crc32c_std": 0x527D5351})  # TestFolly.cc:21
    for c in cases:
        d = materialize(c)
        c["crc32c_raw"] = orc.crc32c(d, c["start"], "table")
        c["crc32_raw"] = orc.crc32(d, c["start"])
        assert (~c["crc32c_raw"]) & 0xFFFFFFFF == c["kat_crc32c_std"], c["name"]
        if "kat_crc32_std" in c:
            assert (~c["crc32_raw"]) & 0xFFFFFFFF == c["kat_crc32_std"], c["name"]

    # Reference test patterns.
    cases.append(crc_case(name="hello", pattern="ascii", text="hello", len=5, start=0))
    cases.append(crc_case(name="world", pattern="ascii", text="world", len=5, start=0))
    cases.append(crc_case(name="etczzz", pattern="ascii", text="etczzz", len=6))
    cases.append(crc_case(name="ff_128KiB", pattern="fill", byte=0xFF, len=128 << 10))
    cases.append(crc_case(name="ff_512B", pattern="fill", byte=0xFF, len=512))
    for i in range(16):
        cases.append(crc_case(name=f"bench_A+{i}_1MiB", pattern="fill", byte=ord("A") + i, len=1 << 20))
    cases.append(crc_case(name="bench_A_128MiB", pattern="fill", byte=ord("A"), len=128 << 20))
    for i in (0, 1, 255, 256 & 0xFF, 300 & 0xFF):
        cases.append(crc_case(name=f"engine_const_{i}_64KiB", pattern="fill", byte=i, len=64 << 10))

    # Lengths around every boundary the kernels care about (16 B pieces, 1 KiB
    # rows, segment sizes, 1 MiB iterator pieces), random starts.
    rng = random.Random(SEED)
    lengths = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 257, 1000, 1023, 1024, 1025,
               2047, 2048, 2049, 4095, 4096, 4097, 16383, 16384, 16385, 65535, 65536, 65537, 262143, 262144, 262145,
               (1 << 20) - 1, 1 << 20, (1 << 20) + 1, (2 << 20) + 12345, 4 << 20]
    for i, n in enumerate(lengths):
        for start in (0xFFFFFFFF, 0, rng.getrandbits(32)):
            cases.append(crc_case(name=f"splitmix_len{n}_s{start:08x}", pattern="splitmix", seed=SEED, chunk=i,
                                  len=n, start=start))
    cases.append(crc_case(name="ramp_1MiB", pattern="ramp", len=1 << 20))
    return cases


def gen_combine_vectors():
    rng = random.Random(SEED + 1)
    out = []
    for len2 in [0, 1, 2, 3, 4, 5, 8, 15, 16, 1023, 1024, 4096, 65536, 1 << 20, (1 << 20) + 3, 64 << 20,
                 (1 << 32) + 7, 1 << 40]:
        for _ in range(3):
            c1, c2 = rng.getrandbits(32), rng.getrandbits(32)
            out.append({"c1": c1, "c2": c2, "len2": len2,
                        "crc32c": orc.lib().orc_crc32c_combine(c1, c2, len2),
                        "crc32": orc.lib().orc_crc32_combine(c1, c2, len2)})
    # TestFolly.cc:9-18 "hello"/"world" with start 0.
    a = orc.crc32c(b"hello", 0)
    b = orc.crc32c(b"world", 0)
    out.append({"c1": a, "c2": b, "len2": 5, "crc32c": orc.crc32c(b"world", a),
                "crc32": orc.lib().orc_crc32_combine(a, b, 5), "name": "testfolly_hello_world"})
    return out


def gen_update_traces():
    """SEQ / JUMP / RAND write traces as in TestStorageClientInterface.cc:381-408."""
    rng = random.Random(SEED + 2)
    traces = []
    for chunk_size in (128 << 10, 512):
        for pattern in ("SEQ", "JUMP", "RAND"):
            chunk = np.zeros(0, dtype=np.uint8)
            offset = length = 0
            ops = []
            for widx in range(1, 101):
                if pattern == "SEQ":
                    offset += length
                elif pattern == "JUMP":
                    offset += length + rng.randint(0, length // 2)
                else:
                    offset = rng.randint(0, chunk_size - 1)
                if offset + 1 >= chunk_size:
                    continue
                length = rng.randint(1, max(1, (chunk_size - offset) // 2))
                seed = rng.getrandbits(48)
                data = orc.splitmix_bytes(length, seed, widx)
                if offset + length > chunk.size:
                    grown = np.zeros(offset + length, dtype=np.uint8)
                    grown[: chunk.size] = chunk
                    chunk = grown
                chunk[offset: offset + length] = data
                ops.append({"offset": offset, "length": length, "seed": seed, "widx": widx,
                            "write_crc32c": orc.crc32c(data),
                            "chunk_size_after": int(chunk.size),
                            "chunk_crc32c": orc.crc32c(chunk)})
            traces.append({"chunk_size": chunk_size, "pattern": pattern, "ops": ops})
    return traces


def main():
    with open(os.path.join(HERE, "crc_vectors.json"), "w") as f:
        json.dump(gen_crc_vectors(), f, indent=0)
    with open(os.path.join(HERE, "combine_vectors.json"), "w") as f:
        json.dump(gen_combine_vectors(), f, indent=0)
    with open(os.path.join(HERE, "update_traces.json"), "w") as f:
        json.dump(gen_update_traces(), f, indent=0)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
