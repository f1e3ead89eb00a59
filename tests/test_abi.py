"""C-ABI library: loads, exports every declared symbol, host arithmetic parity (CPU only).

No payload compute runs here (no GPU in this container); on a GPU-less host the
payload entry points must fail loudly with H3C_ERR_NO_DEVICE, never fall back.
"""
import ctypes
import json
import os
import re

import numpy as np
import pytest

import oracle_lib as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "h3c_crc.h")
COMBINE_VECTORS = json.load(open(os.path.join(ROOT, "tests", "golden", "combine_vectors.json")))


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(h3c_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ("h3c_crc32c_combine", "h3c_crc32_combine", "h3c_batch_create", "h3c_batch_verify",
                 "h3c_batch_combine", "h3c_plan_create", "h3c_plan_run", "h3c_plan_destroy", "h3c_init"):
        assert must in names


def test_library_exports_every_declared_symbol(h3c):
    lib = ctypes.CDLL(h3c.lib_path)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_has_gfx950_code_object(h3c):
    blob = open(h3c.lib_path, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("v", COMBINE_VECTORS)
def test_host_combine_matches_oracle(h3c, v):
    assert h3c.crc32c_combine(v["c1"], v["c2"], v["len2"]) == v["crc32c"]
    assert h3c.crc32_combine(v["c1"], v["c2"], v["len2"]) == v["crc32"]


def test_shift_matches_oracle(h3c):
    rng = np.random.default_rng(3)
    for _ in range(100):
        c = int(rng.integers(0, 1 << 32))
        n = int(rng.integers(0, 1 << 40))
        assert h3c.crc32c_shift(c, n) == orc.lib().orc_shift(c, n, orc.POLY_CRC32C)


def test_checksum_info_combine_mirror(h3c):
    CI, T = h3c.ChecksumInfo, h3c.ChecksumType
    a, b = b"hello ", b"3fs world"
    ca = CI(T.CRC32C, orc.crc32c(a))
    ca.combine(CI(T.CRC32C, orc.crc32c(b)), len(b))
    assert ca == CI(T.CRC32C, orc.crc32c(a + b))
    cn = CI()
    cn.combine(CI(T.CRC32, 7), 3)  # NONE receiver copies (Common.h:186-188)
    assert cn == CI(T.CRC32, 7)
    c0 = CI(T.CRC32C, 5)
    c0.combine(CI(T.CRC32C, 9), 0)  # length 0 no-op (Common.h:184)
    assert c0 == CI(T.CRC32C, 5)
    with pytest.raises(h3c.EngineError) as ei:
        CI(T.CRC32C, 1).combine(CI(T.CRC32, 2), 4)
    assert ei.value.code == 4080
    ieee = CI(T.CRC32, orc.crc32(a))
    ieee.combine(CI(T.CRC32, orc.crc32(b)), len(b))
    assert ieee.value == orc.crc32(a + b)
    assert str(CI(T.CRC32C, 0x1CF96D7C)) == "CRC32C#E3069283"  # formatter prints ~value


def test_no_gpu_fails_loudly(h3c):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(h3c.EngineError) as ei:
        h3c.batch_create([b"abc"])
    assert ei.value.code in (9001, 9002)


def test_folly_signature_entry_aborts_without_a_gpu(h3c):
    """h3c_folly_crc32c keeps folly::crc32c's signature (no error channel): with no usable GPU it
    aborts with the engine's error text instead of returning a wrong checksum."""
    import subprocess
    import sys

    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    code = ("import ctypes; lib = ctypes.CDLL(%r); f = lib.h3c_folly_crc32c; f.restype = ctypes.c_uint32; "
            "f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]; print(f(b'abc', 3, 0xFFFFFFFF))"
            % h3c.lib_path)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "h3c_folly_crc32c" in p.stderr, (p.returncode, p.stdout, p.stderr)


def test_update_ios_rejects_inconsistent_chunk_state(h3c):
    """A chunk state whose size exceeds its chunk_size is a caller bug: the whole call fails
    with kInvalidArg before any device work (so this runs without a GPU)."""
    import numpy as np

    chunks = np.zeros(2, dtype=h3c.CHUNK_STATE_DTYPE)
    chunks["base"] = 1 << 40
    chunks["chunk_size"] = 4096
    chunks["size"] = [4096, 4097]
    chunks["type"] = 1
    ios = np.zeros(1, dtype=h3c.UPDATE_IO_DTYPE)
    ios["kind"] = h3c.UPD_WRITE
    with pytest.raises(h3c.EngineError) as ei:
        h3c.update_ios(chunks, ios)
    assert ei.value.code == 3
