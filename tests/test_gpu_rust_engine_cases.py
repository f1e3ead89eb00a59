"""The Rust chunk engine's own checksum test sequences, replayed through the GPU update path
in the std domain (h3c_update_ios with H3C_UPD_STD_DOMAIN).

Each test restates one test of src/storage/chunk_engine/src/core/engine.rs: the same
writes / truncates in the same order, and the same assertions (the chunk checksum equals
crc32c::crc32c of the chunk's bytes, lengths, checksum-mismatch errors).  crc32c here is
the oracle's (std = ~raw)."""
import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu
MASK = 0xFFFFFFFF
WRITE, TRUNCATE = 1, 4


def std(b):
    return (~orc.crc32c(np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b)) & MASK


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


class Engine:
    """A set of chunks in HBM driven through h3c_update_ios (std domain), one op at a time
    or in batches; mirrors chunk_engine Engine::write / truncate."""

    def __init__(self, h3c, torch, dev, nchunks, capacity):
        self.h3c, self.torch, self.dev = h3c, torch, dev
        self.cap = capacity
        self.slab = torch.zeros(nchunks * capacity, dtype=torch.uint8, device=dev)
        self.state = np.zeros(nchunks, dtype=h3c.CHUNK_STATE_DTYPE)
        for c in range(nchunks):
            # a new chunk: no bytes, checksum of nothing (std 0)
            self.state[c] = (self.slab.data_ptr() + c * capacity, capacity, 0, 0, 1, 0)
        self.keep = []

    def ops(self, ops):
        """ops: list of (chunk, kind, offset, data(bytes|None), length, checksum|None)."""
        ios = np.zeros(len(ops), dtype=self.h3c.UPDATE_IO_DTYPE)
        for i, (c, kind, off, data, length, ck) in enumerate(ops):
            ptr = 0
            if data is not None and len(data):
                t = self.torch.from_numpy(np.frombuffer(bytes(data), dtype=np.uint8).copy()).to(self.dev)
                self.keep.append(t)
                ptr = t.data_ptr()
            ios[i] = (ptr, c, off, length, 0 if ck is None else ck, 0 if ck is None else 1, kind, 0, 0, 0)
        res = self.h3c.update_ios(self.state, ios, std_domain=True)
        self.torch.cuda.synchronize()
        return res

    def write(self, c, data, off, ck):
        return self.ops([(c, WRITE, off, data, len(data), ck)])[0]

    def bytes(self, c):
        n = int(self.state[c]["size"])
        return self.slab[c * self.cap: c * self.cap + n].cpu().numpy()


def test_engine_rs_hello_world_sequence(h3c, torch_dev):
    """engine.rs:734-860: write 12 bytes; a wrong checksum fails; append at 12; zeros at 0."""
    torch, dev = torch_dev
    e = Engine(h3c, torch, dev, 1, 64 << 10)
    data = b"hello world!"
    r = e.write(0, data, 0, 0)  # engine.write(chunk_id, bytes, 0, 0).is_err()
    assert int(r["status"]) == 4080
    r = e.write(0, data, 0, std(data))
    assert int(r["status"]) == 0 and int(e.state[0]["size"]) == 12
    assert bytes(e.bytes(0)) == data and int(e.state[0]["value"]) == std(data)
    r = e.write(0, data, 12, std(data))
    assert int(e.state[0]["size"]) == 24
    zeros = bytes(12)
    r = e.write(0, zeros, 0, std(zeros))
    assert int(e.state[0]["size"]) == 24
    assert bytes(e.bytes(0)) == zeros + data
    assert int(e.state[0]["value"]) == std(zeros + data) == int(r["value"])


def test_engine_rs_test_engine_checksum(h3c, torch_dev):
    """engine.rs:1228-1255 test_engine_checksum: "etc" @0, "zzz" @3 -> crc32c("etczzz");
    then a write without checksum (adopted, :297-302) keeps the invariant."""
    torch, dev = torch_dev
    e = Engine(h3c, torch, dev, 1, 64 << 10)
    e.write(0, b"etc", 0, std(b"etc"))
    r = e.write(0, b"zzz", 3, std(b"zzz"))
    assert bytes(e.bytes(0)) == b"etczzz"
    assert int(r["value"]) == std(b"etczzz") == int(e.state[0]["value"])
    r = e.write(0, b"zzz", 6, None)  # without_checksum: true
    assert int(r["status"]) == 0 and int(r["value"]) == std(b"etczzzzzz")


def test_engine_rs_extend_truncate_512_chunks(h3c, torch_dev):
    """engine.rs:1126-1178: 512 chunks of 64 KiB filled with i; an empty write at i*131
    extends to max(i*131, 64 KiB); truncate to i*137; checksum == crc32c(bytes[..len]) with
    the first min(len, 64 KiB) bytes i and zeros after.  All 1536 ops in one batch."""
    torch, dev = torch_dev
    n, small = 512, 64 << 10
    e = Engine(h3c, torch, dev, n, 128 << 10)
    ops = []
    for i in range(n):
        d = bytes([i & 255]) * small
        ops.append((i, WRITE, 0, d, small, std(d)))
    for i in range(n):
        ops.append((i, WRITE, i * 131, None, 0, 0))  # engine.write(id, &[], length, 0)
    for i in range(n):
        ops.append((i, TRUNCATE, 0, None, i * 137, None))  # engine.truncate(id, length)
    res = e.ops(ops)
    assert (res["status"] == 0).all()
    for i in range(n):
        assert int(res[n + i]["size"]) == max(i * 131, small)  # :1149-1152
        length = i * 137
        assert int(e.state[i]["size"]) == length
        bound = min(length, small)
        want = bytes([i & 255]) * bound + bytes(length - bound)
        assert int(e.state[i]["value"]) == std(want), i
        assert int(res[2 * n + i]["value"]) == std(want)
    got = e.slab.cpu().numpy()
    for i in (0, 1, 300, 478, 479, 511):
        length = i * 137
        assert bytes(got[i * (128 << 10): i * (128 << 10) + length]) == \
            bytes([i & 255]) * min(length, small) + bytes(max(0, length - small))


def test_engine_rs_rewrite_after_reopen(h3c, torch_dev):
    """engine.rs:990-1010: chunks of constant i as u8 (checksum crc32c([i; 64 KiB])), then a
    whole-chunk rewrite with !i (copy_on_write's full-overwrite reuse, chunk.rs:117-160)."""
    torch, dev = torch_dev
    n, small = 64, 64 << 10
    e = Engine(h3c, torch, dev, n, small)
    first = [(i, WRITE, 0, bytes([i & 255]) * small, small, std(bytes([i & 255]) * small)) for i in range(n)]
    e.ops(first)
    for i in range(n):
        assert int(e.state[i]["value"]) == std(np.full(small, i & 255, dtype=np.uint8))
    second = [(i, WRITE, 0, bytes([~i & 255]) * small, small, std(bytes([~i & 255]) * small)) for i in range(n)]
    res = e.ops(second)
    for i in range(n):
        assert int(res[i]["value"]) == std(np.full(small, ~i & 255, dtype=np.uint8))
