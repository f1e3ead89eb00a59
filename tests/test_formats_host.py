"""Host-side pieces of the adjacent formats (no GPU): ChecksumInfo::combine as a C function,
the client's split-read fold, the Rust-crate std combine and the calcSerde low-byte mark,
each against the oracle restatement."""
import importlib

import numpy as np
import pytest

import oracle_lib as orc

MASK = 0xFFFFFFFF


@pytest.fixture(scope="module")
def client(h3c):
    return importlib.import_module("3fs_amd.client")


def test_checksum_combine_c_matches_oracle(h3c):
    rng = np.random.default_rng(3)
    for _ in range(400):
        t, ot = int(rng.integers(0, 3)), int(rng.integers(0, 3))
        v, ov = int(rng.integers(0, 1 << 32)), int(rng.integers(0, 1 << 32))
        ln = int(rng.choice([0, 1, 7, 4096, 1 << 20, int(rng.integers(0, 1 << 26))]))
        want = orc.combine(t, v, ot, ov, ln)
        info = h3c.ChecksumInfo(h3c.ChecksumType(t), v)
        try:
            info.combine(h3c.ChecksumInfo(h3c.ChecksumType(ot), ov), ln)
            rc = 0
        except h3c.EngineError as e:
            rc = e.code
        assert rc == want[0]
        if rc == 0:
            assert (int(info.type), info.value) == (want[1], want[2])


def test_split_read_fold_matches_whole_buffer(h3c, client):
    """StorageClientImpl.cc:1607-1633: folding the pieces' checksums gives the whole read's."""
    rng = np.random.default_rng(4)
    groups, wants = [], []
    for _ in range(20):
        data = rng.integers(0, 256, int(rng.integers(1, 50000)), dtype=np.uint8)
        cuts = sorted(set(int(x) for x in rng.integers(1, data.size, int(rng.integers(0, 6))))) if data.size > 1 else []
        bounds = [0] + cuts + [data.size]
        pieces = []
        for a, b in zip(bounds, bounds[1:]):
            pieces.append((h3c.ChecksumInfo(h3c.ChecksumType.CRC32C, orc.crc32c(data[a:b])), b - a))
        groups.append(pieces)
        wants.append(orc.crc32c(data))
    # a group with a type mismatch fails with kChecksumMismatch
    groups.append([(h3c.ChecksumInfo(h3c.ChecksumType.CRC32C, 1), 10), (h3c.ChecksumInfo(h3c.ChecksumType.CRC32, 2), 5)])
    infos, status = client.fold_split_reads(groups)
    for k, w in enumerate(wants):
        assert status[k] == 0 and infos[k].type == h3c.ChecksumType.CRC32C and infos[k].value == w
    assert status[-1] == 4080


def test_std_combine_matches_oracle(h3c):
    fm = importlib.import_module("3fs_amd.formats")
    rng = np.random.default_rng(5)
    for _ in range(50):
        a = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8)
        b = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8)
        std = lambda x: (~orc.crc32c(x)) & MASK  # noqa: E731
        assert fm.rust_crc32c.crc32c_combine(std(a), std(b), b.size) == std(np.concatenate([a, b]))


def test_serde_mark():
    h3c = importlib.import_module("3fs_amd")
    for crc0 in (0, 0xFFFFFFFF, 0x12345678, 0xDEADBE01):
        for comp in (0, 1):
            m = h3c.lib.h3c_serde_checksum_mark(crc0, comp)
            assert m == (crc0 & ~0xFF) | 0x86 | comp
            fm = importlib.import_module("3fs_amd.formats")
            assert fm.is_serde_message(m) and fm.is_compressed(m) == bool(comp)


def test_checksum_info_serde_roundtrip(h3c):
    """ChecksumInfo serde (TestCommonStruct.cc:46-56): {CRC32, 0xff} serializes to 1 + 1 + 4
    bytes and deserializes back equal.  The byte layout (Varint32 table length, then type and
    little-endian value) is restated from Serde.h; the reference test pins size and round
    trip only."""
    CI, T = h3c.ChecksumInfo, h3c.ChecksumType
    ser = CI(T.CRC32, 0xFF)
    out = ser.serialize()
    assert len(out) == 1 + 1 + 4 and out == b"\x05\x02\xff\x00\x00\x00"
    assert CI.deserialize(out) == ser
    for t, v in ((T.CRC32C, 0xE3069283 ^ 0xFFFFFFFF), (T.NONE, 0)):
        assert CI.deserialize(CI(t, v).serialize()) == CI(t, v)
    assert CI.deserialize(b"\x01\x01") == CI(T.CRC32C, 0)  # missing trailing field keeps its default
    for bad in (b"", b"\x80", b"\x05\x02\xff", b"\x03\x01\x00\x00"):
        with pytest.raises(h3c.EngineError):
            CI.deserialize(bad)


def test_client_checksum_switches(h3c, client):
    """ReadOptions / WriteOptions.verifyChecksum() (StorageClient.h:188-222) and the read
    request's checksum type (StorageClientImpl.cc:703): defaults, debug builds, bypass options;
    a write with checksums off carries the default {NONE, 0} (no engine call)."""
    R, W, D = client.ReadOptions, client.WriteOptions, client.DebugOptions
    assert not R().verify_checksum() and W().verify_checksum()
    assert R(ndebug=False).verify_checksum()  # debug builds always checksum
    assert R(enable_checksum=True).verify_checksum()
    assert not W(debug=D(bypass_disk_io=True)).verify_checksum()
    assert not W(ndebug=False, debug=D(bypass_rdma_xmit=True)).verify_checksum()
    cfg = client.ClientConfig(chunk_checksum_type=h3c.ChecksumType.CRC32)
    assert client.read_checksum_type(cfg, R(enable_checksum=True)) == int(h3c.ChecksumType.CRC32)
    assert client.read_checksum_type(cfg, R()) == int(h3c.ChecksumType.NONE)
    infos = client.write_checksums([b"abc", b"defg"], options=W(enable_checksum=False))
    assert [(int(i.type), i.value) for i in infos] == [(0, 0), (0, 0)]
    st = client.verify_read_checksums([(b"abc", 3, h3c.ChecksumInfo(h3c.ChecksumType.CRC32C, 1))], options=R())
    assert list(st) == [0]  # reads not verified by default
