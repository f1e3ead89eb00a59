"""GPU parity of the adjacent formats and consumers: calcSerde, the Rust crc32c crate API,
the client's write / read-verify checksums, and the scrub (recalculate) pass."""
import importlib

import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu
MASK = 0xFFFFFFFF


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def fm(h3c):
    return importlib.import_module("3fs_amd.formats")


def serde_oracle(data, compressed):
    """Checksum::calcSerde (MessageHeader.h:32-37): folly::crc32c(data, size, 0) + low-byte mark."""
    crc0 = orc.crc32c(data, start=0)
    return (crc0 & ~0xFF) | 0x86 | int(compressed)


def test_serde_checksum_batch_and_verify(h3c, fm, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(1)
    msgs = [rng.integers(0, 256, n, dtype=np.uint8) for n in (0, 1, 8, 63, 64, 1000, 4096 + 5, 70000)]
    comp = [i % 2 for i in range(len(msgs))]
    got = fm.batch_serde_checksum(msgs, comp)
    want = [serde_oracle(m, c) for m, c in zip(msgs, comp)]
    assert [int(x) for x in got] == want
    # device-resident messages, single-message API
    assert fm.Checksum.calc_serde(torch.from_numpy(msgs[5]).to(dev), True) == want[5] | 1
    # receive side: corrupt one message and one header flag
    rec = list(want)
    bad_msgs = [m.copy() for m in msgs]
    bad_msgs[6][100] ^= 1
    rec[3] ^= 0x100  # a CRC bit of the header
    rec[4] ^= 1      # the compressed flag: not covered (the receiver takes it from the header, Processor.h:114)
    ok, nbad = fm.batch_serde_verify(bad_msgs, rec)
    assert nbad == 2 and not ok[6] and not ok[3] and ok[[0, 1, 2, 4, 5, 7]].all()


def test_rust_crc32c_crate_api(h3c, fm, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(2)
    for n in (0, 1, 15, 16, 17, 1023, 1 << 20, (1 << 20) + 3):
        a = rng.integers(0, 256, n, dtype=np.uint8)
        b = rng.integers(0, 256, int(rng.integers(0, 9000)), dtype=np.uint8)
        std_a = (~orc.crc32c(a)) & MASK
        assert fm.rust_crc32c.crc32c(torch.from_numpy(a).to(dev)) == std_a
        # crc32c_append(crc32c(a), b) == crc32c(a ++ b)  (chunk.rs:213,266-269)
        assert fm.rust_crc32c.crc32c_append(std_a, b) == (~orc.crc32c(np.concatenate([a, b]))) & MASK
    # engine.rs:1004 pattern: constant i as u8 chunks
    for i in (0, 7, 255):
        buf = np.full(64 << 10, i, dtype=np.uint8)
        assert fm.rust_crc32c.crc32c(buf) == (~orc.crc32c(buf)) & MASK


def test_client_write_and_read_verify(h3c, torch_dev):
    torch, dev = torch_dev
    client = importlib.import_module("3fs_amd.client")
    rng = np.random.default_rng(3)
    datas = [rng.integers(0, 256, n, dtype=np.uint8) for n in (1, 4096, 65536, 1 << 20, 333)]
    infos = client.write_checksums(datas)
    for d, ck in zip(datas, infos):
        assert ck.type == h3c.ChecksumType.CRC32C and ck.value == orc.crc32c(d)
    # read results: (data, length, server checksum); corrupt #1, short-length #2, NONE server type #3
    dev_datas = [torch.from_numpy(d).to(dev) for d in datas]
    results = [(dev_datas[i], datas[i].size, infos[i]) for i in range(len(datas))]
    bad = dev_datas[1].clone()
    bad[7] ^= 0xFF
    results[1] = (bad, datas[1].size, infos[1])
    results[2] = (dev_datas[2], 1000, h3c.ChecksumInfo(h3c.ChecksumType.CRC32C, orc.crc32c(datas[2][:1000])))
    results[3] = (dev_datas[3], datas[3].size, h3c.ChecksumInfo(h3c.ChecksumType.NONE, 0))
    results.append((dev_datas[0], 0, h3c.ChecksumInfo(h3c.ChecksumType.CRC32C, 12345)))  # length 0: skipped
    st = client.verify_read_checksums(results)
    assert list(st) == [0, client.kChecksumMismatch, 0, 0, 0, 0]


def test_scrub_finds_corrupted_chunks(h3c, torch_dev):
    torch, dev = torch_dev
    scrub = importlib.import_module("3fs_amd.scrub")
    n, cl = 64, 256 << 10
    slab = torch.empty(n * cl, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(slab, cl, n, cl, 20250629)
    host = slab.cpu().numpy().reshape(n, cl)
    stored = []
    for c in range(n):
        if c % 9 == 4:
            stored.append(h3c.ChecksumInfo(h3c.ChecksumType.NONE, 0))
        else:
            stored.append(h3c.ChecksumInfo(h3c.ChecksumType.CRC32C, orc.crc32c(host[c])))
    chunks = [(slab.data_ptr() + c * cl, cl, stored[c]) for c in range(n)]
    s = scrub.Scrubber(chunks)
    assert s.run() == []
    for c, pos in ((3, 0), (17, cl - 1), (41, 12345), (4, 99)):  # chunk 4 is NONE: not detected
        slab[c * cl + pos] ^= 0x40
    assert s.run() == [3, 17, 41]
    rec = s.recomputed()
    assert rec[17] == orc.crc32c(slab[17 * cl:18 * cl].cpu().numpy())
    s.close()
    differ, only_l, only_r = scrub.diff_checksums({1: stored[1], 2: stored[2], 5: stored[5]},
                                                  {1: stored[1], 2: stored[3], 6: stored[6]})
    assert differ == [2] and only_l == [5] and only_r == [6]


def test_read_results_match_setresult_oracle(h3c, torch_dev):
    """AioReadJob::setResult (BatchReadJob.cc:24-55): NONE batch, whole-chunk reuse, partial
    read checksum, recalculate verify (stored value corrupt -> 4080)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(6)
    jobs, want = [], []
    for k in range(60):
        cl = int(rng.integers(1, 300000))
        chunk = rng.integers(0, 256, cl, dtype=np.uint8)
        ctype = [orc.CRC32C, orc.CRC32, orc.NONE][k % 3]
        stored = orc.create(ctype, chunk)[1] if ctype else 0
        if k % 7 == 3:
            stored ^= 0x8  # corrupt stored checksum
        full_read = k % 2 == 0
        off = 0 if full_read else int(rng.integers(0, cl))
        ln = cl if full_read else int(rng.integers(0, cl - off + 1))
        data = chunk[off:off + ln]
        bt = [orc.CRC32C, orc.CRC32C, orc.CRC32, orc.NONE][k % 4]
        recalc = k % 5 != 1
        want.append(orc.read_result_checksum(bt, ctype, stored, cl, off, ln, data, recalc, chunk))
        dd = torch.from_numpy(np.ascontiguousarray(data)).to(dev) if k % 3 else np.ascontiguousarray(data)
        jobs.append((bt, (dd, ln, cl, off, h3c.ChecksumInfo(h3c.ChecksumType(ctype), stored), recalc)))
    for bt in (orc.NONE, orc.CRC32C, orc.CRC32):
        idx = [i for i, (b, _) in enumerate(jobs) if b == bt]
        ctr = {}
        infos, st = h3c.read_results(bt, [jobs[i][1] for i in idx], counters=ctr)
        for k, i in enumerate(idx):
            rc, t, v = want[i]
            assert (int(st[k]), int(infos[k].type), infos[k].value) == (rc, t, v), i
        # storage.aio.checksum_mismatch (BatchReadJob.cc:14, :46): one per 4080
        assert ctr["checksum_mismatch"] == sum(1 for i in idx if want[i][0] == 4080)
    assert any(w[0] == 4080 for w in want)


def test_scalar_folly_shaped_entry_points(h3c, torch_dev):
    """h3c_crc32c / h3c_crc32: folly::crc32c / crc32 (Common.h:158,161) for one buffer,
    host or device memory detected by pointer attributes."""
    torch, dev = torch_dev
    rng = np.random.default_rng(8)
    for n in (0, 1, 9, 4096, 100003):
        a = rng.integers(0, 256, n, dtype=np.uint8)
        for start in (0xFFFFFFFF, 0, 0xABCDEF01):
            assert h3c.crc32c(a, start) == orc.crc32c(a, start)
            assert h3c.crc32c(torch.from_numpy(a).to(dev), start) == orc.crc32c(a, start)
            assert h3c.crc32(a, start) == orc.crc32(a, start)
    assert (~h3c.crc32c(b"123456789")) & MASK == 0xE3069283


def test_create_over_data_iterator(h3c, torch_dev):
    """ChecksumInfo::create(type, DataIterator*, length, start) (Common.h:120-172): the 1 MiB
    MemoryDataIterator, ragged pieces (ChunkFileView's preads), and byte counts that do not
    add up (a short read, or a last piece past `length`) -> {NONE, 0}."""
    torch, dev = torch_dev
    CI, T = h3c.ChecksumInfo, h3c.ChecksumType
    rng = np.random.default_rng(146)
    n = (3 << 20) + 4321
    host = rng.integers(0, 256, n, dtype=np.uint8)
    buf = torch.from_numpy(host).to(dev)
    for t, ref in ((T.CRC32C, orc.crc32c), (T.CRC32, orc.crc32)):
        want = ref(host, 0x1234567)
        got = CI.create_from_iterator(t, CI.memory_data_iterator(buf, n), n, 0x1234567)
        assert (got.type, got.value) == (t, want)
        cuts = [0, 1, 4097, 4097, (1 << 20) + 5, n]  # a zero-size piece in the middle
        pieces = [(buf[a:b], b - a) for a, b in zip(cuts, cuts[1:])] + [(None, 0)]
        got = CI.create_from_iterator(t, iter(pieces), n, 0x1234567)
        assert (got.type, got.value) == (t, want)
        short = [(buf[:1000], 1000), (None, 0)]
        assert CI.create_from_iterator(t, iter(short), 2000) == CI(T.NONE, 0)
        over = [(buf[:1000], 1000), (buf[1000:2000], 1000), (None, 0)]
        assert CI.create_from_iterator(t, iter(over), 1500) == CI(T.NONE, 0)
        assert CI.create_from_iterator(t, iter([(None, 0)]), 0, 77) == CI(t, 77)
    assert CI.create_from_iterator(T.NONE, iter([(buf, n)]), n) == CI(T.NONE, 0)


@pytest.mark.parametrize("n", [0, 1, 15, 4096, 65537, 1 << 20])
def test_folly_signature_entries_match_oracle(h3c, torch_dev, n):
    """h3c_folly_crc32c / h3c_folly_crc32: folly::crc32c / crc32's own signature (Common.h:158,161)
    and raw-register result, on device and host buffers, against the CPU oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(n + 7)
    host = rng.integers(0, 256, size=n, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    torch.cuda.synchronize()
    lib = h3c.engine.lib
    for start in (MASK, 0, 0x12345678):
        dptr = d.data_ptr() if n else None
        assert lib.h3c_folly_crc32c(dptr, n, start) == orc.crc32c(host, start), (n, start)
        assert lib.h3c_folly_crc32c(host.ctypes.data if n else None, n, start) == orc.crc32c(host, start)
        assert lib.h3c_folly_crc32(dptr, n, start) == orc.crc32(host, start), (n, start)
