"""HIP engine vs the CPU oracle, bit-exact (needs an MI355X).

Every call goes through the C ABI (include/h3c_crc.h) of _lib/libh3c_crc.so.
Sizes the oracle finishes in seconds are compared value-for-value; the full
BASELINE size (8192 x 1 MiB) is checked on a sample plus size-independent
properties (split-and-combine linearity, idempotence, bit-flip detection).
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as orc
from golden.gen_golden import materialize

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CRC_VECTORS = json.load(open(os.path.join(HERE, "golden", "crc_vectors.json")))
COMBINE_VECTORS = json.load(open(os.path.join(HERE, "golden", "combine_vectors.json")))
MASK = 0xFFFFFFFF
SEED = 20250629


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch, torch.device("cuda:0")


def to_dev(torch, dev, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).to(dev)


def test_golden_vectors_crc32c_and_crc32(h3c, torch_dev):
    torch, dev = torch_dev
    datas = [to_dev(torch, dev, materialize(c)) for c in CRC_VECTORS]
    items = [(d, c["len"], c["start"]) for d, c in zip(datas, CRC_VECTORS)]
    t, v = h3c.batch_create(items, h3c.ChecksumType.CRC32C)
    bad = [(c["name"], hex(int(x)), hex(c["crc32c_raw"])) for c, x in zip(CRC_VECTORS, v) if int(x) != c["crc32c_raw"]]
    assert not bad, bad[:10]
    assert all(int(x) == 1 for x in t)
    t, v = h3c.batch_create(items, h3c.ChecksumType.CRC32)
    bad = [(c["name"], hex(int(x)), hex(c["crc32_raw"])) for c, x in zip(CRC_VECTORS, v) if int(x) != c["crc32_raw"]]
    assert not bad, bad[:10]
    assert (~int(v[0])) & MASK == 0xCBF43926  # CRC-32 check value ("123456789")


def test_unaligned_ragged_windows(h3c, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, 48 << 20, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    items, want = [], []
    for i in range(600):
        kind = i % 4
        if kind == 0:
            n = int(rng.integers(0, 64))
        elif kind == 1:
            n = int(rng.integers(64, 4096))
        elif kind == 2:
            n = int(rng.integers(4096, 1 << 20))
        else:
            n = int(rng.integers(1 << 20, 5 << 20))
        off = int(rng.integers(0, host.size - n))
        start = int(rng.integers(0, 1 << 32)) if i % 3 else 0xFFFFFFFF
        items.append((buf[off: off + n], n, start))
        want.append(orc.crc32c(host[off: off + n], start))
    _, got = h3c.batch_create(items)
    mism = [i for i, (g, w) in enumerate(zip(got, want)) if int(g) != w]
    assert not mism, [(i, items[i][1]) for i in mism[:10]]


def test_chunk_size_classes(h3c, torch_dev):
    """The 11 chunk sizes of chunk_engine/src/types/constants.rs:3-8 (64 KiB .. 64 MiB)."""
    torch, dev = torch_dev
    sizes = [(64 << 10) << k for k in range(11)]
    datas = [orc.splitmix_bytes(n, SEED, k) for k, n in enumerate(sizes)]
    _, got = h3c.batch_create([to_dev(torch, dev, d) for d in datas])
    for n, d, g in zip(sizes, datas, got):
        assert int(g) == orc.crc32c(d), n


def test_verify_flags_exactly_the_flipped_chunks(h3c, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(5)
    n_chunks, clen = 400, 256 << 10
    host = rng.integers(0, 256, n_chunks * clen, dtype=np.uint8)
    expected = [orc.crc32c(host[i * clen:(i + 1) * clen]) for i in range(n_chunks)]
    flips = sorted(rng.choice(n_chunks, size=n_chunks // 20, replace=False).tolist())
    for c in flips:
        pos = c * clen + int(rng.integers(0, clen))
        host[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    buf = to_dev(torch, dev, host)
    items = [buf[i * clen:(i + 1) * clen] for i in range(n_chunks)]
    raw, ok, nbad = h3c.batch_verify(items, expected)
    assert nbad == len(flips)
    assert sorted(np.nonzero(~ok)[0].tolist()) == flips


def test_create_semantics_none_empty_null(h3c, torch_dev):
    torch, dev = torch_dev
    T = h3c.ChecksumType
    d = to_dev(torch, dev, np.frombuffer(b"123456789", dtype=np.uint8))
    items = [
        (d, 9, 0xFFFFFFFF, T.NONE),  # NONE -> {NONE, 0}
        (d, 0, 0xFFFFFFFF, T.CRC32C),  # empty -> {type, start}
        (d, 0, 0x12345678, T.CRC32C),
        (None, 10, 0xFFFFFFFF, T.CRC32C),  # null with length -> {NONE, 0}
        (None, 0, 0xFFFFFFFF, T.CRC32C),  # create(type, nullptr, 0) -> {type, ~0}
        (d, 9, 0xFFFFFFFF, T.CRC32C),
        (d, 9, 0xFFFFFFFF, T.CRC32),
    ]
    t, v = h3c.batch_create(items)
    assert [(int(a), int(b)) for a, b in zip(t, v)] == [
        orc.create(orc.NONE, b"123456789"),
        (1, 0xFFFFFFFF),
        (1, 0x12345678),
        orc.create(orc.CRC32C, None, 10),
        orc.create(orc.CRC32C, None, 0),
        (1, 0x1CF96D7C),
        (2, orc.crc32(b"123456789")),
    ]
    ci = h3c.ChecksumInfo.create(T.CRC32C, d)
    assert ci == h3c.ChecksumInfo(T.CRC32C, 0x1CF96D7C)


def test_host_payloads_staged(h3c, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(9)
    a = rng.integers(0, 256, (1 << 20) + 77, dtype=np.uint8)
    pinned = torch.from_numpy(a.copy()).pin_memory()
    _, v = h3c.batch_create([a, pinned, a.tobytes(), to_dev(torch, dev, a)])
    assert len(set(int(x) for x in v)) == 1 and int(v[0]) == orc.crc32c(a)


def test_device_batch_combine(h3c, torch_dev):
    torch, dev = torch_dev
    c1 = torch.from_numpy(np.array([v["c1"] for v in COMBINE_VECTORS], dtype=np.uint32).view(np.int32))
    c2 = torch.from_numpy(np.array([v["c2"] for v in COMBINE_VECTORS], dtype=np.uint32).view(np.int32))
    ln = torch.from_numpy(np.array([v["len2"] for v in COMBINE_VECTORS], dtype=np.int64))
    for ty, key in ((h3c.ChecksumType.CRC32C, "crc32c"), (h3c.ChecksumType.CRC32, "crc32")):
        out = torch.zeros_like(c1, device=dev)
        h3c.device_batch_combine(c1.to(dev), c2.to(dev), ln.to(dev), out, ty)
        got = (out.cpu().to(torch.int64) & MASK).tolist()
        assert got == [v[key] for v in COMBINE_VECTORS]


def test_plan_uniform_1024x1MiB_exact(h3c, torch_dev):
    """BASELINE config 1 shape (1024 x 1 MiB), every chunk checked."""
    torch, dev = torch_dev
    n, clen = 1024, 1 << 20
    buf = torch.empty(n * clen, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(buf, clen, n, clen, SEED)
    host = buf.cpu().numpy()
    assert np.array_equal(host[:4096], orc.splitmix_bytes(4096, SEED, 0))  # same generator on both sides
    want = np.zeros(n, dtype=np.uint32)
    orc.lib().orc_batch_crc32c(host.ctypes.data, clen, n, 0xFFFFFFFF, 8, 0, want.ctypes.data)
    plan = h3c.Plan.uniform(buf.data_ptr(), clen, n)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    plan.run(out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    # verify path on device
    exp = torch.from_numpy(want.view(np.int32)).to(dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    mis = torch.zeros(1, dtype=torch.int32, device=dev)
    plan.run(out, expected=exp, ok=ok, mismatch=mis)
    torch.cuda.synchronize()
    assert int(mis.item()) == 0 and bool(ok.bool().all())
    plan.close()


def test_full_size_8192x1MiB_properties(h3c, torch_dev):
    """BASELINE config 2 (8192 x 1 MiB device-resident): sample vs oracle + linearity + idempotence."""
    torch, dev = torch_dev
    n, clen = 8192, 1 << 20
    buf = torch.empty(n * clen, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(buf, clen, n, clen, SEED)
    plan = h3c.Plan.uniform(buf.data_ptr(), clen, n)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    plan.run(out)
    out2 = torch.zeros_like(out)
    plan.run(out2)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    got = out.cpu().numpy().view(np.uint32)
    for c in list(range(0, n, 257)) + [n - 1]:
        assert int(got[c]) == orc.crc32c(orc.splitmix_bytes(clen, SEED, c)), c
    # Split every chunk in halves (start 0 for the second half) and recombine on device.
    half = clen // 2
    lo = h3c.Plan.uniform(buf.data_ptr(), half, n, stride=clen)
    hi = h3c.Plan.uniform(buf.data_ptr() + half, half, n, stride=clen, start=0)
    a = torch.zeros(n, dtype=torch.int32, device=dev)
    b = torch.zeros(n, dtype=torch.int32, device=dev)
    lo.run(a)
    hi.run(b)
    comb = torch.zeros_like(a)
    h3c.device_batch_combine(a, b, torch.full((n,), half, dtype=torch.int64, device=dev), comb)
    torch.cuda.synchronize()
    assert torch.equal(comb, out)
    for p in (plan, lo, hi):
        p.close()
    del buf


def test_mixed_sizes_host_fed_shape(h3c, torch_dev):
    """BASELINE config 5 shapes: log-uniform 64 KiB..64 MiB, 10% ragged lengths."""
    torch, dev = torch_dev
    rng = np.random.default_rng(21)
    lens = []
    for i in range(48):
        n = (64 << 10) << int(rng.integers(0, 11))
        if i % 10 == 3:
            n -= int(rng.integers(1, 4000))
        lens.append(n)
    total = sum(lens)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    items, want, off = [], [], 0
    for n in lens:
        items.append(buf[off: off + n])
        want.append(orc.crc32c(host[off: off + n]))
        off += n
    _, got = h3c.batch_create(items)
    assert [int(x) for x in got] == want


def test_profile_counters(h3c, torch_dev):
    torch, dev = torch_dev
    buf = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    plan = h3c.Plan.uniform(buf.data_ptr(), 1 << 20, 64)
    out = torch.zeros(64, dtype=torch.int32, device=dev)
    h3c.profile_read(reset=True)
    h3c.profile_enable(True)
    plan.run(out)
    plan.run(out)
    h3c.profile_enable(False)
    ms, launches, nbytes = h3c.profile_read(reset=True)
    assert launches == 2 and nbytes == 2 * (64 << 20) and ms > 0
    torch.cuda.synchronize()
    assert (out.cpu().numpy().view(np.uint32) == (~0x14298C12) & MASK).all()  # 1 MiB of zeros
    plan.close()


@pytest.mark.parametrize("seg", [1024, 4096, 16384, 65536, 262144])
@pytest.mark.parametrize("dbg", [0, 1])
def test_forced_segment_sizes_and_paths(h3c, torch_dev, seg, dbg, hooks):
    """Every segment size and both row-loop paths (pipelined / single-row) agree with the oracle."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_SEG_BYTES, seg)
    hooks(h3c.HOOK_DEBUG_FLAGS, dbg)
    rng = np.random.default_rng(seg + dbg)
    sizes = [1, 17, 1024, 4096, 5120, 6144, 7168, 9216, 12345, 16384, 16385, 65543, 262144 + 1000,
             (1 << 20) + 3, 3 << 20]
    host = rng.integers(0, 256, sum(sizes) + 64, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    items, want, off = [], [], 5  # odd base offset: unaligned chunk starts
    for n in sizes:
        items.append((buf[off: off + n], n))
        want.append(orc.crc32c(host[off: off + n]))
        off += n
    _, got = h3c.batch_create(items)
    assert [int(x) for x in got] == want


@pytest.mark.parametrize("seg", [0, 65536])
def test_wave_fold_beyond_the_shift_tables(h3c, torch_dev, seg, hooks):
    """Chunks of > 16 segments are folded by a wave whose lanes shift their Horner sums by x^(8e)
    from the x4k / xb tables when e < 2^26 and by the square-and-multiply chain beyond: a 72 MiB
    chunk (1,152 segments of 64 KiB forced; lanes on both sides of 2^26) and ragged neighbours,
    against the oracle (seg 0: the plan's own segment pick)."""
    torch, dev = torch_dev
    if seg:
        hooks(h3c.HOOK_SEG_BYTES, seg)
    rng = np.random.default_rng(72 + seg)
    sizes = [(72 << 20) + 4093, (17 << 20) + 1, (1 << 20) * 3 + 11, 4096, 77]
    host = rng.integers(0, 256, sum(sizes) + 64, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    items, want, off = [], [], 3
    for n in sizes:
        items.append((buf[off: off + n], n))
        want.append(orc.crc32c(host[off: off + n]))
        off += n
    _, got = h3c.batch_create(items)
    assert [int(x) for x in got] == want


def test_none_type_chunks_among_multi_segment_folds(h3c, torch_dev, hooks):
    """NONE-type chunks long enough for many segments, beside chunks folded by both finalize mappings
    (thread per <= 16 segments, wave per more): {NONE, 0} for them, the oracle's value for the rest."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_SEG_BYTES, 65536)
    T = h3c.ChecksumType
    rng = np.random.default_rng(4242)
    sizes = [(3 << 20) + 5, (3 << 20) + 5, 700000, 700000, 65536 * 17 + 1, 65536 * 17 + 1, 333]
    kinds = [T.NONE, T.CRC32C, T.NONE, T.CRC32C, T.NONE, T.CRC32C, T.CRC32C]
    host = rng.integers(0, 256, sum(sizes) + 64, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    items, want, off = [], [], 1
    for n, k in zip(sizes, kinds):
        items.append((buf[off: off + n], n, 0xFFFFFFFF, k))
        want.append(orc.create(orc.NONE, host[off: off + n].tobytes()) if k == T.NONE else (1, orc.crc32c(host[off: off + n])))
        off += n
    t, v = h3c.batch_create(items)
    assert [(int(a), int(b)) for a, b in zip(t, v)] == want


@pytest.mark.parametrize("flags", ["0", "2"])
def test_small_chunk_batches(h3c, torch_dev, hooks, flags):
    """Batches whose every chunk is one short segment run seg_small_kernel (flags 0); flags 2
    (H3C_DEBUG_FLAGS bit1) forces the general kernel on the same batches.  Sizes 1 B..7 KiB at
    every alignment, device-resident and host-staged, create and verify."""
    hooks(h3c.HOOK_DEBUG_FLAGS, int(flags, 0))
    torch, dev = torch_dev
    rng = np.random.default_rng(41)
    host = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    for trial in range(3):
        n = [1, 700, 5000][trial]
        items, want, hitems = [], [], []
        for _ in range(n):
            ln = int(rng.choice([1, 15, 16, 17, 1023, 1024, 1025, 4096, int(rng.integers(1, 7 * 1024))]))
            off = int(rng.integers(0, (8 << 20) - ln))
            items.append((buf[off: off + ln], ln))
            hitems.append((host[off: off + ln], ln))
            want.append(orc.crc32c(host[off: off + ln]))
        t, v = h3c.batch_create(items)
        assert [int(x) for x in v] == want
        exp = list(want)
        bad = sorted(set(int(x) for x in rng.integers(0, n, max(1, n // 50))))
        for b in bad:
            exp[b] ^= 0x1000
        raw, ok, nbad = h3c.batch_verify(items, exp)
        assert nbad == len(bad) and sorted(np.nonzero(~ok)[0].tolist()) == bad
        t, v = h3c.batch_create(hitems[:300])  # host-staged copies (own alignment)
        assert [int(x) for x in v] == want[:300]
    # a device plan of 4 KiB chunks (the small kernel on the asynchronous path)
    plan = h3c.Plan.uniform(buf.data_ptr(), 4096, 2048)
    out = torch.zeros(2048, dtype=torch.int32, device=dev)
    plan.run(out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    for k in range(0, 2048, 97):
        assert int(got[k]) == orc.crc32c(host[k * 4096:(k + 1) * 4096])
    plan.close()


def test_plan_verify_4mib_chunks_config4_shape(h3c, torch_dev):
    """BASELINE config 4's chunk size in one process: 64 x 4 MiB splitmix chunks through a
    device-resident Plan verify, with flips at the first, last and middle bytes; every chunk's
    raw checksum and ok flag against the oracle."""
    torch, dev = torch_dev
    n, clen, seed = 64, 4 << 20, 404
    buf = torch.empty(n * clen, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(buf, clen, n, clen, seed)
    expected = np.array([orc.crc32c(orc.splitmix_bytes(clen, seed, c)) for c in range(n)], dtype=np.uint32)
    flips = {0: 0, 9: clen - 1, 33: clen // 2 + 5}
    want = expected.copy()
    for c, off in flips.items():
        buf[c * clen + off] = buf[c * clen + off] ^ 0x40
        d = orc.splitmix_bytes(clen, seed, c)
        d[off] ^= 0x40
        want[c] = orc.crc32c(d)
    plan = h3c.Plan.uniform(buf.data_ptr(), clen, n)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    mis = torch.zeros(1, dtype=torch.int32, device=dev)
    plan.run(out, expected=torch.from_numpy(expected.view(np.int32)).to(dev), ok=ok, mismatch=mis)
    torch.cuda.synchronize()
    plan.close()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == sorted(flips)
    assert int(mis.item()) == len(flips)


@pytest.mark.parametrize("flags", ["0", "4"])
@pytest.mark.parametrize("clen", [64, 1024, 4096, 6144, 8192, 12288])
def test_uniform_small_chunk_batches(h3c, torch_dev, hooks, flags, clen):
    """Uniform batches (one length, row-aligned, one start) run seg_uni_kernel (flags 0); flags 4
    (H3C_DEBUG_FLAGS bit2) forces seg_quad_kernel on the same batches.  Contiguous plans (no
    descriptors), strided plans, scattered aligned buffers and a verify with flips; a batch
    that is almost uniform (one odd length) must take the general small kernel correctly."""
    hooks(h3c.HOOK_DEBUG_FLAGS, int(flags, 0))
    torch, dev = torch_dev
    rng = np.random.default_rng(clen)
    n = 3001
    size = max(16 << 20, n * (clen + 4096))  # room for the strided plan below
    host = rng.integers(0, 256, size, dtype=np.uint8)
    buf = to_dev(torch, dev, host)
    for stride in (clen, clen + 4096):
        assert (n - 1) * stride + clen <= size
        plan = h3c.Plan.uniform(buf.data_ptr(), clen, n, stride=stride)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        exp = np.array([orc.crc32c(host[k * stride: k * stride + clen]) for k in range(n)], dtype=np.uint32)
        flips = sorted(set(int(x) for x in rng.integers(0, n, 20)))
        bad = exp.copy()
        bad[flips] ^= 0x80
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        plan.run(out, expected=torch.from_numpy(bad.view(np.int32)).to(dev), ok=ok)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
        assert np.nonzero(ok.cpu().numpy() == 0)[0].tolist() == flips
        plan.close()
    # scattered row-aligned buffers (descriptors, not contiguous), then one odd length
    offs = sorted(int(x) * 256 for x in rng.choice((16 << 20) // 256 - 64, 700, replace=False))
    items = [(buf[o: o + clen], clen) for o in offs]
    want = [orc.crc32c(host[o: o + clen]) for o in offs]
    t, v = h3c.batch_create(items)
    assert [int(x) for x in v] == want
    items[5] = (buf[offs[5]: offs[5] + clen - 1], clen - 1)
    want[5] = orc.crc32c(host[offs[5]: offs[5] + clen - 1])
    t, v = h3c.batch_create(items)
    assert [int(x) for x in v] == want


@pytest.mark.parametrize("n", [1, 7, 17, 63, 300, 4097])
def test_uniform_small_chunk_counts(h3c, torch_dev, n):
    """seg_uni_kernel's waves take steps from a per-workgroup counter: batches smaller than a
    step, than a wave's worth of groups and than the grid, and one just past a grid multiple."""
    torch, dev = torch_dev
    rng = np.random.default_rng(n)
    for clen in (4096, 1024):
        host = rng.integers(0, 256, n * clen, dtype=np.uint8)
        buf = to_dev(torch, dev, host)
        plan = h3c.Plan.uniform(buf.data_ptr(), clen, n)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        plan.run(out)
        torch.cuda.synchronize()
        exp = np.array([orc.crc32c(host[k * clen:(k + 1) * clen]) for k in range(n)], dtype=np.uint32)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), exp), (n, clen)
        plan.close()



def test_plan_extent_is_checked_before_launch(h3c, torch_dev):
    """a plan whose layout runs past its buffer is rejected with kInvalidArg
    before any upload or launch -- by Plan.uniform against the tensor's (or a given) extent, and
    by h3c_plan_create against the HIP allocation holding each descriptor.  Nothing here is ever
    run: only plan creation is attempted."""
    torch, dev = torch_dev
    buf = torch.zeros(16 << 20, dtype=torch.uint8, device=dev)
    with pytest.raises(h3c.EngineError) as e:
        h3c.Plan.uniform(buf, 4096, 3001, stride=8192)  # 24 MiB > 16 MiB
    assert e.value.code == h3c.StatusCode.kInvalidArg
    with pytest.raises(h3c.EngineError):
        h3c.Plan.uniform(buf.data_ptr(), 4096, 2049, extent=8 << 20)
    h3c.Plan.uniform(buf, 4096, 4096).close()  # exactly the buffer: fine
    # library level: a descriptor ending 400 GiB past its allocation (beyond any HBM)
    d = np.zeros(2, dtype=h3c.engine.DESC_DTYPE)
    d["ptr"] = [buf.data_ptr(), buf.data_ptr() + (8 << 20)]
    d["len"] = [4096, 400 << 30]
    d["start_raw"] = 0xFFFFFFFF
    d["type"] = 1
    with pytest.raises(h3c.EngineError) as e:
        h3c.Plan(d, dev.index or 0)
    assert e.value.code == h3c.StatusCode.kInvalidArg and "past the end" in str(e.value)
    # the synchronous batch path checks device payloads the same way (and launches nothing)
    d["mem"] = 0
    out_t, out_v = np.zeros(2, dtype=np.uint8), np.zeros(2, dtype=np.uint32)
    rc = h3c.engine.lib.h3c_batch_create(d.ctypes.data, 2, out_t.ctypes.data, out_v.ctypes.data, None)
    assert rc == h3c.StatusCode.kInvalidArg
