"""Seeded fuzz of the batch entry points against the oracle's ChecksumInfo::create
(Common.h:146-177): every batch mixes polynomials (CRC32C, CRC32, NONE), starting values,
memory kinds (device, pinned, pageable, null) and lengths from 0 through the small-chunk
kernel's range to multi-segment chunks, at random alignments -- so one batch exercises the
general and small-chunk kernels, host staging and the NONE / empty / null cases together.
Also the asynchronous plan path over the same descriptors, and verify with flipped values."""
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


def random_batch(rng, n, pool_bytes, small_only=0):
    """n descriptors (offset, length, type, start, mem) into a pool of pool_bytes; with
    small_only, lengths up to that many bytes, all device-resident and typed (a batch the
    small-chunk kernel takes whole: 8-lane groups up to ~5 KiB, 16-lane groups above)."""
    out = []
    for _ in range(n):
        u = rng.random()
        if small_only:
            ln = int(rng.integers(1, small_only + 1))
        elif u < 0.45:
            ln = int(rng.integers(1, 16 << 10))
        elif u < 0.55:
            ln = 0
        elif u < 0.9:
            ln = int(rng.integers(16 << 10, 1 << 20))
        else:
            ln = int(rng.integers(1 << 20, 9 << 20))
        off = int(rng.integers(0, pool_bytes - ln))
        # CRC32C mostly, some CRC32 and NONE (a NONE chunk keeps its polynomial group on the
        # general kernel, so the small-only batches leave it out)
        t = int(rng.choice([1, 1, 2] if small_only else [1, 1, 1, 2, 0]))
        start = int(rng.choice([0xFFFFFFFF, 0, int(rng.integers(0, 1 << 32))]))
        mem = "dev" if small_only else str(rng.choice(["dev", "dev", "dev", "pinned", "pageable", "null"]))
        out.append((off, ln, t, start, mem))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fuzz_mixed_batches_create_and_verify(h3c, torch_dev, seed):
    torch, dev = torch_dev
    rng = np.random.default_rng(1000 + seed)
    pool = 24 << 20
    host = rng.integers(0, 256, pool, dtype=np.uint8)
    dbuf = torch.from_numpy(host).to(dev)
    pinned = torch.from_numpy(host).pin_memory()
    for small_only in (0, 4096, 8192):
        batch = random_batch(rng, 300, pool, small_only)
        items, want = [], []
        for off, ln, t, start, mem in batch:
            if mem == "null":
                items.append((None, ln, start, t))
                want.append(orc.create(t, None, ln, start))
                continue
            src = {"dev": dbuf, "pinned": pinned, "pageable": host}[mem]
            items.append((src[off: off + ln], ln, start, t))
            want.append(orc.create(t, host[off: off + ln], ln, start))
        types, vals = h3c.batch_create(items)
        got = [(int(a), int(b)) for a, b in zip(types, vals)]
        assert got == want, [(i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w][:5]
        # verify: flip ~5 % of the expected values; exactly those fail
        exp = [w[1] for w in want]
        bad = sorted(set(int(x) for x in rng.integers(0, len(items), 15)))
        for b in bad:
            exp[b] ^= 1 << int(rng.integers(0, 32))
        raw, ok, nbad = h3c.batch_verify(items, exp)
        assert sorted(np.nonzero(~ok)[0].tolist()) == bad and nbad == len(bad)


def test_fuzz_device_plan_matches_batch(h3c, torch_dev):
    """The asynchronous plan (h3c_plan_create / run) over device descriptors of mixed sizes
    and both polynomials gives the synchronous batch's values."""
    torch, dev = torch_dev
    rng = np.random.default_rng(77)
    pool = 24 << 20
    host = rng.integers(0, 256, pool, dtype=np.uint8)
    dbuf = torch.from_numpy(host).to(dev)
    for small_only in (0, 4096, 8192):
        batch = [b for b in random_batch(rng, 400, pool, small_only) if b[4] == "dev" and b[2] != 0]
        d = np.zeros(len(batch), dtype=h3c.engine.DESC_DTYPE)
        for i, (off, ln, t, start, _) in enumerate(batch):
            d[i] = (dbuf.data_ptr() + off, ln, start, t, 0, 0)
        plan = h3c.Plan(d, 0)
        out = torch.zeros(len(batch), dtype=torch.int32, device=dev)
        plan.run(out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        plan.close()
        for i, (off, ln, t, start, _) in enumerate(batch):
            assert int(got[i]) == orc.create(t, host[off: off + ln], ln, start)[1], i


@pytest.mark.parametrize("maxlen", [5000, 15000])
def test_small_kernel_many_groups_per_wave(h3c, torch_dev, maxlen):
    """300k ragged small chunks in one plan: each wave of the small-chunk kernel walks
    several 64-chunk descriptor groups, so the next group's descriptors and first rows are
    fetched across group boundaries.  Lengths up to ~5 KiB take the 4-lane groups, up to
    16 rows of 1 KiB the 16-lane groups; random offsets, starting values, and a verify pass with a
    few flipped expected values."""
    torch, dev = torch_dev
    rng = np.random.default_rng(500 + maxlen)
    pool = 64 << 20
    host = rng.integers(0, 256, pool, dtype=np.uint8)
    dbuf = torch.from_numpy(host).to(dev)
    n = 300_000
    lens = rng.integers(1, maxlen + 1, n).astype(np.uint64)
    offs = (rng.random(n) * (pool - lens)).astype(np.uint64)
    starts = rng.choice(np.array([0xFFFFFFFF, 0, 0x12345678], dtype=np.uint32), n)
    d = np.zeros(n, dtype=h3c.engine.DESC_DTYPE)
    d["ptr"] = np.uint64(dbuf.data_ptr()) + offs
    d["len"] = lens
    d["start_raw"] = starts
    d["type"] = int(h3c.ChecksumType.CRC32C)
    d["mem"] = int(h3c.engine.MemKind.DEVICE)
    base = host.ctypes.data
    f = orc.lib().orc_crc32c_sse42
    want = np.array([f(base + int(o), int(ln), int(s)) for o, ln, s in zip(offs, lens, starts)], dtype=np.uint32)
    plan = h3c.Plan(d, 0)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    plan.run(out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad_at = np.nonzero(got != want)[0]
    assert bad_at.size == 0, (bad_at[:5].tolist(), bad_at.size)
    exp = want.copy()
    flip = np.unique(rng.integers(0, n, 40))
    exp[flip] ^= np.uint32(1 << 7)
    exp_t = torch.from_numpy(exp.view(np.int32)).to(dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    mism = torch.zeros(1, dtype=torch.int32, device=dev)
    plan.run(out, expected=exp_t, ok=ok, mismatch=mism)
    torch.cuda.synchronize()
    plan.close()
    assert np.array_equal(np.nonzero(ok.cpu().numpy() == 0)[0], flip)
    assert int(mism.item()) == flip.size
