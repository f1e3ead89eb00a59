"""h3c_multi_* on the GPU: one process, one worker thread per listed device, against the oracle.

The box has one MI355X, so the engine is built over devices {0, 0}: two workers on the one GPU,
each with its own stream, plan and host-fed pipeline -- every line of the split / run / scatter
path runs as it does over 8 GPUs (the device-routing rule is exercised by placing payloads on the
device both workers share).  What each test pins:

* a mixed batch (device, pinned host through the workers' H2D pipelines, pageable host, NONE,
  null, empty, CRC32) through h3c_multi_batch_create / h3c_multi_verify equals the oracle's
  ChecksumInfo::create (Common.h:146-177) and flags exactly the corrupted expectations;
* h3c_multi_plan_* (the resync scrub shape, BatchReadJob.cc:43-54) over a resident 1 MiB set and a
  mixed-size one, results written in place through the workers' pinned mirrors;
* h3c_multi_update_ios over a random mix of WRITE / TRUNCATE / EXTEND / invalid ops equals the
  ChunkReplica::update replay (ChunkReplica.cc:131-394) op by op, chunk bytes and counters included.

Config 3 at full shape through the multi engine is in test_gpu_config3.py.
"""
import importlib

import numpy as np
import pytest

import oracle_lib as orc
import test_gpu_updio as tu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def multi(h3c, torch_dev):
    m = h3c.Multi([0, 0])
    yield m
    m.close()


def test_multi_mixed_batch_create_and_verify(h3c, torch_dev, multi):
    torch, dev = torch_dev
    rng = np.random.default_rng(606)
    items, want = [], []
    hb = h3c.HostBuffer(0, 40 << 20)  # pinned, NUMA-local: 36 MiB of it goes through the H2D pipelines
    try:
        off = 0
        for k in range(36):
            n = (1 << 20) - int(rng.integers(0, 3)) * 17
            a = hb.array[off:off + n]
            a[:] = rng.integers(0, 256, n, dtype=np.uint8)
            items.append(a)
            want.append((orc.CRC32C, orc.crc32c(a)))
            off += n + 64
        for n in (0, 1, 15, 1023, 4096 + 3, 65536, (1 << 20) + 13, 3 << 20):
            h = rng.integers(0, 256, n, dtype=np.uint8)
            items.append(torch.from_numpy(h).to(dev))
            want.append((orc.CRC32C, orc.crc32c(h)))
            items.append((torch.from_numpy(h.copy()).to(dev), None, 0xFFFFFFFF, orc.CRC32))
            want.append((orc.CRC32, orc.crc32(h)))
            items.append(h.copy())  # pageable host
            want.append((orc.CRC32C, orc.crc32c(h)))
        items.append((None, 4096))  # a null payload with a length: ChecksumInfo {NONE, 0}
        want.append((orc.NONE, 0))
        items.append((torch.zeros(64, dtype=torch.uint8, device=dev), None, 0xFFFFFFFF, orc.NONE))
        want.append((orc.NONE, 0))
        items.append((torch.arange(100, dtype=torch.uint8, device=dev), None, 0x12345678))  # a start value
        want.append((orc.CRC32C, orc.crc32c(np.arange(100, dtype=np.uint8), 0x12345678)))
        # single-engine answer for the same descriptors
        t1, v1 = h3c.batch_create(items)
        types, raws = multi.batch_create(items)
        assert types.tolist() == [w[0] for w in want]
        assert raws.tolist() == [w[1] for w in want]
        assert t1.tolist() == types.tolist() and v1.tolist() == raws.tolist()
        stats = multi.last_stats()
        assert len(stats) == 2 and all(u > 0 for u, _, _ in stats), stats
        exp = raws.copy()
        bad = sorted(rng.choice(len(items), 9, replace=False).tolist())
        for b in bad:
            exp[b] ^= 1 << int(rng.integers(0, 32))
        out, ok, nbad = multi.verify(items, exp)
        assert out.tolist() == raws.tolist()
        assert sorted(np.nonzero(~ok)[0].tolist()) == bad and nbad == len(bad)
        r1, ok1, n1 = h3c.batch_verify(items, exp)
        assert ok1.tolist() == ok.tolist() and n1 == nbad
    finally:
        hb.close()


def test_multi_plan_resident_set_with_flips(h3c, torch_dev, multi):
    torch, dev = torch_dev
    n, cl = 512, 1 << 20
    slab = torch.empty(n * cl, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(slab, cl, n, cl, 20250629)
    torch.cuda.synchronize()
    host = slab.cpu().numpy()
    want = np.zeros(n, dtype=np.uint32)
    orc.lib().orc_batch_crc32c(host.ctypes.data, cl, n, 0xFFFFFFFF, 16, 0, want.ctypes.data)
    eng = importlib.import_module("3fs_amd.engine")
    d = np.zeros(n, dtype=eng.DESC_DTYPE)
    d["ptr"] = slab.data_ptr() + np.arange(n, dtype=np.uint64) * np.uint64(cl)
    d["len"] = cl
    d["start_raw"] = 0xFFFFFFFF
    d["type"] = orc.CRC32C
    d["mem"] = 0
    plan = multi.plan(d)
    try:
        assert plan.verify(want) == 0 and plan.ok.all() and np.array_equal(plan.out, want)
        stats = multi.last_stats()
        assert [s[0] for s in stats] == [256, 256] and [s[1] for s in stats] == [256 * cl] * 2
        exp = want.copy()
        flips = [0, 1, 255, 256, 511]
        exp[flips] ^= 0x80
        assert plan.verify(exp) == len(flips)
        assert sorted(np.nonzero(plan.ok == 0)[0].tolist()) == flips
        assert np.array_equal(plan.out, want)
        # expected values change from call to call: nothing of the previous call's may be seen
        assert plan.verify(want) == 0 and plan.ok.all()
        exp = want.copy()
        exp[[3, 300]] ^= 1
        assert plan.verify(exp) == 2 and sorted(np.nonzero(plan.ok == 0)[0].tolist()) == [3, 300]
    finally:
        plan.close()


def test_multi_plan_mixed_sizes_in_place(h3c, torch_dev, multi):
    """A resident set of mixed, ragged, unaligned chunks (one segment each up to many: the segment
    kernel, both finalize mappings and the small-chunk kernels write their results straight into the
    workers' pinned mirrors), NONE-type chunks among them, verified three times with changing
    expectations against the oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(919)
    sizes = [int(x) for x in rng.choice([777, 4096, 65536 + 3, 300000, (1 << 20) + 11, (3 << 20) - 5, 9 << 20], 160)]
    kinds = [orc.NONE if i % 13 == 5 else orc.CRC32C for i in range(len(sizes))]
    host = rng.integers(0, 256, sum(sizes) + 64, dtype=np.uint8)
    buf = torch.from_numpy(host).to(dev)
    eng = importlib.import_module("3fs_amd.engine")
    d = np.zeros(len(sizes), dtype=eng.DESC_DTYPE)
    offs = 7 + np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    d["ptr"] = np.uint64(buf.data_ptr()) + offs
    d["len"] = sizes
    d["start_raw"] = 0xFFFFFFFF
    d["type"] = kinds
    d["mem"] = 0
    want = np.array([orc.create(k, host[o: o + n].tobytes())[1] for k, o, n in zip(kinds, offs.tolist(), sizes)],
                    dtype=np.uint32)
    plan = multi.plan(d)
    try:
        assert plan.verify(want) == 0 and plan.ok.all() and np.array_equal(plan.out, want)
        for flips in ([0, 17, 159], [5, 18, 40, 41]):
            exp = want.copy()
            exp[flips] ^= 0x10000
            assert plan.verify(exp) == len(flips)
            assert sorted(np.nonzero(plan.ok == 0)[0].tolist()) == flips
            assert np.array_equal(plan.out, want)
    finally:
        plan.close()


@pytest.mark.parametrize("seed", [7, 8])
def test_multi_update_ios_matches_replica_replay(h3c, torch_dev, multi, seed):
    torch, dev = torch_dev
    rng = np.random.default_rng(seed)
    sc = tu.random_scenario(h3c, torch, dev, rng, nchunks=9, chunk_size=64 << 10, nops=1500)
    sc.add(orc.UPD_WRITE, 9, 0, 16)  # a chunk index past the table: kInvalidArg on worker 0
    chunks, ios = sc.device_ios()
    sc.counters = h3c.UpdateCounters()
    res = multi.update_ios(chunks, ios, counters=sc.counters)
    torch.cuda.synchronize()
    sc.check(chunks, res)
    units = [s[0] for s in multi.last_stats()]
    assert sum(units) == len(ios) and min(units) > 0


def test_multi_update_ios_exact_aligned_with_stale_chunks(h3c, torch_dev, multi):
    """H3C_UPD_EXACT through h3c_multi_update_ios: an aligned batch (each worker's share runs the aligned
    sub-branch after its chunks' piece pass) on chunks whose stored checksums are partly stale; results,
    states and the summed stale count against the ChunkReplica::update replay."""
    from test_gpu_updio_aligned import aligned_scenario

    torch, dev = torch_dev
    rng = np.random.default_rng(61)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=10, chunk_size=128 << 10, nops=1500, stale=0.6,
                          full_size=False)
    chunks, ios = sc.device_ios()
    sc.counters = h3c.UpdateCounters()
    before = h3c.diag_counters()
    res = multi.update_ios(chunks, ios, exact=True, counters=sc.counters)
    torch.cuda.synchronize()
    diag = {k: v - before[k] for k, v in h3c.diag_counters().items()}
    sc.check(chunks, res)
    assert sc.stale_chunks > 0 and int(sc.counters.stale_chunks) == sc.stale_chunks
    assert diag["aligned_batches"] == 2 and diag["aligned_abandoned"] == 0, diag


def test_multi_rejects_payload_on_a_device_it_does_not_drive(h3c, torch_dev):
    """Descriptors on device 0 given to an engine that does not list device 0 cannot be routed: only
    checkable with 2+ GPUs, so here the engine over {0} must accept what {0, 0} accepts."""
    torch, dev = torch_dev
    if torch.cuda.device_count() < 2:
        m = h3c.Multi([0])
        try:
            x = torch.arange(4096, dtype=torch.int32, device=dev).view(torch.uint8)
            t, v = m.batch_create([x])
            assert int(v[0]) == orc.crc32c(x.cpu().numpy())
        finally:
            m.close()
        return
    m = h3c.Multi([1])
    try:
        x = torch.zeros(4096, dtype=torch.uint8, device=dev)
        with pytest.raises(h3c.EngineError) as ei:
            m.batch_create([x])
        assert ei.value.code == 3
    finally:
        m.close()
