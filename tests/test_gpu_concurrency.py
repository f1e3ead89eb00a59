"""The shim's threading contract: entry points are called concurrently
from many host threads (32 AIO + 32 update threads in the reference,
src/storage/aio/AioReadWorker.h:27, src/storage/update/UpdateWorker.h:15), each with its
own stream.  ctypes releases the GIL during the calls, so these threads really overlap.
Also: a device-resident plan is capturable into a HIP graph (a scrub pass replayed with
one launch)."""
import threading

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


def test_concurrent_threads_own_streams(h3c, torch_dev):
    torch, dev = torch_dev
    nthreads, per = 16, 24
    rng = np.random.default_rng(1)
    host = [[rng.integers(0, 256, int(rng.integers(1, 3 << 20)), dtype=np.uint8) for _ in range(per)]
            for _ in range(nthreads)]
    want = [[orc.crc32c(d) for d in hs] for hs in host]
    dev_bufs = [[torch.from_numpy(d).to(dev) for d in hs] for hs in host]
    torch.cuda.synchronize()
    errors, results = [], [None] * nthreads
    start = threading.Barrier(nthreads)

    def work(k):
        try:
            s = torch.cuda.Stream(device=dev)
            start.wait()
            for it in range(3):
                exp = list(want[k])
                exp[it] ^= 1  # one mismatch per round
                raw, ok, nbad = h3c.batch_verify(dev_bufs[k], exp, stream=s)
                if nbad != 1 or ok[it] or list(map(int, raw)) != want[k]:
                    errors.append((k, it, nbad))
                # host-staged payloads and the general update path on the same thread
                t, v = h3c.batch_create(host[k][:4], stream=s)
                if list(map(int, v)) != want[k][:4]:
                    errors.append((k, it, "host"))
            results[k] = True
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors[:5]
    assert all(results)


def test_concurrent_update_batches_distinct_chunks(h3c, torch_dev):
    """Update threads each own a chunk set (the reference shards update jobs by chunk)."""
    torch, dev = torch_dev
    nthreads, nchunks, cl = 8, 4, 1 << 20
    G = 4096
    slabs, states, ioss, pays, finals = [], [], [], [], []
    rng = np.random.default_rng(2)
    for k in range(nthreads):
        slab = torch.empty(nchunks * cl, dtype=torch.uint8, device=dev)
        h3c.fill_splitmix(slab, cl, nchunks, cl, 100 + k)
        host = slab.cpu().numpy().reshape(nchunks, cl).copy()
        st = np.zeros(nchunks, dtype=h3c.CHUNK_STATE_DTYPE)
        for c in range(nchunks):
            st[c] = (slab.data_ptr() + c * cl, cl, cl, orc.crc32c(host[c]), 1, 0)
        nw = 300
        pay = rng.integers(0, 256, (nw, G), dtype=np.uint8)
        io = np.zeros(nw, dtype=h3c.UPDATE_IO_DTYPE)
        dpay = torch.from_numpy(pay.reshape(-1)).to(dev)
        for i in range(nw):
            c, b = int(rng.integers(0, nchunks)), int(rng.integers(0, cl // G))
            io[i] = (dpay.data_ptr() + i * G, c, b * G, G, orc.crc32c(pay[i]), 1, h3c.UPD_WRITE, 0, 0, 0)
            host[c, b * G:(b + 1) * G] = pay[i]
        slabs.append(slab)
        states.append(st)
        ioss.append(io)
        pays.append(dpay)
        finals.append([orc.crc32c(host[c]) for c in range(nchunks)])
    torch.cuda.synchronize()
    errors = []

    def work(k):
        try:
            s = torch.cuda.Stream(device=dev)
            res = h3c.update_ios(states[k], ioss[k], stream=s)
            if not (res["status"] == 0).all() or list(map(int, states[k]["value"])) != finals[k]:
                errors.append(k)
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors


def test_plan_run_captured_in_hip_graph(h3c, torch_dev):
    """A scrub pass (plan_run: seg + finalize kernels, no host sync) captured once into a
    HIP graph and replayed; every replay sees the current bytes."""
    torch, dev = torch_dev
    n, cl = 256, 256 << 10
    slab = torch.empty(n * cl, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(slab, cl, n, cl, 7)
    plan = h3c.Plan.uniform(slab.data_ptr(), cl, n)
    want = torch.zeros(n, dtype=torch.int32, device=dev)
    plan.run(want)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    mis = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            mis.zero_()
            plan.run(out, want, ok, mis, stream=s)
    g.replay()
    torch.cuda.synchronize()
    assert int(mis.item()) == 0 and torch.equal(out, want)
    slab[5 * cl + 17] ^= 1
    slab[200 * cl] ^= 0x80
    g.replay()
    torch.cuda.synchronize()
    assert int(mis.item()) == 2
    assert sorted(np.nonzero(ok.cpu().numpy() == 0)[0].tolist()) == [5, 200]
    plan.close()


def test_coalescing_queue_many_threads(h3c, torch_dev):
    """h3c_set_coalescing: 32 threads on the default stream, each mixing single-buffer verifies
    (host and device payloads, one injected mismatch per round), multi-buffer creates and
    h3c_crc32c; every result against the oracle, then the same with coalescing off."""
    torch, dev = torch_dev
    nthreads, rounds = 32, 6
    rng = np.random.default_rng(9)
    host = [[rng.integers(0, 256, int(rng.integers(1, 300 << 10)), dtype=np.uint8) for _ in range(4)]
            for _ in range(nthreads)]
    want = [[orc.crc32c(d) for d in hs] for hs in host]
    dev_bufs = [[torch.from_numpy(d).to(dev) for d in hs] for hs in host]
    torch.cuda.synchronize()
    for on in (True, False):
        h3c.set_coalescing(on)
        errors = []
        start = threading.Barrier(nthreads)

        def work(k):
            try:
                start.wait()
                for it in range(rounds):
                    j = it % 4
                    bufs = dev_bufs[k] if it % 2 else host[k]
                    exp = want[k][j] ^ (1 if it == 3 else 0)
                    raw, ok, nbad = h3c.batch_verify([bufs[j]], [exp])
                    if int(raw[0]) != want[k][j] or bool(ok[0]) != (it != 3) or nbad != (it == 3):
                        errors.append((k, it, "verify"))
                    t, v = h3c.batch_create(host[k])
                    if list(map(int, v)) != want[k]:
                        errors.append((k, it, "create"))
                    if h3c.crc32c(host[k][j]) != want[k][j]:
                        errors.append((k, it, "crc32c"))
            except Exception as e:  # noqa: BLE001
                errors.append((k, repr(e)))

        threads = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=120)
        h3c.set_coalescing(False)
        assert not errors, (on, errors[:5])


def test_coalescing_isolates_a_failing_caller(h3c, torch_dev):
    """with coalescing on, one caller's bad request (a device descriptor that runs past
    its allocation -> kInvalidArg) fails that caller only; the requests merged with it still get
    their own correct results."""
    import ctypes

    torch, dev = torch_dev
    nthreads, rounds = 24, 8
    rng = np.random.default_rng(19)
    host = [rng.integers(0, 256, int(rng.integers(1, 64 << 10)), dtype=np.uint8) for _ in range(nthreads)]
    want = [orc.crc32c(d) for d in host]
    big = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    bad = np.zeros(1, dtype=h3c.engine.DESC_DTYPE)
    bad["ptr"] = big.data_ptr() + (1 << 19)
    bad["len"] = 400 << 30  # beyond any HBM: rejected before launch
    bad["start_raw"] = 0xFFFFFFFF
    bad["type"] = 1
    h3c.set_coalescing(True)
    errors = []
    start = threading.Barrier(nthreads)

    def work(k):
        try:
            start.wait()
            for it in range(rounds):
                if k % 6 == 0 and it % 2 == 0:
                    out_t, out_v = np.zeros(1, dtype=np.uint8), np.zeros(1, dtype=np.uint32)
                    rc = h3c.engine.lib.h3c_batch_create(bad.ctypes.data, 1, out_t.ctypes.data, out_v.ctypes.data, None)
                    if rc != h3c.StatusCode.kInvalidArg:
                        errors.append((k, it, "bad request rc", rc))
                else:
                    t, v = h3c.batch_create([host[k]])
                    if int(v[0]) != want[k]:
                        errors.append((k, it, "create"))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    threads = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    h3c.set_coalescing(False)
    assert not errors, errors[:5]


def test_sync_bench_driver(h3c, torch_dev):
    """h3c_diag_sync_bench returns one latency per call and flags no mismatch (it checks every
    result against the buffer's own create)."""
    for on in (False, True):
        h3c.set_coalescing(on)
        lat, wall = h3c.sync_bench(8, 4096, 50)
        assert lat.shape == (400,) and (lat > 0).all() and wall > 0
    h3c.set_coalescing(False)


@pytest.mark.parametrize("exact", [False, True])
def test_update_blocks_captured_in_hip_graph_cold_cache(h3c, torch_dev, exact):
    """h3c_update_blocks(_ex) captured into a HIP graph on its first call for a chunk geometry
    (the shift-table cache is cold, so the table is computed on the capturing stream instead of
    being built and published), then replayed: the chunk checksums equal a fresh create of the
    bytes, and the counters are written by the graph."""
    torch, dev = torch_dev
    nchunks, cl, G = 5, (7 << 16) + (1 << 12) * (3 if exact else 5), 4096  # geometries no other test uses
    bpc = cl // G
    slab = torch.empty(nchunks * cl, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(slab, cl, nchunks, cl, 11)
    plan = h3c.Plan.uniform(slab.data_ptr(), cl, nchunks)
    raw_in = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    plan.run(raw_in)
    rng = np.random.default_rng(3)
    nw = 300
    wc = torch.from_numpy(rng.integers(0, nchunks, nw).astype(np.int32)).to(dev)
    wb = torch.from_numpy(rng.integers(0, bpc, nw).astype(np.int32)).to(dev)
    pay = torch.empty(nw * G, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(pay, G, nw, G, 12)
    bases = torch.arange(nchunks, dtype=torch.int64, device=dev) * cl + slab.data_ptr()
    out = torch.zeros(nw, dtype=torch.int32, device=dev)
    raw_out = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    ctr = torch.zeros(8, dtype=torch.int64, device=dev)
    ws = torch.empty(h3c.update_workspace_bytes(nw, nchunks, cl, G), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            h3c.update_blocks(bases, cl, raw_in, wc, wb, pay, out, raw_out, block_bytes=G, workspace=ws, stream=s,
                              exact=exact, counters=ctr)
    g.replay()
    torch.cuda.synchronize()
    fresh = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    plan.run(fresh)
    torch.cuda.synchronize()
    assert torch.equal(fresh, raw_out)
    assert ctr.cpu().tolist() == [0, 0, 0, nw, 0, 0, 0, 0]
    plan.close()


def _fast_tables(h3c, torch, dev, rng, nchunks, cl, nw, seed):
    """A fast-branch batch (one-block 4 KiB writes) on its own slab: device tables and the expected
    final checksums after k applications are computed by the caller from the returned host copy."""
    G = 4096
    slab = torch.empty(nchunks * cl, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(slab, cl, nchunks, cl, seed)
    host = slab.cpu().numpy().reshape(nchunks, cl).copy()
    st = np.zeros(nchunks, dtype=h3c.CHUNK_STATE_DTYPE)
    for c in range(nchunks):
        st[c] = (slab.data_ptr() + c * cl, cl, cl, orc.crc32c(host[c]), 1, 0)
    pay = rng.integers(0, 256, (nw, G), dtype=np.uint8)
    dpay = torch.from_numpy(pay.reshape(-1)).to(dev)
    io = np.zeros(nw, dtype=h3c.UPDATE_IO_DTYPE)
    for i in range(nw):
        c, b = int(rng.integers(0, nchunks)), int(rng.integers(0, cl // G))
        io[i] = (dpay.data_ptr() + i * G, c, b * G, G, orc.crc32c(pay[i]), 1, h3c.UPD_WRITE, 0, 0, 0)
        host[c, b * G:(b + 1) * G] = pay[i]
    d_state = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
    d_ios = torch.from_numpy(io.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(nw * h3c.UPDATE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    final = [orc.crc32c(host[c]) for c in range(nchunks)]
    return slab, dpay, d_state, d_ios, d_res, final


@pytest.mark.parametrize("graphs", [False, True])
def test_fast_branch_threads_beside_legacy_stream_calls(h3c, torch_dev, graphs):
    """Update threads repeating device-table fast-branch batches (each its own tables, stream and
    per-thread scratch; with graphs, captures happen during the run) while other threads make
    synchronous legacy-default-stream verify calls: every batch's final checksums equal the CRC of
    the chunks' bytes and every verify is right (a capture holds h3c_rt::capture_gate(), which the
    legacy-stream entries wait out instead of failing)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(7)
    nupd, nleg, reps = 4, 4, 6
    tabs = [_fast_tables(h3c, torch, dev, rng, 8, 1 << 20, 600, 300 + k) for k in range(nupd)]
    host = [[rng.integers(0, 256, 4096 * (1 + j), dtype=np.uint8) for j in range(4)] for _ in range(nleg)]
    want = [[orc.crc32c(d) for d in hs] for hs in host]
    torch.cuda.synchronize()
    errors = []
    start = threading.Barrier(nupd + nleg)

    def upd(k):
        try:
            slab, dpay, d_state, d_ios, d_res, final = tabs[k]
            s = torch.cuda.Stream(device=dev)
            bound = h3c.UpdateIosDev(d_state, d_ios, d_res, stream=s, graphs=graphs)
            start.wait()
            for r in range(reps):
                bound.run()
                s.synchronize()
                fin = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
                if list(map(int, fin["value"])) != final:  # (the same writes again: same bytes, same values)
                    errors.append((k, r, "state"))
                if not (d_res.cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)["status"] == 0).all():
                    errors.append((k, r, "status"))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    def leg(k):
        try:
            start.wait()
            for r in range(3 * reps):
                t, v = h3c.batch_create(host[k])  # (stream None: the legacy default stream)
                if list(map(int, v)) != want[k]:
                    errors.append(("legacy", k, r))
        except Exception as e:  # noqa: BLE001
            errors.append(("legacy", k, repr(e)))

    b = h3c.diag_counters()
    threads = [threading.Thread(target=upd, args=(k,)) for k in range(nupd)]
    threads += [threading.Thread(target=leg, args=(k,)) for k in range(nleg)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors[:5]
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["fast_batches"] == nupd * reps and d["fast_abandoned"] == 0, d
    if graphs:
        assert d["graph_capture_failures"] == 0, d


def test_fast_branch_wide_tables_concurrent_against_oracle(h3c, torch_dev):
    """VERDICT r04 #1 (the fast branch's early return): 4 threads, each with its own 100-127-chunk device
    tables, stream and payloads, run fast-branch batches at once, so the leases one thread's batch returns
    on its outcome word are taken by another's next batch at once.  Chunks 64-127 are committed by
    uio_fast_res_kernel's wave 1; the outcome word now follows every wave's reads of misc / chunks_out and
    its commit stores.  Each repetition restores the thread's bytes and table on its own stream and must
    give every op's result, every final chunk state and every byte the oracle's ChunkReplica::update
    replay gives (ChunkReplica.cc:131-394), 2 % of the ops failing A6."""
    torch, dev = torch_dev
    G, CL, NW, REPS = 4096, 64 << 10, 1500, 8
    rng = np.random.default_rng(2026)
    tabs = []
    for k in range(4):
        nch = 100 + 9 * k  # 100, 109, 118, 127 chunks: wave 1 commits chunks 64 and up
        raw = torch.empty(nch * CL + G, dtype=torch.uint8, device=dev)
        off = (-raw.data_ptr()) % G
        slab = raw[off:off + nch * CL]
        h3c.fill_splitmix(slab, CL, nch, CL, 900 + k)
        host0 = slab.cpu().numpy().reshape(nch, CL).copy()
        st = np.zeros(nch, dtype=h3c.CHUNK_STATE_DTYPE)
        for c in range(nch):
            st[c] = (slab.data_ptr() + c * CL, CL, CL, orc.crc32c(host0[c]), 1, 0)
        pay = rng.integers(0, 256, (NW, G), dtype=np.uint8)
        dpay = torch.from_numpy(pay.reshape(-1)).to(dev)
        io = np.zeros(NW, dtype=h3c.UPDATE_IO_DTYPE)
        wc = rng.integers(0, nch, NW)
        wc[:nch] = np.arange(nch)  # every chunk written, the high ones included
        wb = rng.integers(0, CL // G, NW)
        good = rng.random(NW) >= 0.02
        # the oracle: every op replayed in sequence order on host copies
        host = host0.copy()
        meta = [{"size": CL, "type": orc.CRC32C, "value": int(st["value"][c])} for c in range(nch)]
        want = np.zeros(NW, dtype=h3c.UPDATE_RESULT_DTYPE)
        for i in range(NW):
            c, b = int(wc[i]), int(wb[i])
            ck = orc.crc32c(pay[i]) ^ (0 if good[i] else 0x5A5A)
            io[i] = (dpay.data_ptr() + i * G, c, b * G, G, ck, 1, h3c.UPD_WRITE, 0, 0, 0)
            r, meta[c] = orc.replica_update(meta[c], host[c], CL,
                                            {"kind": orc.UPD_WRITE, "offset": b * G, "length": G,
                                             "type": orc.CRC32C, "value": ck}, pay[i])
            want[i] = (r["status"], r["size"], r["value"], r["type"], 0)
        d_init = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
        tabs.append(dict(nch=nch, slab=slab, raw=raw, dpay=dpay, bytes0=slab.clone(), d_init=d_init,
                         d_state=d_init.clone(), d_ios=torch.from_numpy(io.view(np.uint8).copy()).to(dev),
                         d_res=torch.zeros(NW * h3c.UPDATE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev),
                         want=want, host=host, final=meta))
    torch.cuda.synchronize()
    errors = []
    start = threading.Barrier(len(tabs))

    def upd(k):
        tb = tabs[k]
        try:
            s = torch.cuda.Stream(device=dev)
            bound = h3c.UpdateIosDev(tb["d_state"], tb["d_ios"], tb["d_res"], stream=s)
            start.wait()
            for r in range(REPS):
                with torch.cuda.stream(s):
                    tb["slab"].copy_(tb["bytes0"])
                    tb["d_state"].copy_(tb["d_init"])
                bound.run()
                s.synchronize()
                res = tb["d_res"].cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)
                for f in ("status", "size", "value", "type"):
                    if not np.array_equal(res[f], tb["want"][f]):
                        bad = np.nonzero(res[f] != tb["want"][f])[0]
                        errors.append((k, r, "result " + f, int(bad[0]), len(bad)))
                fin = tb["d_state"].cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
                got = [(int(fin["size"][c]), int(fin["type"][c]), int(fin["value"][c])) for c in range(tb["nch"])]
                exp = [(m["size"], m["type"], m["value"]) for m in tb["final"]]
                if got != exp:
                    errors.append((k, r, "state", [c for c in range(tb["nch"]) if got[c] != exp[c]][:8]))
            if not np.array_equal(tb["slab"].cpu().numpy().reshape(tb["nch"], CL), tb["host"]):
                errors.append((k, "bytes"))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    b = h3c.diag_counters()
    threads = [threading.Thread(target=upd, args=(k,)) for k in range(len(tabs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not errors, errors[:8]
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["fast_batches"] == len(tabs) * REPS and d["fast_abandoned"] == 0, d
