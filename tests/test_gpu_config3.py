"""BASELINE config 3 at its real shape through both UpdateIO branches, pinned to the oracle.

100k random 4 KiB WRITE UpdateIOs into 64 x 64 MiB chunks (h3c_update_ios_dev, tables in HBM),
trusted and exact, each run once through the general pipeline (h3c_test_hook(H3C_HOOK_UPD_FAST, 1):
prep, sort, piece pass, front, block and phase-B kernels), once through the chain-based fast branch
(FAST 2, H3C_HOOK_UPD_ALIGNED 1: prep, link, uio_fast_kernel and its tail) and once through the
aligned sub-branch (ALIGNED 2: uio_aprep_kernel + uio_afused_kernel; exact mode adds the chunks' piece
pass first); the engine's diag counters must say which one ran.  The
reference semantics replaced are ChunkReplica::update + updateChecksum
(src/storage/store/ChunkReplica.cc:131-394).  What is checked against the CPU oracle
(oracle/crc_oracle.c), not against another GPU pass (the oracle side is computed once per mode and
shared by both branches):

* every op of 2 chunks (~3,100 ops) replayed one by one through the ChunkReplica::update
  restatement (case iv re-reads the 64 MiB chunk per op): status, size and stored checksum;
* every one of the 100,000 ops' stored checksums against a host delta chain built from the
  oracle's own primitives: r_k = r_prev ^ shift(crc0(old ^ new), bytes after the write), where
  `old` is the window's initial bytes or its previous writer's payload.  The chain is first
  asserted equal to the ChunkReplica::update replay on the 2 replayed chunks, so the shortcut is
  itself pinned to the case-(iv) restatement before it judges the other ~97k ops;
* all 64 chunks' final bytes against a host replay of every op's bytes, and all 64 final stored
  checksums against the oracle's CRC of those bytes;
* every op's status and the reference's case counters.

In exact mode 4 chunks start with stale stored checksums (two of them replayed op by op): the
reference's case (iv) re-reads the bytes, so the first op on such a chunk heals it (the delta chain
therefore starts from each chunk's true CRC in both modes).  Since round 6 the aligned sub-branch takes
exact batches too: t0 from the chunks' bytes, every op and the stale count as the other branches.
"""
import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu
G = 4096
NCH, CL, NW = 64, 64 << 20, 100_000
SEED = 20250629


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


def _host_crcs(host):
    out = np.zeros(NCH, dtype=np.uint32)
    orc.lib().orc_batch_crc32c(host.ctypes.data, CL, NCH, 0xFFFFFFFF, 16, 0, out.ctypes.data)
    return out


_ORACLE = {}


def _inputs(exact):
    """The batch (seeded) and, once per mode, what the oracle says about it."""
    rng = np.random.default_rng(SEED + exact)
    wc = rng.integers(0, NCH, NW).astype(np.uint32)
    wb = rng.integers(0, CL // G, NW).astype(np.uint32)
    pay = rng.integers(0, 256, (NW, G), dtype=np.uint8)
    stale = {}
    if exact:
        stale = {c: int(rng.integers(1, 1 << 32)) for c in (int(wc[0]), int(wc[1]), 17, 40)}
    if exact not in _ORACLE:
        # chunks: the same splitmix generator on both sides (checked on one chunk in the test)
        host = np.empty((NCH, CL), dtype=np.uint8)
        for c in range(NCH):
            orc.lib().orc_fill_splitmix(host[c].ctypes.data, CL, SEED, c)
        chunk1 = host[1].copy()
        stored = _host_crcs(host)
        cks = np.array([orc.crc32c(pay[k]) for k in range(NW)], dtype=np.uint32)
        values = stored ^ np.array([stale.get(c, 0) for c in range(NCH)], dtype=np.uint32)
        # 2 chunks replayed op by op through ChunkReplica::update (before `host` takes every op's bytes)
        replay = sorted({int(wc[0]), int(wc[1])} | ({(int(wc[0]) + 1) % NCH} if wc[0] == wc[1] else set()))
        per_op, finals = {}, {}
        for c in replay:
            chunk = host[c].copy()
            meta = {"size": CL, "type": orc.CRC32C, "value": int(values[c])}
            ks = np.nonzero(wc == c)[0]
            assert len(ks) > 1400
            for k in ks:
                io = {"kind": orc.UPD_WRITE, "offset": int(wb[k]) * G, "length": G, "type": orc.CRC32C,
                      "value": int(cks[k])}
                want, meta = orc.replica_update(meta, chunk, CL, io, pay[k])
                per_op[int(k)] = (want["status"], want["size"], want["type"], want["value"])
            finals[c] = (meta["size"], meta["type"], meta["value"])
        # every op's stored checksum by the delta chain (before `host` takes every op's bytes)
        rows = host.reshape(NCH, CL // G, G)
        slot = wc.astype(np.int64) * (CL // G) + wb
        order = np.argsort(slot, kind="stable")  # by slot, sequence order within a slot
        same = np.zeros(NW, dtype=bool)
        same[1:] = slot[order[1:]] == slot[order[:-1]]
        old = rows[wc, wb]  # each window's initial bytes (a copy)
        prev = order[np.nonzero(same)[0] - 1]  # the previous writer of those ops' window
        old[order[same]] = pay[prev]
        np.bitwise_xor(old, pay, out=old)
        dcrc = np.zeros(NW, dtype=np.uint32)
        orc.lib().orc_batch_crc32c(old.ctypes.data, G, NW, 0, 16, 0, dcrc.ctypes.data)  # init 0: crc0
        del old
        shift = orc.lib().orc_shift
        chain = stored.copy()  # the true CRCs: case (iv) re-reads, so a stale value heals at once
        exp_all = np.zeros(NW, dtype=np.uint32)
        for k in range(NW):
            c = int(wc[k])
            chain[c] ^= shift(int(dcrc[k]), CL - (int(wb[k]) + 1) * G, orc.POLY_CRC32C)
            exp_all[k] = chain[c]
        # the shortcut is pinned to the ChunkReplica::update replay before it judges every op
        for k, want in per_op.items():
            assert int(exp_all[k]) == want[3], k
        # every op's bytes on the host: the final bytes and checksums of all 64 chunks
        _, last_rev = np.unique(slot[::-1], return_index=True)
        last = NW - 1 - last_rev  # each slot's last writer in sequence order
        rows[wc[last], wb[last]] = pay[last]
        _ORACLE[exact] = dict(chunk1=chunk1, cks=cks, values=values, per_op=per_op, finals=finals,
                              final_bytes=host, want_final=_host_crcs(host), exp_all=exp_all)
        assert np.array_equal(chain, _ORACLE[exact]["want_final"])
    return wc, wb, pay, stale, _ORACLE[exact]


@pytest.mark.parametrize("branch", ["general", "fast", "aligned"])
@pytest.mark.parametrize("exact", [False, True])
def test_updio_config3_full_shape_against_oracle(h3c, torch_dev, hooks, exact, branch):
    torch, dev = torch_dev
    wc, wb, pay, stale, o = _inputs(exact)
    hooks(h3c.HOOK_UPD_FAST, 1 if branch == "general" else 2)
    hooks(h3c.HOOK_UPD_ALIGNED, 2 if branch == "aligned" else 1)
    dchunks = torch.empty(NCH * CL, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(dchunks, CL, NCH, CL, SEED)
    dpay = torch.from_numpy(pay).to(dev)
    assert np.array_equal(dchunks[CL: 2 * CL].cpu().numpy(), o["chunk1"])
    state = np.zeros(NCH, dtype=h3c.CHUNK_STATE_DTYPE)
    state["base"] = dchunks.data_ptr() + np.arange(NCH, dtype=np.uint64) * np.uint64(CL)
    state["chunk_size"] = CL
    state["size"] = CL
    state["value"] = o["values"]
    state["type"] = orc.CRC32C
    ios = np.zeros(NW, dtype=h3c.UPDATE_IO_DTYPE)
    ios["payload"] = dpay.data_ptr() + np.arange(NW, dtype=np.uint64) * np.uint64(G)
    ios["chunk"] = wc
    ios["offset"] = wb * G
    ios["length"] = G
    ios["checksum_value"] = o["cks"]
    ios["checksum_type"] = orc.CRC32C
    ios["kind"] = h3c.UPD_WRITE
    d_state = torch.from_numpy(state.view(np.uint8).copy()).to(dev)
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(NW * h3c.UPDATE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_ctr = torch.zeros(8, dtype=torch.int64, device=dev)
    before = h3c.diag_counters()
    h3c.update_ios_dev(d_state, d_ios, d_res, exact=exact, counters=d_ctr)
    torch.cuda.synchronize()
    diag = {k: v - before[k] for k, v in h3c.diag_counters().items()}
    # the branch that ran is the branch named, with no redo of any kind
    took_aligned = branch == "aligned"
    assert diag["fast_batches"] == (0 if branch == "general" else 1), diag
    assert diag["aligned_batches"] == (1 if took_aligned else 0), diag
    assert diag["fast_abandoned"] == 0 and diag["fast_recovered"] == 0, diag
    assert diag["aligned_abandoned"] == 0 and diag["aligned_recovered"] == 0, diag
    assert all(diag[k] == 0 for k in ("redo_front_void", "rerun_phase_b_void", "redo_failed_a6",
                                      "redo_short_fragment_guess")), diag
    fin = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
    res = d_res.cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)
    ctr = d_ctr.cpu().tolist()
    for k, want in o["per_op"].items():
        got = (int(res["status"][k]), int(res["size"][k]), int(res["type"][k]), int(res["value"][k]))
        assert got == want, (branch, k)
    # all 100,000 ops' stored checksums against the pinned delta chain
    bad = np.nonzero(res["value"] != o["exp_all"])[0]
    assert bad.size == 0, (branch, exact, bad.size, bad[:8].tolist())
    assert (res["type"] == orc.CRC32C).all()
    for c, want in o["finals"].items():
        assert (int(fin["size"][c]), int(fin["type"][c]), int(fin["value"][c])) == want, c
    assert np.array_equal(dchunks.cpu().numpy().reshape(NCH, CL), o["final_bytes"])
    want_final = o["want_final"]
    touched = np.zeros(NCH, dtype=bool)
    touched[wc] = True
    assert touched.all()
    assert np.array_equal(fin["value"], want_final)
    assert (fin["size"] == CL).all() and (fin["type"] == orc.CRC32C).all()
    assert (res["status"] == 0).all() and (res["size"] == CL).all()
    # the last op of each chunk reports the chunk's final checksum
    for c in range(NCH):
        assert int(res["value"][np.nonzero(wc == c)[0][-1]]) == int(want_final[c])
    # every op is updateChecksum case (iv) (ChunkReplica.cc:356-390)
    assert ctr == [0, 0, 0, NW, 0, 0, 0, len(stale)]


def test_updio_config3_full_shape_multi_engine(h3c, torch_dev):
    """The same 100k-op batch through h3c_multi_update_ios over devices {0, 0} (two worker threads on
    the one GPU, the chunks split 32 / 32 by capacity): host tables, every op pinned to the delta chain."""
    torch, dev = torch_dev
    wc, wb, pay, stale, o = _inputs(False)
    dchunks = torch.empty(NCH * CL, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(dchunks, CL, NCH, CL, SEED)
    dpay = torch.from_numpy(pay).to(dev)
    torch.cuda.synchronize()
    state = np.zeros(NCH, dtype=h3c.CHUNK_STATE_DTYPE)
    state["base"] = dchunks.data_ptr() + np.arange(NCH, dtype=np.uint64) * np.uint64(CL)
    state["chunk_size"] = CL
    state["size"] = CL
    state["value"] = o["values"]
    state["type"] = orc.CRC32C
    ios = np.zeros(NW, dtype=h3c.UPDATE_IO_DTYPE)
    ios["payload"] = dpay.data_ptr() + np.arange(NW, dtype=np.uint64) * np.uint64(G)
    ios["chunk"] = wc
    ios["offset"] = wb * G
    ios["length"] = G
    ios["checksum_value"] = o["cks"]
    ios["checksum_type"] = orc.CRC32C
    ios["kind"] = h3c.UPD_WRITE
    m = h3c.Multi([0, 0])
    try:
        ctr = h3c.UpdateCounters()
        res = m.update_ios(state, ios, counters=ctr)
        torch.cuda.synchronize()
        stats = m.last_stats()
    finally:
        m.close()
    units = [s[0] for s in stats]
    assert sum(units) == NW and units == [int((wc < NCH // 2).sum()), int((wc >= NCH // 2).sum())], units
    assert (res["status"] == 0).all() and (res["size"] == CL).all() and (res["type"] == orc.CRC32C).all()
    bad = np.nonzero(res["value"] != o["exp_all"])[0]
    assert bad.size == 0, (bad.size, bad[:8].tolist())
    assert np.array_equal(state["value"], o["want_final"])
    assert np.array_equal(dchunks.cpu().numpy().reshape(NCH, CL), o["final_bytes"])
    assert ctr.as_dict()["read_chunk"] == NW and ctr.as_dict()["checksum_mismatch"] == 0
