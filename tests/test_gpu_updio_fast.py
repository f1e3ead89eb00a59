"""The fast branch of h3c_update_ios (uio_fast_kernel) against the oracle and against the general
pipeline, and the engine's give-up / redo paths.

A batch takes the fast branch when every op is a typed WRITE inside one 4 KiB block of a chunk stored
under the batch polynomial, not growing it (updateChecksum case (iv), ChunkReplica.cc:356-390; the
Rust engine's copy_on_write, chunk.rs:89-158).  Each fixture here is replayed through the oracle's
ChunkReplica::update restatement (Scenario.check) and run twice: through the fast branch
(h3c_test_hook(H3C_HOOK_UPD_FAST, 2)) and through the general pipeline (hook value 1); the two must
agree on every result, every final chunk state, every counter and every chunk byte.
"""
import numpy as np
import pytest

import oracle_lib as orc
from test_gpu_updio import Scenario, random_scenario

pytestmark = pytest.mark.gpu
MASK = 0xFFFFFFFF
BLK = 4096


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


def aligned_slab(torch, dev, host):
    """A device copy of `host` (chunks x bytes) starting on a 4 KiB boundary (blocks are absolute
    4 KiB addresses); returns (view, backing tensor)."""
    raw = torch.empty(host.size + BLK, dtype=torch.uint8, device=dev)
    off = (-raw.data_ptr()) % BLK
    view = raw[off:off + host.size].view(host.shape)
    view.copy_(torch.from_numpy(host.copy()).to(dev))
    return view, raw


def qualifies(sc, type_=orc.CRC32C) -> bool:
    """The host's restatement of fast_op (h3c_updio.hip) over a scenario's ops, in sequence order."""
    meta = [dict(m) for m in sc.init_meta]
    if not 1 <= sc.nchunks <= 128:
        return False
    for c, io in sc.ops:
        if c >= sc.nchunks or io["kind"] != orc.UPD_WRITE or io["type"] != type_ or not io["length"]:
            return False
        m = meta[c]
        a = sc.slab.data_ptr() + c * sc.chunk_size + io["offset"]
        if m["type"] != type_ or io["offset"] + io["length"] > m["size"] or io.get("syncing"):
            return False
        if io["offset"] == 0 and io["length"] >= m["size"]:
            return False
        if a // BLK != (a + io["length"] - 1) // BLK:
            return False
    return True


def fast_scenario(h3c, torch, dev, rng, nchunks, chunk_size, nops, aligned=0.5, bad=0.02, hot_blocks=None,
                  type_=orc.CRC32C, stale=0.0, full_size=True):
    """One-block writes into CRC-stored chunks: aligned 4 KiB blocks or arbitrary ranges inside one
    block, some failing A6; hot_blocks: the writes land on that many blocks of each chunk only (chains
    of many ops per block, across prep tiles)."""
    sizes = [chunk_size] * nchunks if full_size else [int(rng.integers(3 * BLK, chunk_size + 1)) for _ in
                                                         range(nchunks)]
    sc = Scenario(h3c, torch, dev, nchunks, chunk_size, rng, init="crc", crc_type=type_, stale=stale, sizes=sizes)
    sc.slab, sc._raw = aligned_slab(torch, dev, sc.host)
    for _ in range(nops):
        c = int(rng.integers(0, nchunks))
        size = sc.meta[c]["size"]
        nblk = size // BLK
        b = int(rng.integers(0, nblk if hot_blocks is None else min(hot_blocks, nblk)))
        if rng.random() < aligned:
            off, ln = b * BLK, BLK
        else:
            lo = int(rng.integers(0, BLK))
            ln = int(rng.integers(1, BLK - lo + 1))
            off = b * BLK + lo
        if off == 0 and ln >= size:
            ln = size - 1
        sc.add(orc.UPD_WRITE, c, off, ln, type_, good=rng.random() >= bad)
    return sc


def run_both(h3c, hooks, sc, **kw):
    """The scenario through the fast branch, then (on a fresh replica) through the general pipeline;
    returns both (chunks, results, counters, bytes)."""
    out = []
    for mode in (2, 1):
        hooks(h3c.HOOK_UPD_FAST, mode)
        sc.slab.copy_(sc.torch.from_numpy(sc._initial_bytes).to(sc.dev))
        before = h3c.diag_counters()
        chunks, res = sc.run(**kw)
        after = h3c.diag_counters()
        out.append((chunks.copy(), res.copy(), dict(sc.counters.as_dict()), sc.slab.cpu().numpy().copy(),
                    {k: after[k] - before[k] for k in after}))
    return out


def check_both(h3c, hooks, sc, expect_fast=True, **kw):
    sc._initial_bytes = sc.slab.cpu().numpy().copy()
    assert qualifies(sc, kw.get("poly", orc.CRC32C)) == expect_fast
    kw.pop("poly", None)
    (fc, fr, fk, fb, fd), (gc, gr, gk, gb, gd) = run_both(h3c, hooks, sc, **kw)
    if expect_fast:
        assert fd["fast_batches"] == 1 and fd["fast_abandoned"] == 0, fd
    else:
        assert fd["fast_batches"] == 0 and fd["fast_abandoned"] == 1, fd
    assert gd["fast_batches"] == 0 and gd["fast_abandoned"] == 0, gd
    for f in ("status", "size", "value", "type"):
        bad = np.nonzero(fr[f] != gr[f])[0]
        assert not len(bad), (f, [(int(i), fr[i], gr[i]) for i in bad[:5]])
    for f in ("size", "value", "type"):
        assert np.array_equal(fc[f], gc[f]), f
    assert fk == gk, (fk, gk)
    assert np.array_equal(fb, gb)
    # and both against the oracle (the slab holds the general run's bytes, identical to the fast run's)
    sc.counters = type(sc.counters)()
    for f, _ in sc.counters._fields_:
        setattr(sc.counters, f, fk[f])
    sc.check(gc, gr)
    return fd


@pytest.mark.parametrize("dev_api", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_fast_branch_random_one_block_writes(h3c, torch_dev, hooks, seed, dev_api):
    torch, dev = torch_dev
    rng = np.random.default_rng(100 + seed)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=16, chunk_size=256 << 10, nops=3000,
                       full_size=bool(seed % 2))
    check_both(h3c, hooks, sc, dev_api=dev_api)


def test_fast_branch_hot_blocks_chains_across_tiles(h3c, torch_dev, hooks):
    """8 blocks per chunk take 6000 writes: every block's chain runs through every prep tile of 1,024 ops
    (the tile links and the bucket lists), with failed A6 checks inside chains."""
    torch, dev = torch_dev
    rng = np.random.default_rng(7)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=4, chunk_size=64 << 10, nops=6000, hot_blocks=8, bad=0.05)
    check_both(h3c, hooks, sc, dev_api=True)


def test_fast_branch_one_hammered_block(h3c, torch_dev, hooks):
    """Every op on one block of one chunk (a single chain of 2,500 ops)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(8)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=1, chunk_size=64 << 10, nops=2500, hot_blocks=1, bad=0.01)
    check_both(h3c, hooks, sc)


def test_fast_branch_128_chunks_and_failed_checks(h3c, torch_dev, hooks):
    """The largest chunk count the branch takes (lane c holds chunks c and c + 64); a fifth of the
    client checksums fail, and some chunks see only failed writes (they keep their stored state)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(9)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=128, chunk_size=32 << 10, nops=5000, bad=0.2)
    for _ in range(3):
        sc.add(orc.UPD_WRITE, 127, 4096, 100, good=False)
    check_both(h3c, hooks, sc, dev_api=True)


def test_fast_branch_chunks_sharing_blocks(h3c, torch_dev, hooks):
    """Chunks packed at a stride that is not a multiple of 4 KiB, so neighbouring chunks share absolute
    4 KiB blocks: small writes inside one absolute block of either chunk make two chains (two keys) on
    the same physical block, each storing only its own chunk's bytes.  Both branches and the oracle
    agree, and so do the bytes of the shared blocks."""
    torch, dev = torch_dev
    rng = np.random.default_rng(29)
    cs = 3 * BLK + 1000  # (chunk c starts 1000 * c bytes past a block boundary, mod 4 KiB)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=16, chunk_size=cs, nops=0)
    base = sc.slab.data_ptr()
    for _ in range(3000):
        c = int(rng.integers(0, 16))
        size = sc.meta[c]["size"]
        o = int(rng.integers(0, size))
        a = base + c * cs + o
        room = min(size - o, (a | (BLK - 1)) + 1 - a)
        ln = int(rng.integers(1, room + 1))
        if o == 0 and ln >= size:
            continue
        sc.add(orc.UPD_WRITE, c, o, ln, orc.CRC32C, good=rng.random() >= 0.02)
    check_both(h3c, hooks, sc)


def test_fast_branch_single_op_and_two_ops(h3c, torch_dev, hooks):
    """The smallest batches: one op, then two ops on the same block (a chain of two)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(31)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=1, chunk_size=64 << 10, nops=1, bad=0.0)
    check_both(h3c, hooks, sc)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=2, chunk_size=64 << 10, nops=0)
    sc.add(orc.UPD_WRITE, 1, 5 * BLK + 100, 300, orc.CRC32C)
    sc.add(orc.UPD_WRITE, 1, 5 * BLK + 200, 3000, orc.CRC32C)
    check_both(h3c, hooks, sc)


def test_fast_branch_129_chunks_takes_the_general_pipeline(h3c, torch_dev, hooks):
    torch, dev = torch_dev
    rng = np.random.default_rng(10)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=129, chunk_size=16 << 10, nops=500)
    sc._initial_bytes = sc.slab.cpu().numpy().copy()
    hooks(h3c.HOOK_UPD_FAST, 2)
    before = h3c.diag_counters()
    sc.check(*sc.run())
    d = {k: v - before[k] for k, v in h3c.diag_counters().items()}
    assert d["fast_batches"] == 0 and d["fast_abandoned"] == 0


@pytest.mark.parametrize("stale", [0.0, 0.6])
def test_fast_branch_exact_mode(h3c, torch_dev, hooks, stale):
    """H3C_UPD_EXACT: t0 from the chunks' bytes (the piece pass before uio_fast_kernel), stale stored
    values counted; case (iv) re-reads, so every result is the bytes' CRC."""
    torch, dev = torch_dev
    rng = np.random.default_rng(11)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=12, chunk_size=128 << 10, nops=2000, stale=stale,
                       full_size=False)
    for dev_api in (False, True):
        sc2 = sc if not dev_api else fast_scenario(h3c, torch, dev, np.random.default_rng(12), nchunks=12,
                                                    chunk_size=128 << 10, nops=2000, stale=stale, full_size=False)
        check_both(h3c, hooks, sc2, exact=True, dev_api=dev_api)
        assert int(sc2.counters.stale_chunks) == sc2.stale_chunks


def test_fast_branch_crc32_polynomial(h3c, torch_dev, hooks):
    torch, dev = torch_dev
    rng = np.random.default_rng(13)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=6, chunk_size=64 << 10, nops=1500, type_=orc.CRC32)
    check_both(h3c, hooks, sc, type_=h3c.ChecksumType.CRC32, poly=orc.CRC32)


def test_fast_branch_std_domain_matches_general(h3c, torch_dev, hooks):
    """H3C_UPD_STD_DOMAIN (the Rust chunk engine's copy_on_write): both branches agree, and every
    applied op's value is ~crc32c of the chunk bytes after it."""
    torch, dev = torch_dev
    rng = np.random.default_rng(14)
    n, cs = 5, 64 << 10
    host = rng.integers(0, 256, (n, cs), dtype=np.uint8)
    outs = []
    for mode in (2, 1):
        hooks(h3c.HOOK_UPD_FAST, mode)
        slab, _raw = aligned_slab(torch, dev, host)
        chunks = np.zeros(n, dtype=h3c.CHUNK_STATE_DTYPE)
        for c in range(n):
            chunks[c] = (slab.data_ptr() + c * cs, cs, cs, (~orc.crc32c(host[c])) & MASK, 1, 0)
        r2 = np.random.default_rng(15)
        pays, ios = [], np.zeros(800, dtype=h3c.UPDATE_IO_DTYPE)
        for i in range(800):
            c, b = int(r2.integers(0, n)), int(r2.integers(0, 4))
            lo = int(r2.integers(0, 4000))
            ln = int(r2.integers(1, BLK - lo + 1))
            p = torch.from_numpy(r2.integers(0, 256, ln, dtype=np.uint8)).to(dev)
            pays.append(p)
            v = (~orc.crc32c(p.cpu().numpy())) & MASK
            ios[i] = (p.data_ptr(), c, b * BLK + lo, ln, v if r2.random() > 0.05 else v ^ 4, 1, h3c.UPD_WRITE, 0, 0, 0)
        before = h3c.diag_counters()
        ctr = h3c.UpdateCounters()
        res = h3c.update_ios(chunks, ios, std_domain=True, counters=ctr)
        d = {k: v - before[k] for k, v in h3c.diag_counters().items()}
        outs.append((res.copy(), chunks.copy(), slab.cpu().numpy(), ctr.as_dict(), d))
    (fr, fc, fb, fk, fd), (gr, gc, gb, gk, gd) = outs
    assert fd["fast_batches"] == 1 and gd["fast_batches"] == 0
    for f in ("status", "size", "value", "type"):
        assert np.array_equal(fr[f], gr[f]), f
    for f in ("size", "value", "type"):
        assert np.array_equal(fc[f], gc[f]), f
    assert np.array_equal(fb, gb) and fk == gk
    assert fk["recalculate"] == int((fr["status"] == 0).sum()) and fk["read_chunk"] == 0
    for c in range(n):
        assert int(fc[c]["value"]) == (~orc.crc32c(fb[c])) & MASK


def test_fast_branch_abandons_a_general_batch(h3c, torch_dev, hooks):
    """A batch with one op the branch does not take (an append) is abandoned before any byte moves
    and the general pipeline runs it; the engine then predicts the general pipeline for that shape."""
    torch, dev = torch_dev
    rng = np.random.default_rng(16)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=4, chunk_size=64 << 10, nops=700, full_size=False)
    c = 2
    sc.add(orc.UPD_WRITE, c, sc.meta[c]["size"], 10)  # append: case (iii)
    d = check_both(h3c, hooks, sc, expect_fast=False)
    assert d["fast_abandoned"] == 1


def test_fast_branch_prediction_follows_the_last_outcome(h3c, torch_dev, hooks):
    """Default policy (hook 0): a shape whose last batch was abandoned goes straight to the general
    pipeline; a qualifying batch of a new shape takes the fast branch at once."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_FAST, 0)
    rng = np.random.default_rng(17)
    sc = random_scenario(h3c, torch, dev, rng, nchunks=6, chunk_size=32 << 10, nops=300)
    chunks, ios = sc.device_ios()
    d_chunks = torch.from_numpy(chunks.view(np.uint8).copy()).to(dev)
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(len(ios) * 16, dtype=torch.uint8, device=dev)
    snaps = []
    for _ in range(3):
        b = h3c.diag_counters()
        h3c.update_ios_dev(d_chunks, d_ios, d_res)
        torch.cuda.synchronize()
        snaps.append({k: v - b[k] for k, v in h3c.diag_counters().items()})
    assert snaps[0]["fast_abandoned"] == 1
    assert snaps[1]["fast_abandoned"] == 0 and snaps[2]["fast_abandoned"] == 0
    sc2 = fast_scenario(h3c, torch, dev, np.random.default_rng(18), nchunks=3, chunk_size=32 << 10, nops=200)
    b = h3c.diag_counters()
    sc2.check(*sc2.run())
    assert h3c.diag_counters()["fast_batches"] - b["fast_batches"] == 1


@pytest.mark.parametrize("graphs", [False, True])
def test_fast_branch_repeated_batches(h3c, torch_dev, hooks, graphs):
    """The same tables run repeatedly (each batch on top of the last, as the bench does), plain or as one
    captured graph per shape: every batch's final checksums equal the CRC of the chunks' bytes."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_GRAPHS, 2 if graphs else 1)
    hooks(h3c.HOOK_UPD_FAST, 0)
    rng = np.random.default_rng(19)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=4000, bad=0.0)
    chunks, ios = sc.device_ios()
    d_chunks = torch.from_numpy(chunks.view(np.uint8).copy()).to(dev)
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(len(ios) * 16, dtype=torch.uint8, device=dev)
    d_ctr = torch.zeros(8, dtype=torch.int64, device=dev)
    b = h3c.diag_counters()
    bound = h3c.UpdateIosDev(d_chunks, d_ios, d_res, counters=d_ctr, graphs=graphs)  # (odd batches: the bound call)
    for k in range(5):
        if k % 2:
            bound.run()
        else:
            h3c.update_ios_dev(d_chunks, d_ios, d_res, counters=d_ctr, graphs=graphs)
        torch.cuda.synchronize()
        fin = d_chunks.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
        got = sc.slab.cpu().numpy()
        for c in range(8):
            assert int(fin[c]["value"]) == orc.crc32c(got[c, :int(fin[c]["size"])]), (k, c)
        assert d_ctr.cpu().tolist()[3] == len(ios)
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["fast_batches"] == 5
    if graphs:
        assert d["graph_captures"] == 1 and d["graph_replays"] >= 3


def test_fast_branch_give_up_recovers(h3c, torch_dev, hooks):
    """H3C_HOOK_UPD_GIVEUP bit 2: uio_fast_kernel's workgroup with ticket 1 gives up its look-back at
    once, as a starved wait would.  The bytes and per-op deltas are complete; the recovery kernel
    recomputes every result, final state and counter: equal to the oracle's, one recovery counted."""
    torch, dev = torch_dev
    rng = np.random.default_rng(21)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=16, chunk_size=128 << 10, nops=20000, bad=0.03)
    hooks(h3c.HOOK_UPD_FAST, 2)
    hooks(h3c.HOOK_UPD_GIVEUP, 4)
    b = h3c.diag_counters()
    sc.check(*sc.run(dev_api=True))
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["fast_batches"] == 1 and d["fast_recovered"] == 1, d


@pytest.mark.parametrize("bit,counter", [(1, "redo_front_void"), (2, "rerun_phase_b_void")])
def test_general_pipeline_give_up_paths(h3c, torch_dev, hooks, bit, counter):
    """H3C_HOOK_UPD_GIVEUP bits 0 / 1: the front kernel's tile 1 (the pass is void: the host redoes the
    batch on the scan-based stage) or phase B's tile 1 (phase B rerun the scan-based way) gives up at
    once.  Results, chunk states and counters equal the oracle's; the redo is counted once."""
    torch, dev = torch_dev
    rng = np.random.default_rng(22 + bit)
    sc = random_scenario(h3c, torch, dev, rng, nchunks=10, chunk_size=64 << 10, nops=6000)
    hooks(h3c.HOOK_UPD_FAST, 1)
    hooks(h3c.HOOK_UPD_GIVEUP, bit)
    for dev_api in (False, True):
        sc2 = sc if not dev_api else random_scenario(h3c, torch, dev, np.random.default_rng(40 + bit), nchunks=10,
                                                     chunk_size=64 << 10, nops=6000)
        b = h3c.diag_counters()
        sc2.check(*sc2.run(dev_api=dev_api))
        d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
        assert d[counter] == 1, d


def test_config3_shape_counts_no_redo(h3c, torch_dev, hooks):
    """A config-3-like batch (block-aligned 4 KiB writes, 64 chunks) runs on the fast branch with no
    redo, no recovery and no abandoned attempt."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_FAST, 0)
    rng = np.random.default_rng(23)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=64, chunk_size=1 << 20, nops=20000, aligned=1.0, bad=0.0)
    b = h3c.diag_counters()
    sc.check(*sc.run(dev_api=True))
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["fast_batches"] == 1
    assert all(d[k] == 0 for k in ("redo_front_void", "rerun_phase_b_void", "redo_failed_a6",
                                   "redo_short_fragment_guess", "fast_abandoned", "fast_recovered")), d


@pytest.mark.parametrize("fast", [False, True])
def test_captured_pipeline_is_one_chain(h3c, torch_dev, hooks, fast):
    """every captured UpdateIO pipeline is one chain of kernel nodes -- one root, every
    node reachable from it through edges, no memset / memcpy node, no fork (h3c_diag_last_graph); the
    engine refuses to instantiate anything else (h3c_diag_counter 10 stays 0 here)."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_GRAPHS, 2)
    hooks(h3c.HOOK_UPD_FAST, 2 if fast else 1)
    rng = np.random.default_rng(31 + fast)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=3000, bad=0.0) if fast else \
        random_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=3000)
    chunks, ios = sc.device_ios()
    d_chunks = torch.from_numpy(chunks.view(np.uint8).copy()).to(dev)
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(len(ios) * 16, dtype=torch.uint8, device=dev)
    b = h3c.diag_counters()
    for _ in range(6):  # plain until the shape repeats on the same scratch leases, one capture, replays
        h3c.update_ios_dev(d_chunks, d_ios, d_res, graphs=True)
        torch.cuda.synchronize()
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["graph_captures"] >= 1 and d["graph_topology_refused"] == 0 and d["graph_replays"] >= 1, d
    g = h3c.diag_last_graph()
    assert g["copies"] == 0 and g["roots"] == 1 and g["reachable"] == g["nodes"] == g["kernels"], g
    assert g["edges"] == g["nodes"] - 1 and g["max_out"] == 1, g
    assert g["nodes"] >= (5 if fast else 8), g
    # every pointer argument of every node lies inside a buffer the graph key names
    assert d["graph_pointer_refused"] == 0, d
    a = h3c.diag_last_graph_audit()
    assert a["kernels"] == g["kernels"] and a["outside"] == 0 and a["unknown"] == 0, a
    assert a["pointers"] >= 4 * a["kernels"], a


@pytest.mark.parametrize("fast", [False, True])
def test_pointer_audit_refuses_a_pointer_outside_the_key(h3c, torch_dev, hooks, fast):
    """The audit's refusal path: with H3C_HOOK_UPD_GRAPHS = 3 the first device lease (which every
    pipeline kernel points into) is left out of the audited buffers, so every capture is refused
    (h3c_diag_counter 11), nothing is replayed, and the batches run as plain launches with the results
    of the plain first run (the state restored before each run)."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_GRAPHS, 3)
    hooks(h3c.HOOK_UPD_FAST, 2 if fast else 1)
    rng = np.random.default_rng(41 + fast)
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=2000, bad=0.0) if fast else \
        random_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=2000)
    chunks, ios = sc.device_ios()
    d_chunks0 = torch.from_numpy(chunks.view(np.uint8).copy()).to(dev)
    d_chunks = d_chunks0.clone()
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(len(ios) * 16, dtype=torch.uint8, device=dev)
    slab0 = sc.slab.clone()
    b = h3c.diag_counters()
    outs = []
    for _ in range(5):
        sc.slab.copy_(slab0)
        d_chunks.copy_(d_chunks0)
        torch.cuda.synchronize()
        h3c.update_ios_dev(d_chunks, d_ios, d_res)
        torch.cuda.synchronize()
        outs.append((d_res.cpu().numpy().copy(), d_chunks.cpu().numpy().copy(), sc.slab.cpu().numpy().copy()))
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["graph_pointer_refused"] >= 1 and d["graph_replays"] == 0, d
    a = h3c.diag_last_graph_audit()
    assert a["outside"] >= 1 and a["unknown"] == 0, a
    for o in outs[1:]:
        for x, y in zip(o, outs[0]):
            assert np.array_equal(x, y)
