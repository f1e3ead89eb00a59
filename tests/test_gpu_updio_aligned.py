"""The fast branch's aligned sub-branch of h3c_update_ios (uio_aprep_kernel + uio_afused_kernel, VERDICT r04
#5) against the oracle, the chain-based fast branch and the general pipeline.

A batch takes it when every op is a full, block-aligned 4 KiB typed WRITE from a 16-byte-aligned payload into a
chunk stored under the batch polynomial (BASELINE config 3 exactly; updateChecksum case (iv),
ChunkReplica.cc:356-390; the Rust engine's copy_on_write, chunk.rs:89-158, in the std domain).  Each fixture
is replayed through the oracle's ChunkReplica::update restatement (Scenario.check) and run three times on
fresh replicas: aligned (H3C_HOOK_UPD_ALIGNED 2), chain-based fast (ALIGNED 1, FAST 2) and general (FAST 1);
the three must agree on every result, final chunk state, counter and byte.  Failed A6 checks make the pass
void and uio_afix_kernel recompute it (diag counter aligned_recovered); a block whose last write fails its
check is written by uio_afix_kernel (the deferred list).
"""
import numpy as np
import pytest

import oracle_lib as orc
from test_gpu_updio_fast import fast_scenario

pytestmark = pytest.mark.gpu
BLK = 4096


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


MODES = {"aligned": ((10, 2), (7, 2)), "fast": ((10, 1), (7, 2)), "general": ((10, 1), (7, 1))}


def run_modes(h3c, hooks, sc, modes=("aligned", "fast", "general"), **kw):
    out = {}
    for m in modes:
        for key, val in MODES[m]:
            hooks(key, val)
        sc.slab.copy_(sc.torch.from_numpy(sc._initial_bytes).to(sc.dev))
        before = h3c.diag_counters()
        chunks, res = sc.run(**kw)
        after = h3c.diag_counters()
        out[m] = (chunks.copy(), res.copy(), dict(sc.counters.as_dict()), sc.slab.cpu().numpy().copy(),
                  {k: after[k] - before[k] for k in after})
    return out


def check_modes(h3c, hooks, sc, expect_aligned=True, recovered=None, **kw):
    sc._initial_bytes = sc.slab.cpu().numpy().copy()
    kw.pop("poly", None)
    out = run_modes(h3c, hooks, sc, **kw)
    ad = out["aligned"][4]
    if expect_aligned:
        assert ad["aligned_batches"] == 1 and ad["aligned_abandoned"] == 0 and ad["fast_batches"] == 1, ad
        if recovered is not None:
            assert ad["aligned_recovered"] == recovered, ad
    else:
        assert ad["aligned_batches"] == 0 and ad["aligned_abandoned"] == 1, ad
    assert out["fast"][4]["aligned_batches"] == 0 and out["general"][4]["fast_batches"] == 0
    # each mode against the oracle's results first (names the mode that is wrong)
    for m in ("aligned", "fast", "general"):
        mr = out[m][1]
        bad = [i for i, e in enumerate(sc.expect) if (int(mr["status"][i]), int(mr["value"][i])) !=
               (e["status"], e["value"] & 0xFFFFFFFF)]
        assert not bad, (m, len(bad), bad[:5])
    ac, ar, ak, ab, _ = out["aligned"]
    for other in ("fast", "general"):
        oc, orr, ok, ob, _ = out[other]
        for f in ("status", "size", "value", "type"):
            bad = np.nonzero(ar[f] != orr[f])[0]
            assert not len(bad), (other, f, [(int(i), ar[i], orr[i]) for i in bad[:5]])
        for f in ("size", "value", "type"):
            assert np.array_equal(ac[f], oc[f]), (other, f)
        assert ak == ok, (other, ak, ok)
        assert np.array_equal(ab, ob), other
    # and against the oracle (the slab holds the general run's bytes, identical to the others)
    sc.counters = type(sc.counters)()
    for f, _ in sc.counters._fields_:
        setattr(sc.counters, f, ak[f])
    sc.check(ac, ar)
    return ad


def aligned_scenario(h3c, torch, dev, rng, nchunks, chunk_size, nops, bad=0.0, hot_blocks=None, type_=orc.CRC32C,
                     full_size=True, stale=0.0):
    sc = fast_scenario(h3c, torch, dev, rng, nchunks=nchunks, chunk_size=chunk_size, nops=nops, aligned=1.0, bad=bad,
                       hot_blocks=hot_blocks, type_=type_, full_size=full_size, stale=stale)
    sc.pay_align = 16
    return sc


@pytest.mark.parametrize("dev_api", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_aligned_random_block_writes(h3c, torch_dev, hooks, seed, dev_api):
    torch, dev = torch_dev
    rng = np.random.default_rng(500 + seed)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=16, chunk_size=256 << 10, nops=3000, full_size=bool(seed % 2))
    check_modes(h3c, hooks, sc, recovered=0, dev_api=dev_api)


@pytest.mark.parametrize("bad", [0.02, 0.2])
@pytest.mark.parametrize("dev_api", [False, True])
def test_aligned_failed_checks_recovered(h3c, torch_dev, hooks, bad, dev_api):
    """Failed A6 checks (corrupted transfers): the pass is void and uio_afix_kernel recomputes every result
    from the per-op records; on hot blocks some blocks' last write fails too (their bytes are deferred)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(int(bad * 100) + 7 * dev_api)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=2500, bad=bad, hot_blocks=6)
    check_modes(h3c, hooks, sc, recovered=1, dev_api=dev_api)


@pytest.mark.parametrize("stale", [0.0, 0.6])
@pytest.mark.parametrize("dev_api", [False, True])
def test_aligned_exact_mode(h3c, torch_dev, hooks, stale, dev_api):
    """H3C_UPD_EXACT on the aligned sub-branch: t0 from the chunks' bytes (uio_apiece_kernel + the piece
    pass), so a stale stored value is healed by the chunk's first write (case iv re-reads,
    ChunkReplica.cc:356-390) and counted; against the oracle and both other branches, all exact."""
    torch, dev = torch_dev
    rng = np.random.default_rng(41 + int(stale * 10) + 3 * dev_api)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=12, chunk_size=128 << 10, nops=2000, stale=stale,
                          full_size=False)
    check_modes(h3c, hooks, sc, recovered=0, exact=True, dev_api=dev_api)
    assert int(sc.counters.stale_chunks) == sc.stale_chunks


def test_aligned_exact_mode_untouched_chunks_and_failed_checks(h3c, torch_dev, hooks):
    """Exact mode with chunks no op writes (they keep their stored values, stale ones included) and, in a
    second batch, failed A6 checks over hot blocks (a void pass: uio_afix_kernel recomputes in exact mode)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(47)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=16, chunk_size=64 << 10, nops=24, stale=0.7)
    check_modes(h3c, hooks, sc, recovered=0, exact=True)
    assert int(sc.counters.stale_chunks) == sc.stale_chunks
    rng = np.random.default_rng(48)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=2500, bad=0.2, hot_blocks=6,
                          stale=0.5)
    check_modes(h3c, hooks, sc, recovered=1, exact=True)
    assert int(sc.counters.stale_chunks) == sc.stale_chunks


def test_aligned_hot_blocks_chains_across_tiles(h3c, torch_dev, hooks):
    """8 blocks per chunk take 6000 writes: every block's writers span all 256-op prep tiles (tile links and
    the epoch-tagged bucket lists), and each block's first writer leaves its last writer's bytes."""
    torch, dev = torch_dev
    rng = np.random.default_rng(17)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=4, chunk_size=64 << 10, nops=6000, hot_blocks=8)
    check_modes(h3c, hooks, sc, recovered=0)


def test_aligned_every_last_write_fails(h3c, torch_dev, hooks):
    """Every block is written 3 times and the last write of each fails A6: every multi-write block is
    deferred, and uio_afix_kernel writes the last passing payload (or leaves the block)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(23)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=4, chunk_size=64 << 10, nops=0)
    order = [(c, b) for c in range(4) for b in range(16)]
    for rep in range(3):
        for c, b in order:
            good = rep < 2 if (c + b) % 3 else rep == 0  # some blocks: only the first write passes
            sc.add(orc.UPD_WRITE, c, b * BLK, BLK, orc.CRC32C, good=good)
    check_modes(h3c, hooks, sc, recovered=1, dev_api=True)


def test_aligned_128_chunks_and_crc32(h3c, torch_dev, hooks):
    """128 chunks (lanes c and c + 64 of the look-back), and the CRC32 polynomial."""
    torch, dev = torch_dev
    rng = np.random.default_rng(29)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=128, chunk_size=32 << 10, nops=4000, bad=0.0)
    check_modes(h3c, hooks, sc, recovered=0, dev_api=True)
    rng = np.random.default_rng(31)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=32, chunk_size=64 << 10, nops=2000, type_=orc.CRC32)
    check_modes(h3c, hooks, sc, recovered=0, poly=orc.CRC32, type_=orc.CRC32)


def test_aligned_abandoned_for_an_unaligned_payload(h3c, torch_dev, hooks):
    """A payload that is not 16-byte aligned (or one unaligned write) leaves the batch to the chain-based fast
    branch: nothing is written by the aligned attempt."""
    torch, dev = torch_dev
    rng = np.random.default_rng(37)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=1500)
    sc.pay_align = 0  # payloads at odd offsets
    check_modes(h3c, hooks, sc, expect_aligned=False)


def test_aligned_give_up_recovers(h3c, torch_dev, hooks):
    """H3C_HOOK_UPD_GIVEUP bit 3: the aligned workgroup with ticket 1 gives up its look-back at once; the pass is
    void and uio_afix_kernel recomputes the results (the bytes were written right)."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_GIVEUP, 8)
    rng = np.random.default_rng(41)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=256 << 10, nops=20000)
    check_modes(h3c, hooks, sc, recovered=1, dev_api=True)


def test_aligned_repeated_batches_graphs_and_epochs(h3c, torch_dev, hooks):
    """The same device-table batch 300 times on the same buffers with graphs (capture, replays, the pointer
    audit) and through more than one epoch wrap of the scratch (the host zeroes it every 240 aligned batches):
    the state restored before each run, every run's results and final states equal the first run's, which
    equals the oracle."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_GRAPHS, 2)
    hooks(h3c.HOOK_UPD_ALIGNED, 2)
    rng = np.random.default_rng(43)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=1200, hot_blocks=4)
    chunks, ios = sc.device_ios()
    d_chunks0 = torch.from_numpy(chunks.view(np.uint8).copy()).to(dev)
    d_chunks = d_chunks0.clone()
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(len(ios) * 16, dtype=torch.uint8, device=dev)
    d_ctr = torch.zeros(8, dtype=torch.int64, device=dev)
    slab0 = sc.slab.clone()
    b = h3c.diag_counters()
    first = None
    for it in range(300):
        sc.slab.copy_(slab0)
        d_chunks.copy_(d_chunks0)
        h3c.update_ios_dev(d_chunks, d_ios, d_res, counters=d_ctr, graphs=True)
        if it in (0, 1, 2, 239, 240, 241, 299):
            torch.cuda.synchronize()
            got = (d_res.cpu().numpy().copy(), d_chunks.cpu().numpy().copy(), d_ctr.cpu().numpy().copy(),
                   sc.slab.cpu().numpy().copy())
            if first is None:
                first = got
                sc.counters = h3c.UpdateCounters()
                for f, v in zip(h3c.UpdateCounters._fields_, got[2].tolist()):
                    setattr(sc.counters, f[0], v)
                sc.check(got[1].view(h3c.CHUNK_STATE_DTYPE), got[0].view(h3c.UPDATE_RESULT_DTYPE))
            else:
                for x, y in zip(got, first):
                    assert np.array_equal(x, y), it
    torch.cuda.synchronize()
    d = {k: v - b[k] for k, v in h3c.diag_counters().items()}
    assert d["aligned_batches"] == 300 and d["aligned_recovered"] == 0, d
    assert d["graph_replays"] >= 290 and d["graph_pointer_refused"] == 0 and d["graph_topology_refused"] == 0, d


def test_aligned_std_domain_matches_other_branches(h3c, torch_dev, hooks):
    """H3C_UPD_STD_DOMAIN (the Rust chunk engine's copy_on_write, chunk.rs:89-158): the three forms agree, and
    every applied op's value is ~crc32c of its chunk's bytes after the batch for each chunk's last op."""
    from test_gpu_updio_fast import aligned_slab
    torch, dev = torch_dev
    MASK = 0xFFFFFFFF
    rng = np.random.default_rng(14)
    n, cs = 5, 64 << 10
    host = rng.integers(0, 256, (n, cs), dtype=np.uint8)
    outs = {}
    for m in ("aligned", "fast", "general"):
        for key, val in MODES[m]:
            hooks(key, val)
        slab, _raw = aligned_slab(torch, dev, host)
        chunks = np.zeros(n, dtype=h3c.CHUNK_STATE_DTYPE)
        for c in range(n):
            chunks[c] = (slab.data_ptr() + c * cs, cs, cs, (~orc.crc32c(host[c])) & MASK, 1, 0)
        r2 = np.random.default_rng(15)
        pay = torch.from_numpy(r2.integers(0, 256, 900 * BLK, dtype=np.uint8)).to(dev)
        ios = np.zeros(900, dtype=h3c.UPDATE_IO_DTYPE)
        for i in range(900):
            c, b = int(r2.integers(0, n)), int(r2.integers(0, 6))
            v = (~orc.crc32c(pay[i * BLK:(i + 1) * BLK].cpu().numpy())) & MASK
            ios[i] = (pay.data_ptr() + i * BLK, c, b * BLK, BLK, v if r2.random() > 0.05 else v ^ 4, 1, h3c.UPD_WRITE,
                      0, 0, 0)
        before = h3c.diag_counters()
        ctr = h3c.UpdateCounters()
        res = h3c.update_ios(chunks, ios, std_domain=True, counters=ctr)
        d = {k: v - before[k] for k, v in h3c.diag_counters().items()}
        outs[m] = (res.copy(), chunks.copy(), slab.cpu().numpy(), ctr.as_dict(), d)
    ar, ac, ab, ak, ad = outs["aligned"]
    assert ad["aligned_batches"] == 1 and ad["aligned_recovered"] == 1, ad  # (5 % failed checks: void, recomputed)
    for other in ("fast", "general"):
        orr, oc, ob, ok, _ = outs[other]
        for f in ("status", "size", "value", "type"):
            assert np.array_equal(ar[f], orr[f]), (other, f)
        for f in ("size", "value", "type"):
            assert np.array_equal(ac[f], oc[f]), (other, f)
        assert np.array_equal(ab, ob) and ak == ok, other
    assert ak["recalculate"] == int((ar["status"] == 0).sum()) and ak["read_chunk"] == 0
    for c in range(n):
        assert int(ac[c]["value"]) == (~orc.crc32c(ab[c])) & MASK


@pytest.mark.parametrize("giveup", [8, 16])
def test_aligned_void_pass_multi_write_blocks_first_writer_failed(h3c, torch_dev, hooks, giveup):
    """A void aligned pass (GIVEUP bit 3: ticket 1 gives up its look-back; bit 4: the pass reports itself void)
    over hot multi-write blocks where 30 % of the checks fail, first writers included: uio_afix_kernel must
    rebuild each op's delta against the last passing op before it on its block, or -- when every earlier op of
    the block failed -- against the block's original bytes through the FIRST op's records (crc0(old) =
    D_first ^ crc0(new_first)).  r05l (work-in-progress code, never committed) returned wrong results from
    the first block-first-writer op of a forced void pass onward; check_modes' per-mode oracle comparison
    names the mode and the ops."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_GIVEUP, giveup)
    rng = np.random.default_rng(61 + giveup)
    sc = aligned_scenario(h3c, torch, dev, rng, nchunks=8, chunk_size=64 << 10, nops=6000, bad=0.3, hot_blocks=5)
    check_modes(h3c, hooks, sc, recovered=1, dev_api=True)
