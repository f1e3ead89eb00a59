"""Batched partial updates on the GPU vs the reference's updateChecksum, replayed write by write.

The oracle replays every write through its restatement of ChunkReplica::updateChecksum
(src/storage/store/ChunkReplica.cc:319-394, case iv: prefix + write + suffix CRCs and two
combines over the whole chunk) and the engine must reproduce the stored checksum after
each write, the final chunk bytes, and the final checksums.
"""
import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu
MASK = 0xFFFFFFFF
G = 4096


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def i32(arr, torch, dev):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(arr, dtype=np.uint32)).view(np.int32)).to(dev)


def run_case(h3c, torch, dev, nchunks, chunk_len, writes, seed, replay_chunks=None, invalid=(), stale=None,
             exact=False):
    """writes: list of (chunk, first_block, nblocks).  stale: {chunk: error} XORed into the
    stored checksum (bit rot / a torn write): the oracle replays the reference literally, whose
    case (iv) re-reads the chunk; exact mode must match it, trusted mode must be off by exactly
    the stored error (a uniform-length chunk's error is never shifted)."""
    rng = np.random.default_rng(seed)
    bpc = chunk_len // G
    chunks = rng.integers(0, 256, (nchunks, chunk_len), dtype=np.uint8)
    true0 = np.array([orc.crc32c(chunks[c]) for c in range(nchunks)], dtype=np.uint32)
    err = np.zeros(nchunks, dtype=np.uint32)
    for c, e in (stale or {}).items():
        err[c] = e
    raw0 = true0 ^ err
    # expand writes into block writes (sequence order); last block index of each write
    blk_chunk, blk_index, last_of_write = [], [], []
    for (c, b0, nb) in writes:
        for k in range(nb):
            blk_chunk.append(c)
            blk_index.append(b0 + k)
        last_of_write.append(len(blk_chunk) - 1)
    for pos, (c, b) in invalid:  # out-of-range entries inserted at given positions
        blk_chunk.insert(pos, c)
        blk_index.insert(pos, b)
        last_of_write = [x + (1 if x >= pos else 0) for x in last_of_write]
    n = len(blk_chunk)
    payload = rng.integers(0, 256, (n, G), dtype=np.uint8)

    dchunks = torch.from_numpy(chunks.copy()).to(dev)
    bases = torch.tensor([dchunks[c].data_ptr() for c in range(nchunks)], dtype=torch.int64, device=dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    raw_out = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    ninv = torch.full((1,), -1, dtype=torch.int32, device=dev)
    ctr = torch.full((8,), -1, dtype=torch.int64, device=dev)
    h3c.update_blocks(bases, chunk_len, i32(raw0, torch, dev), i32(blk_chunk, torch, dev),
                      i32(blk_index, torch, dev), torch.from_numpy(payload).to(dev), out, raw_out,
                      block_bytes=G, n_invalid=ninv, exact=exact, counters=ctr)
    torch.cuda.synchronize()
    got = u32(out)
    got_final = u32(raw_out)
    got_chunks = dchunks.cpu().numpy()

    # Host replay, write by write, through the updateChecksum restatement.
    host = chunks.copy()
    meta = [{"size": chunk_len, "type": orc.CRC32C, "value": int(raw0[c])} for c in range(nchunks)]
    want = {}
    valid = [(c < nchunks and b < bpc) for c, b in zip(blk_chunk, blk_index)]
    replay = set(range(nchunks)) if replay_chunks is None else set(replay_chunks)
    i = 0
    for w, (c, b0, nb) in enumerate(writes):
        # indices of this write's block entries (skip invalid ones interleaved)
        idx = []
        while len(idx) < nb:
            if valid[i]:
                idx.append(i)
            i += 1
        data = np.concatenate([payload[j] for j in idx])
        off = b0 * G
        host[c, off: off + nb * G] = data
        if c in replay:
            wt, wv = orc.create(orc.CRC32C, data)
            rc, meta[c] = orc.update_checksum(meta[c], {"offset": off, "length": nb * G, "type": wt, "value": wv},
                                              chunk_len, off == chunk_len, host[c])
            assert rc == 0
            want[idx[-1]] = meta[c]["value"]
    off_by = {} if exact else {k: int(err[blk_chunk[k]]) for k in want}  # trusted: the stored error persists
    bad = [(k, hex(int(got[k])), hex(v)) for k, v in want.items() if int(got[k]) != v ^ off_by.get(k, 0)]
    assert not bad, bad[:10]
    assert np.array_equal(got_chunks, host), "chunk bytes after write-back"
    touched = {c for c, b in zip(blk_chunk, blk_index) if c < nchunks and b < bpc}
    for c in range(nchunks):
        if c in touched:
            assert int(got_final[c]) == orc.crc32c(host[c]) ^ (0 if exact else int(err[c])), c
        else:  # no write reached it: the stored value stays, stale or not
            assert int(got_final[c]) == int(raw0[c]), c
    for k, v in enumerate(valid):
        if not v:
            assert int(got[k]) == 0
    n_bad = sum(1 for v in valid if not v)
    assert int(ninv.item()) == n_bad
    n_ok = len(valid) - n_bad
    reuse = chunk_len == G
    assert ctr.cpu().tolist() == [0, n_ok if reuse else 0, 0, 0 if reuse else n_ok, 0, 0, n_bad,
                                  int((err != 0).sum()) if exact else 0]


@pytest.fixture(params=["fused", "tiles", "sort"])
def scan_mode(request, h3c, hooks):
    """Every per-chunk scan path: the fused launch (default for 4 KiB blocks and <= 128 chunks),
    dense tiles, and the rocPRIM sort + scan_by_key fallback for many chunks (forced through
    h3c_test_hook)."""
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS[request.param])
    return request.param


def test_update_small_random_with_collisions(h3c, torch_dev, scan_mode):
    torch, dev = torch_dev
    rng = np.random.default_rng(1)
    nchunks, chunk_len = 6, 256 << 10  # 64 blocks per chunk -> many same-slot rewrites
    writes = [(int(rng.integers(0, nchunks)), int(rng.integers(0, 64)), 1) for _ in range(2500)]
    run_case(h3c, torch, dev, nchunks, chunk_len, writes, seed=2)


def test_update_multiblock_and_reuse_and_invalid(h3c, torch_dev, scan_mode):
    torch, dev = torch_dev
    rng = np.random.default_rng(3)
    nchunks, chunk_len = 4, 128 << 10
    writes = []
    for _ in range(600):
        c = int(rng.integers(0, nchunks))
        nb = int(rng.integers(1, 6))
        b0 = int(rng.integers(0, 32 - nb + 1))
        writes.append((c, b0, nb))
    writes.append((1, 0, 32))  # whole-chunk overwrite: updateChecksum's reuse case (:337-339)
    writes.append((1, 3, 2))
    run_case(h3c, torch, dev, nchunks, chunk_len, writes, seed=4,
             invalid=[(5, (nchunks, 0)), (77, (0, 999)), (300, (7, 7))])


def test_update_single_slot_hammer(h3c, torch_dev, scan_mode):
    """Every write hits one slot: the longest possible previous-writer chain."""
    torch, dev = torch_dev
    run_case(h3c, torch, dev, 2, 64 << 10, [(1, 5, 1)] * 700 + [(0, 15, 1)] * 3, seed=5)


@pytest.mark.parametrize("exact", [False, True])
def test_update_blocks_stale_stored_checksums(h3c, torch_dev, scan_mode, exact):
    """Stored checksums that disagree with the bytes, through every scan
    path: H3C_UPD_EXACT reproduces the reference's case (iv) re-read exactly; trusted mode
    carries each chunk's stored error unchanged; chunks no write reaches keep their value."""
    torch, dev = torch_dev
    rng = np.random.default_rng(61 + exact)
    nchunks, chunk_len = 9, 128 << 10
    writes = [(int(rng.integers(0, nchunks - 1)), int(rng.integers(0, 31)), int(rng.integers(1, 3)))
              for _ in range(700)]  # chunk 8 gets no write
    stale = {c: int(rng.integers(1, 1 << 32)) for c in (0, 3, 5, 8)}
    run_case(h3c, torch, dev, nchunks, chunk_len, writes, seed=62, stale=stale, exact=exact,
             invalid=[(9, (nchunks, 0)), (400, (2, 32))])


@pytest.mark.parametrize("exact", [False, True])
def test_update_blocks_whole_chunk_reuse_case(h3c, torch_dev, exact):
    """block_bytes == chunk_len: every write replaces the chunk, updateChecksum's reuse case
    (ChunkReplica.cc:337-339) -- the client checksum, i.e. the payload's CRC in exact mode."""
    torch, dev = torch_dev
    rng = np.random.default_rng(71)
    writes = [(int(rng.integers(0, 5)), 0, 1) for _ in range(300)]
    run_case(h3c, torch, dev, 5, G, writes, seed=72, stale={1: 0x1234, 4: 0xFFFF0000}, exact=exact)


def test_update_blocks_large_chunk_count_paths(h3c, torch_dev, hooks):
    """200 chunks (beyond the fused path's 128 columns): tiles by default, sort when forced."""
    torch, dev = torch_dev
    rng = np.random.default_rng(81)
    writes = [(int(rng.integers(0, 200)), int(rng.integers(0, 16)), 1) for _ in range(3000)]
    run_case(h3c, torch, dev, 200, 64 << 10, writes, seed=82, stale={7: 5}, exact=True)
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["sort"])
    run_case(h3c, torch, dev, 200, 64 << 10, writes, seed=83, stale={9: 5}, exact=True)


def test_update_config3_shape_full_size(h3c, torch_dev):
    """BASELINE config 3: 100k random 4 KiB writes into 64 x 64 MiB chunks.

    Every chunk's final checksum equals the oracle's CRC of its final bytes (and a fresh GPU
    create), and chunk 0 is replayed write by write through the oracle's updateChecksum."""
    torch, dev = torch_dev
    nchunks, chunk_len, nw = 64, 64 << 20, 100_000
    bpc = chunk_len // G
    rng = np.random.default_rng(20250629)
    wc = rng.integers(0, nchunks, nw).astype(np.uint32)
    wb = rng.integers(0, bpc, nw).astype(np.uint32)
    dchunks = torch.empty(nchunks * chunk_len, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(dchunks, chunk_len, nchunks, chunk_len, 20250629)
    payload = torch.empty(nw * G, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(payload, G, nw, G, 777)
    plan = h3c.Plan.uniform(dchunks.data_ptr(), chunk_len, nchunks)
    raw0 = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    plan.run(raw0)
    host0 = dchunks[:chunk_len].cpu().numpy().copy()  # chunk 0 before
    bases = torch.tensor([dchunks.data_ptr() + c * chunk_len for c in range(nchunks)], dtype=torch.int64, device=dev)
    out = torch.zeros(nw, dtype=torch.int32, device=dev)
    raw_out = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    h3c.update_blocks(bases, chunk_len, raw0, i32(wc, torch, dev), i32(wb, torch, dev), payload, out, raw_out)
    fresh = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    plan.run(fresh)
    torch.cuda.synchronize()
    assert torch.equal(fresh, raw_out)
    final_bytes = dchunks.cpu().numpy()
    want_final = np.zeros(nchunks, dtype=np.uint32)
    orc.lib().orc_batch_crc32c(final_bytes.ctypes.data, chunk_len, nchunks, 0xFFFFFFFF, 16, 0, want_final.ctypes.data)
    assert np.array_equal(u32(raw_out), want_final)  # all 64 chunks against the oracle
    del final_bytes
    got = u32(out)
    # chunk 0, write by write, through the oracle's updateChecksum (case iv over 64 MiB)
    pay = payload.cpu().numpy().reshape(nw, G)
    host = host0
    meta = {"size": chunk_len, "type": orc.CRC32C, "value": int(u32(raw0)[0])}
    idx = np.nonzero(wc == 0)[0]
    for k in idx[:200]:  # each replay step CRCs 64 MiB on the host
        off = int(wb[k]) * G
        host[off: off + G] = pay[k]
        wt, wv = orc.create(orc.CRC32C, pay[k])
        rc, meta = orc.update_checksum(meta, {"offset": off, "length": G, "type": wt, "value": wv},
                                       chunk_len, False, host)
        assert rc == 0 and int(got[k]) == meta["value"], k
    # last write of every chunk == its final checksum
    fin = u32(raw_out)
    for c in range(nchunks):
        last = np.nonzero(wc == c)[0][-1]
        assert int(got[last]) == int(fin[c])
    plan.close()


def test_update_blocks_crc32_ieee(h3c, torch_dev):
    """ChecksumType::CRC32 (IEEE polynomial, Common.h:161,195) through the block-update path:
    the chunk checksum after every write equals crc32 of the whole chunk."""
    torch, dev = torch_dev
    rng = np.random.default_rng(12)
    nchunks, chunk_len = 3, 64 << 10
    bpc = chunk_len // G
    chunks = rng.integers(0, 256, (nchunks, chunk_len), dtype=np.uint8)
    raw0 = np.array([orc.crc32(chunks[c]) for c in range(nchunks)], dtype=np.uint32)
    nw = 200
    wc = rng.integers(0, nchunks, nw).astype(np.uint32)
    wb = rng.integers(0, bpc, nw).astype(np.uint32)
    pay = rng.integers(0, 256, (nw, G), dtype=np.uint8)
    d = torch.from_numpy(chunks.copy()).to(dev)
    bases = torch.tensor([d[c].data_ptr() for c in range(nchunks)], dtype=torch.int64, device=dev)
    out = torch.zeros(nw, dtype=torch.int32, device=dev)
    raw_out = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    h3c.update_blocks(bases, chunk_len, i32(raw0, torch, dev), i32(wc, torch, dev), i32(wb, torch, dev),
                      torch.from_numpy(pay).to(dev), out, raw_out, type_=h3c.ChecksumType.CRC32)
    torch.cuda.synchronize()
    got = u32(out)
    host = chunks.copy()
    for k in range(nw):
        c, b = int(wc[k]), int(wb[k])
        host[c, b * G:(b + 1) * G] = pay[k]
        assert int(got[k]) == orc.crc32(host[c]), k
    assert np.array_equal(d.cpu().numpy(), host)


def test_update_fused_lookback_gives_up_and_reports_void_batch(h3c, torch_dev, hooks):
    """a fused-path workgroup that gives up its look-back wait (forced for ticket 1
    through H3C_HOOK_UPD_LOOKBACK) must not pass as a good batch: *n_invalid = UINT32_MAX and
    counters.invalid = UINT64_MAX; the chunk bytes are still right.  Without the hook the same
    batch is exact (run_case)."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(99)
    nchunks, chunk_len, nw = 8, 256 << 10, 20000  # many workgroups: ticket 1 has a predecessor
    wc = rng.integers(0, nchunks, nw).astype(np.uint32)
    wb = rng.integers(0, chunk_len // G, nw).astype(np.uint32)
    chunks = rng.integers(0, 256, (nchunks, chunk_len), dtype=np.uint8)
    raw0 = np.array([orc.crc32c(chunks[c]) for c in range(nchunks)], dtype=np.uint32)
    pay = rng.integers(0, 256, (nw, G), dtype=np.uint8)
    d = torch.from_numpy(chunks.copy()).to(dev)
    bases = torch.tensor([d[c].data_ptr() for c in range(nchunks)], dtype=torch.int64, device=dev)
    out = torch.zeros(nw, dtype=torch.int32, device=dev)
    raw_out = torch.zeros(nchunks, dtype=torch.int32, device=dev)
    ninv = torch.zeros(1, dtype=torch.int32, device=dev)
    ctr = torch.zeros(8, dtype=torch.int64, device=dev)
    hooks(h3c.HOOK_UPD_LOOKBACK, 1)
    h3c.update_blocks(bases, chunk_len, i32(raw0, torch, dev), i32(wc, torch, dev), i32(wb, torch, dev),
                      torch.from_numpy(pay).to(dev), out, raw_out, n_invalid=ninv, counters=ctr)
    torch.cuda.synchronize()
    assert int(ninv.item()) == -1 and int(ctr[6].item()) == -1
    host = chunks.copy()
    for k in range(nw):
        host[wc[k], wb[k] * G:(wb[k] + 1) * G] = pay[k]
    assert np.array_equal(d.cpu().numpy(), host)
    hooks(h3c.HOOK_UPD_LOOKBACK, 0)
    writes = [(int(c), int(b), 1) for c, b in zip(wc[:3000], wb[:3000])]
    run_case(h3c, torch, dev, nchunks, chunk_len, writes, seed=100)
