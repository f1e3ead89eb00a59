"""BASELINE config 3 at its real shape through the general UpdateIO path, pinned to the oracle.

100k random 4 KiB WRITE UpdateIOs into 64 x 64 MiB chunks (h3c_update_ios_dev, tables in HBM),
trusted and exact.  The reference semantics replaced are ChunkReplica::update + updateChecksum
(src/storage/store/ChunkReplica.cc:131-394).  What is checked against the CPU oracle
(oracle/crc_oracle.c), not against another GPU pass:

* every op of 2 chunks (~3,100 ops) replayed one by one through the ChunkReplica::update
  restatement (case iv re-reads the 64 MiB chunk per op): status, size and stored checksum;
* all 64 chunks' final bytes against a host replay of every op's bytes, and all 64 final stored
  checksums against the oracle's CRC of those bytes;
* every op's status and the reference's case counters.

In exact mode 4 chunks start with stale stored checksums (two of them replayed op by op): the
reference's case (iv) re-reads the bytes, so the first op on such a chunk heals it.
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


@pytest.mark.parametrize("exact", [False, True])
def test_updio_config3_full_shape_against_oracle(h3c, torch_dev, exact):
    torch, dev = torch_dev
    rng = np.random.default_rng(SEED + exact)
    wc = rng.integers(0, NCH, NW).astype(np.uint32)
    wb = rng.integers(0, CL // G, NW).astype(np.uint32)
    # chunks: the same splitmix generator on both sides (checked on one chunk below)
    host = np.empty((NCH, CL), dtype=np.uint8)
    for c in range(NCH):
        orc.lib().orc_fill_splitmix(host[c].ctypes.data, CL, SEED, c)
    dchunks = torch.empty(NCH * CL, dtype=torch.uint8, device=dev)
    h3c.fill_splitmix(dchunks, CL, NCH, CL, SEED)
    pay = rng.integers(0, 256, (NW, G), dtype=np.uint8)
    dpay = torch.from_numpy(pay).to(dev)
    assert np.array_equal(dchunks[CL: 2 * CL].cpu().numpy(), host[1])
    stored = _host_crcs(host)
    stale = {}
    if exact:
        stale = {c: int(rng.integers(1, 1 << 32)) for c in (int(wc[0]), int(wc[1]), 17, 40)}
    # client checksums from the oracle
    cks = np.array([orc.crc32c(pay[k]) for k in range(NW)], dtype=np.uint32)
    state = np.zeros(NCH, dtype=h3c.CHUNK_STATE_DTYPE)
    state["base"] = dchunks.data_ptr() + np.arange(NCH, dtype=np.uint64) * np.uint64(CL)
    state["chunk_size"] = CL
    state["size"] = CL
    state["value"] = stored ^ np.array([stale.get(c, 0) for c in range(NCH)], dtype=np.uint32)
    state["type"] = orc.CRC32C
    ios = np.zeros(NW, dtype=h3c.UPDATE_IO_DTYPE)
    ios["payload"] = dpay.data_ptr() + np.arange(NW, dtype=np.uint64) * np.uint64(G)
    ios["chunk"] = wc
    ios["offset"] = wb * G
    ios["length"] = G
    ios["checksum_value"] = cks
    ios["checksum_type"] = orc.CRC32C
    ios["kind"] = h3c.UPD_WRITE
    init_state = state.copy()
    d_state = torch.from_numpy(state.view(np.uint8).copy()).to(dev)
    d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(NW * h3c.UPDATE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_ctr = torch.zeros(8, dtype=torch.int64, device=dev)
    h3c.update_ios_dev(d_state, d_ios, d_res, exact=exact, counters=d_ctr)
    torch.cuda.synchronize()
    fin = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
    res = d_res.cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)
    ctr = d_ctr.cpu().tolist()
    got_bytes = dchunks.cpu().numpy().reshape(NCH, CL)

    # 2 chunks replayed op by op through ChunkReplica::update (before `host` takes every op's bytes)
    replay = sorted({int(wc[0]), int(wc[1])} | ({(int(wc[0]) + 1) % NCH} if wc[0] == wc[1] else set()))
    for c in replay:
        chunk = host[c].copy()
        meta = {"size": CL, "type": orc.CRC32C, "value": int(init_state["value"][c])}
        ks = np.nonzero(wc == c)[0]
        for k in ks:
            io = {"kind": orc.UPD_WRITE, "offset": int(wb[k]) * G, "length": G, "type": orc.CRC32C,
                  "value": int(cks[k])}
            want, meta = orc.replica_update(meta, chunk, CL, io, pay[k])
            got = (int(res["status"][k]), int(res["size"][k]), int(res["type"][k]), int(res["value"][k]))
            assert got == (want["status"], want["size"], want["type"], want["value"]), (c, k)
        assert (int(fin["size"][c]), int(fin["type"][c]), int(fin["value"][c])) == \
            (meta["size"], meta["type"], meta["value"]), c
        assert len(ks) > 1400

    # every op's bytes on the host; all 64 chunks' bytes and final stored checksums
    rows = host.reshape(NCH, CL // G, G)
    slot = wc.astype(np.int64) * (CL // G) + wb
    _, last_rev = np.unique(slot[::-1], return_index=True)
    last = NW - 1 - last_rev  # each slot's last writer in sequence order
    rows[wc[last], wb[last]] = pay[last]
    assert np.array_equal(got_bytes, host)
    want_final = _host_crcs(host)
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
