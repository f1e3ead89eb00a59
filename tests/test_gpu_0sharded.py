"""Two ranks on the HIP engine (BASELINE config 4 shape): shard.run_sharded verify
over 64 x 4 MiB splitmix chunks with injected bit flips, and shard.run_sharded_updates driving
h3c_update_ios on each rank's chunk range.  Both ranks share cuda:0 (one GPU on the test box);
the gather is gloo (control plane only -- per-chunk / per-op results).  The parent process makes
no GPU call before spawning (this file sorts ahead of the other GPU tests), and checks the
gathered results against the oracle.
"""
import importlib
import os
import socket

import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu

NCHUNKS, CLEN, SEED = 64, 4 << 20, 20251016
FLIPS = [(3, 17, 0), (17, CLEN - 1, 7), (40, 2 << 20, 3), (63, 0, 5)]  # (chunk, byte, bit)
U_CHUNKS, U_CS, U_OPS = 16, 256 << 10, 3000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _update_plan():
    """The update workload, identical in the parent and in every rank: initial chunk states
    and a sequence of ops (kind, chunk, offset, length, payload seed)."""
    rng = np.random.default_rng(SEED)
    sizes = rng.integers(0, U_CS + 1, U_CHUNKS)
    ops = []
    for i in range(U_OPS):
        c = int(rng.integers(0, U_CHUNKS + 1))  # U_CHUNKS: a chunk outside the table
        u = rng.random()
        if u < 0.8:
            off = int(rng.integers(0, U_CS))
            ops.append((orc.UPD_WRITE, c, off, int(rng.integers(0, min(U_CS - off, 9000) + 1))))
        elif u < 0.9:
            ops.append((orc.UPD_TRUNCATE, c, 0, int(rng.integers(0, U_CS + 1))))
        else:
            ops.append((orc.UPD_EXTEND, c, 0, int(rng.integers(0, U_CS + 1))))
    return sizes, ops


def _payload(i, n):
    return orc.splitmix_bytes(n, SEED + 1, i) if n else np.zeros(0, dtype=np.uint8)


def _worker(rank, world, port, q, expected):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        h3c = importlib.import_module("3fs_amd")
        shard = importlib.import_module("3fs_amd.shard")
        dev = torch.device("cuda:0")

        def verify(items, exp):  # this rank's contiguous chunk slice, in HBM
            lo, n = items[0], len(items)
            buf = torch.empty(n * CLEN, dtype=torch.uint8, device=dev)
            h3c.fill_splitmix(buf, CLEN, n, CLEN, SEED, first_chunk=lo)
            for c, off, bit in FLIPS:
                if lo <= c < lo + n:
                    k = (c - lo) * CLEN + off
                    buf[k] = buf[k] ^ (1 << bit)
            plan = h3c.Plan.uniform(buf.data_ptr(), CLEN, n, device=0)
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            ok = torch.zeros(n, dtype=torch.uint8, device=dev)
            exp_t = torch.from_numpy(np.asarray(exp, dtype=np.uint32).view(np.int32)).to(dev)
            plan.run(out, expected=exp_t, ok=ok)
            torch.cuda.synchronize()
            plan.close()
            return out.cpu().numpy().view(np.uint32), ok.cpu().numpy().astype(bool)

        raw, ok = shard.run_sharded(list(range(NCHUNKS)), expected, verify, rank, world, lengths=[CLEN] * NCHUNKS)

        # updates: this rank owns a contiguous chunk range; its ops keep their sequence order
        sizes, ops = _update_plan()
        chunk_bytes = [U_CS] * U_CHUNKS
        lo, hi = shard.partition(chunk_bytes, world)[rank]
        slab = torch.zeros(max(hi - lo, 1) * U_CS, dtype=torch.uint8, device=dev)
        for c in range(lo, hi):
            slab[(c - lo) * U_CS:(c - lo) * U_CS + int(sizes[c])] = torch.from_numpy(
                orc.splitmix_bytes(int(sizes[c]), SEED + 2, c)).to(dev)
        table = np.zeros(hi - lo, dtype=h3c.CHUNK_STATE_DTYPE)
        for c in range(lo, hi):
            data = orc.splitmix_bytes(int(sizes[c]), SEED + 2, c)
            table[c - lo] = (slab.data_ptr() + (c - lo) * U_CS, U_CS, int(sizes[c]),
                             orc.crc32c(data) if sizes[c] else 0, orc.CRC32C, 0)
        keep = []

        def apply(idx):
            ios = np.zeros(len(idx), dtype=h3c.UPDATE_IO_DTYPE)
            for k, i in enumerate(idx):
                kind, c, off, ln = ops[i]
                local = c - lo if lo <= c < hi else 0xFFFFFFFF  # outside this rank's table: invalid
                ptr, value, ctype = 0, 0, orc.NONE
                if kind == orc.UPD_WRITE:
                    p = _payload(i, ln)
                    t = torch.from_numpy(np.ascontiguousarray(p)).to(dev) if ln else None
                    keep.append(t)
                    ptr = t.data_ptr() if ln else 0
                    ctype, value = orc.CRC32C, orc.create(orc.CRC32C, p, ln)[1]
                ios[k] = (ptr, local, off, ln, value, ctype, kind, 0, 0, 0)
            return h3c.update_ios(table, ios)

        res = shard.run_sharded_updates([o[1] for o in ops], chunk_bytes, apply, rank, world)
        torch.cuda.synchronize()
        final = [(int(t["size"]), int(t["type"]), int(t["value"])) for t in table]
        finals = [None] * world
        dist.all_gather_object(finals, (lo, final))
        q.put((rank, raw.tolist(), ok.tolist(), res.tolist(), finals))
    except Exception as e:  # surface the failure to the parent instead of hanging it
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_hip_sharded_verify_and_update():
    import torch.multiprocessing as mp

    # oracle side (CPU only): expected checksums of the unflipped chunks, the flipped ones' CRCs
    expected = [orc.crc32c(orc.splitmix_bytes(CLEN, SEED, c)) for c in range(NCHUNKS)]
    want_raw = list(expected)
    for c, off, bit in FLIPS:
        d = orc.splitmix_bytes(CLEN, SEED, c)
        d[off] ^= 1 << bit
        want_raw[c] = orc.crc32c(d)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, expected)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=120)
    for rank, raw, ok, res, finals in got:
        assert ok is not None, raw  # the worker's exception
        assert raw == want_raw, rank
        assert sorted(i for i, x in enumerate(ok) if not x) == sorted(c for c, _, _ in FLIPS)
    assert all(p.exitcode == 0 for p in procs)

    # updates: replay every op through the oracle's ChunkReplica::update on host copies
    sizes, ops = _update_plan()
    host = np.zeros((U_CHUNKS, U_CS), dtype=np.uint8)
    meta = []
    for c in range(U_CHUNKS):
        d = orc.splitmix_bytes(int(sizes[c]), SEED + 2, c)
        host[c, :len(d)] = d
        meta.append({"size": int(sizes[c]), "type": orc.CRC32C, "value": orc.crc32c(d) if sizes[c] else 0})
    want = []
    for i, (kind, c, off, ln) in enumerate(ops):
        if c >= U_CHUNKS:
            want.append((3, 0, 0, 0))
            continue
        p = _payload(i, ln) if kind == orc.UPD_WRITE else None
        io = {"kind": kind, "offset": off, "length": ln, "type": orc.CRC32C if kind == orc.UPD_WRITE else orc.NONE,
              "value": orc.create(orc.CRC32C, p, ln)[1] if kind == orc.UPD_WRITE else 0, "syncing": 0}
        r, meta[c] = orc.replica_update(meta[c], host[c], U_CS, io, p)
        want.append((r["status"], r["size"], r["type"], r["value"] & 0xFFFFFFFF))
    for rank, _, _, res, finals in got:
        # UPDATE_RESULT_DTYPE records: (status, size, value, type, reserved)
        bad = [(i, tuple(r), w) for i, (r, w) in enumerate(zip(res, want))
               if (int(r[0]), int(r[1]), int(r[3]), int(r[2])) != w]
        assert not bad, (rank, bad[:5])
        for lo, final in finals:
            for k, f in enumerate(final):
                m = meta[lo + k]
                assert f == (m["size"], m["type"], m["value"] & 0xFFFFFFFF), (lo + k, f, m)
