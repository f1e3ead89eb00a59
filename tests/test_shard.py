"""Multi-rank sharding (CPU, gloo, world_size 2 and 4): partition + gather of per-chunk results.

The per-rank compute function here is the oracle (this runs without a GPU); on
the GPU box the same run_sharded() drives the HIP engine, one rank per GPU.
"""
import importlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_lib as orc

shard = importlib.import_module("3fs_amd.shard")


def test_partition_properties():
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 4, 8):
        for n in (0, 1, 5, 100, 8192):
            lens = rng.integers(1 << 16, 1 << 26, n).tolist()
            parts = shard.partition(lens, world)
            assert len(parts) == world
            assert parts[0][0] == 0 and parts[-1][1] == n
            for (a, b), (c, d) in zip(parts, parts[1:]):
                assert b == c and a <= b
            if n >= world * 4:
                tot = sum(lens)
                mx = max(lens)
                for a, b in parts:
                    assert abs(sum(lens[a:b]) - tot / world) <= mx


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)  # same batch on every rank
        lens = rng.integers(1, 200000, 64).tolist()
        items = [orc.splitmix_bytes(n, 7, i) for i, n in enumerate(lens)]
        expected = [orc.crc32c(d) for d in items]
        bad = {3, 17, 40}
        for b in bad:
            expected[b] ^= 1

        def verify(its, exp):
            raw = [orc.crc32c(d) for d in its]
            return raw, [r == e for r, e in zip(raw, exp)]

        raw, ok = shard.run_sharded(items, expected, verify, rank, world, lengths=lens)
        want_raw = np.array([orc.crc32c(d) for d in items], dtype=np.uint32)
        q.put((rank, bool(np.array_equal(raw, want_raw)), sorted(np.nonzero(~ok)[0].tolist()) == sorted(bad)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_sharded_verify(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] and r[2] for r in res), res


def test_partition_updates_keeps_chunks_on_one_rank():
    rng = np.random.default_rng(1)
    nchunks = 37
    cb = rng.integers(1 << 20, 64 << 20, nchunks).tolist()
    ops = rng.integers(-1, nchunks + 2, 5000).tolist()
    for world in (1, 2, 3, 8):
        parts = shard.partition_updates(ops, cb, world)
        seen = np.concatenate(parts)
        assert sorted(seen.tolist()) == list(range(len(ops)))
        owner = {}
        for r, idx in enumerate(parts):
            assert np.all(np.diff(idx) > 0)  # sequence order kept
            for i in idx:
                c = ops[i]
                if 0 <= c < nchunks:
                    assert owner.setdefault(c, r) == r


def _upd_worker(rank, world, port, q):
    """Each rank replays its chunks' ops through the ChunkReplica::update restatement; the
    gathered per-op results must equal a single-rank replay of the whole sequence."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(9)
        nchunks, cs = 6, 16384
        ops = []
        for _ in range(400):
            c = int(rng.integers(0, nchunks))
            off = int(rng.integers(0, cs))
            ln = int(rng.integers(0, min(cs - off, 3000) + 1))
            p = rng.integers(0, 256, ln, dtype=np.uint8)
            ops.append((c, {"kind": orc.UPD_WRITE, "offset": off, "length": ln, "type": orc.CRC32C,
                            "value": orc.create(orc.CRC32C, p, ln)[1]}, p))

        def replay(idx):
            chunks = np.zeros((nchunks, cs), dtype=np.uint8)
            meta = [{"size": 0, "type": orc.NONE, "value": 0} for _ in range(nchunks)]
            out = np.zeros(len(idx), dtype=np.int64)
            for k, i in enumerate(idx):
                c, io, p = ops[i]
                res, meta[c] = orc.replica_update(meta[c], chunks[c], cs, io, p)
                out[k] = (res["status"] << 40) | (res["size"] << 32) | res["value"]
            return out

        got = shard.run_sharded_updates([o[0] for o in ops], [cs] * nchunks, replay, rank, world)
        want = replay(list(range(len(ops))))
        q.put((rank, bool(np.array_equal(got, want))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_sharded_updates(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_upd_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
