"""Multi-rank sharding (CPU, gloo, world_size 2): partition + gather of per-chunk results.

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


def test_gloo_world2_sharded_verify():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] and r[2] for r in res), res
