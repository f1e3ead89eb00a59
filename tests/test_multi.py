"""The multi-GPU engine's host side (CPU only): the C++ partition behind h3c_multi_* equals
3fs_amd/shard.py::partition, and without a GPU the multi engine fails loudly.

h3c_multi_partition (3fs_amd/csrc/h3c_multi.hip) is what splits every h3c_multi_verify /
h3c_multi_update_ios batch; the Python partition is what the torchrun harness
(bench.py --gpus N, shard.run_sharded) uses.  Both must cut at the same indices, so a C++ storage
service and the harness agree on which GPU owns which chunks.
"""
import importlib

import numpy as np
import pytest

shard = importlib.import_module("3fs_amd.shard")


def _cases():
    rng = np.random.default_rng(20250629)
    yield [], "empty"
    yield [1 << 20], "one"
    yield [0, 0, 0], "zeros"
    yield [1 << 20] * 8192, "config2"
    yield [4 << 20] * 65536, "config4"
    yield [7, 0, 5, 0, 0, 9], "ragged-zeros"
    for k in range(60):
        n = int(rng.integers(1, 300))
        kind = k % 5
        if kind == 0:
            lens = rng.integers(0, 1 << 26, n)
        elif kind == 1:  # config 5: log-uniform 64 KiB .. 64 MiB with 10 % ragged
            lens = (2 ** rng.integers(16, 27, n)).astype(np.int64)
            rag = rng.random(n) < 0.1
            lens[rag] = rng.integers(1, 64 << 20, int(rag.sum()))
        elif kind == 2:
            lens = rng.choice([0, 65536, 1 << 26, 12345], n)
        elif kind == 3:  # one huge chunk among small ones
            lens = rng.integers(1, 4096, n)
            lens[int(rng.integers(0, n))] = 1 << 36
        else:
            lens = rng.integers(1, 4, n)
        yield lens.tolist(), f"random{k}"


@pytest.mark.parametrize("world", range(1, 9))
def test_cpp_partition_equals_shard_partition(h3c, world):
    for lens, name in _cases():
        assert h3c.multi_partition(lens, world) == shard.partition(lens, world), (name, world)


def test_cpp_partition_of_chunk_capacities_matches_partition_updates(h3c):
    """h3c_multi_update_ios splits chunks by capacity exactly as shard.partition_updates does."""
    rng = np.random.default_rng(5)
    cap = rng.integers(1 << 20, 64 << 20, 37).tolist()
    ops = rng.integers(0, 37, 4000)
    for world in (1, 2, 3, 8):
        owner = np.zeros(37, dtype=np.int64)
        for r, (lo, hi) in enumerate(h3c.multi_partition(cap, world)):
            owner[lo:hi] = r
        parts = shard.partition_updates(ops.tolist(), cap, world)
        for r, idx in enumerate(parts):
            assert (owner[ops[idx]] == r).all()


def test_cpp_partition_rejects_bad_world(h3c):
    with pytest.raises(h3c.EngineError) as ei:
        h3c.multi_partition([1, 2], 0)
    assert ei.value.code == 3


def test_multi_engine_without_gpu_fails_loudly(h3c):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(h3c.EngineError) as ei:
        h3c.Multi([0, 0])
    assert ei.value.code in (3, 9001, 9002)
