"""Host-fed pipeline (BASELINE config 5 shapes) vs the oracle: payloads in host memory."""
import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


def mixed_lengths(rng, n):
    lens = []
    for i in range(n):
        L = (64 << 10) << int(rng.integers(0, 9))  # 64 KiB .. 16 MiB here (sizes bounded for the test)
        if i % 10 == 3:
            L -= int(rng.integers(1, 5000))  # ragged tail
        lens.append(L)
    return lens


@pytest.mark.parametrize("window", [1 << 20, 8 << 20, 64 << 20])
def test_hostfed_pinned_contiguous(h3c, torch_dev, window):
    torch, dev = torch_dev
    rng = np.random.default_rng(window)
    lens = mixed_lengths(rng, 40)
    total = sum(lens)
    pinned = torch.from_numpy(rng.integers(0, 256, total + 64, dtype=np.uint8)).pin_memory()
    host = pinned.numpy()
    items, want, off = [], [], 3  # odd start: unaligned host pointers
    for L in lens:
        items.append((pinned[off: off + L], L))
        want.append(orc.crc32c(host[off: off + L]))
        off += L
    hf = h3c.HostFed(0, window)
    got = hf.run(items)
    assert [int(x) for x in got] == want
    exp = np.array(want, dtype=np.uint32)
    bad = [1, 7, 30]
    exp[bad] ^= 0x10
    raw, ok, nbad = hf.run(items, expected=exp)
    assert nbad == 3 and sorted(np.nonzero(~ok)[0].tolist()) == bad
    hf.close()


def test_hostfed_scattered_pageable_and_semantics(h3c, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(9)
    T = h3c.ChecksumType
    bufs = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in (0, 1, 15, 1024, 4096 + 3, 3 << 20, 1 << 20)]
    items = [(b, b.size, 0xFFFFFFFF, T.CRC32C) for b in bufs]
    items.append((None, 10, 0xFFFFFFFF, T.CRC32C))  # null -> NONE -> 0
    items.append((bufs[5], 100, 0x1234, T.NONE))  # NONE -> 0
    items.append((bufs[5], bufs[5].size, 0x5678, T.CRC32C))  # custom start
    hf = h3c.HostFed(0, 1 << 20)
    got = hf.run(items)
    want = [orc.crc32c(b) for b in bufs] + [0, 0, orc.crc32c(bufs[5], 0x5678)]
    assert [int(x) for x in got] == want
    hf.close()


def test_hostfed_crc32_type(h3c, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(4)
    bufs = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in (77, 5 << 20, 999999)]
    hf = h3c.HostFed(0, 2 << 20)
    got = hf.run(bufs, type_=h3c.ChecksumType.CRC32)
    assert [int(x) for x in got] == [orc.crc32(b) for b in bufs]
    hf.close()


def test_hostfed_numa_local_host_buffer(h3c, torch_dev):
    """h3c_host_alloc: pinned pages on the GPU's NUMA node.  The buffer
    reports the node the device sits on (or -1 with no binding), its numpy slices go to the
    pipeline as pinned payloads, and the results match the oracle."""
    from importlib import import_module

    eng = import_module("3fs_amd.engine")
    torch, dev = torch_dev
    rng = np.random.default_rng(5)
    lens = mixed_lengths(rng, 24)
    total = sum(lens) + 64
    hb = h3c.HostBuffer(0, total)
    try:
        assert hb.node in (-1, h3c.device_numa_node(0))
        hb.array[:] = rng.integers(0, 256, total, dtype=np.uint8)
        items, want, off = [], [], 5
        for L in lens:
            items.append((hb.array[off: off + L], L))
            want.append(orc.crc32c(hb.array[off: off + L]))
            off += L
        assert eng._payload(items[0][0], None)[2] == eng.MemKind.HOST_PINNED
        hf = h3c.HostFed(0, 8 << 20)
        raw, ok, nbad = hf.run(items, expected=want)
        hf.close()
        assert nbad == 0 and ok.all() and [int(x) for x in raw] == want
    finally:
        hb.close()
    assert not eng._in_host_buffer(hb.ptr or 1, 1)


def test_hostfed_mixed_types_error_leaves_device_and_pipeline_usable(h3c, torch_dev):
    """A mixed CRC32C / CRC32 run fails with kInvalidArg before any transfer; the caller stays
    on its device and the pipeline keeps working (the early returns restore the device and
    drain the streams before the pinned lease is pooled again)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(12)
    a = rng.integers(0, 256, 5000, dtype=np.uint8)
    b = rng.integers(0, 256, 7000, dtype=np.uint8)
    T = h3c.ChecksumType
    hf = h3c.HostFed(0, 1 << 20)
    before = torch.cuda.current_device()
    with pytest.raises(h3c.EngineError) as ei:
        hf.run([(a, a.size, 0xFFFFFFFF, T.CRC32C), (b, b.size, 0xFFFFFFFF, T.CRC32)])
    assert ei.value.code == 3
    assert torch.cuda.current_device() == before
    got = hf.run([a, b])
    assert [int(x) for x in got] == [orc.crc32c(a), orc.crc32c(b)]
    hf.close()


@pytest.mark.parametrize("window", [8 << 20, 64 << 20])
def test_hostfed_32_and_64_mib_chunks(h3c, torch_dev, window):
    """Config 5's upper size classes: 32 and 64 MiB chunks (split across the staging windows
    when larger than one), a ragged 64 MiB - 4093 B chunk, and small ones between them."""
    torch, dev = torch_dev
    rng = np.random.default_rng(window + 1)
    lens = [32 << 20, 64 << 20, 65536, (64 << 20) - 4093, 1 << 20, 32 << 20]
    total = sum(lens) + 16
    pinned = torch.empty(total, dtype=torch.uint8).pin_memory()
    host = pinned.numpy()
    host[:] = rng.integers(0, 256, total, dtype=np.uint8)
    items, want, off = [], [], 7
    for L in lens:
        items.append((pinned[off: off + L], L))
        want.append(orc.crc32c(host[off: off + L]))
        off += L
    hf = h3c.HostFed(0, window)
    exp = np.array(want, dtype=np.uint32)
    exp[1] ^= 1
    raw, ok, nbad = hf.run(items, expected=exp)
    hf.close()
    assert [int(x) for x in raw] == want
    assert nbad == 1 and np.nonzero(~ok)[0].tolist() == [1]
