"""The block-update fused path's per-stream scratch (h3c_update.hip UpdScratch): no per-call memset.

Hash heads, touched marks and look-back granules carry the batch's 8-bit epoch and are never cleared
between batches; the last workgroup resets the control words.  These tests run many batches back to
back on one stream -- sizes that change the hash layout, more batches than the re-zero period (240),
invalid entries (the error count must not leak into the next batch), a void batch followed by good
ones, two streams interleaved, and several threads on one stream -- and check every batch against the
oracle: each chunk's final checksum is the CRC32C of its bytes (oracle C), the last write of each chunk
reports it, the bytes match a host replay, and the invalid count is exact.
"""
import threading

import numpy as np
import pytest

import oracle_lib as orc

pytestmark = pytest.mark.gpu
G = 4096


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    return torch, torch.device("cuda:0")


def i32(arr, torch, dev):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(arr, dtype=np.uint32)).view(np.int32)).to(dev)


class Store:
    """nchunks chunks on the GPU with their host mirror and stored checksums."""

    def __init__(self, torch, dev, rng, nchunks, chunk_len):
        self.torch, self.dev, self.nchunks, self.chunk_len = torch, dev, nchunks, chunk_len
        self.host = rng.integers(0, 256, (nchunks, chunk_len), dtype=np.uint8)
        self.d = torch.from_numpy(self.host.copy()).to(dev)
        self.bases = torch.tensor([self.d[c].data_ptr() for c in range(nchunks)], dtype=torch.int64, device=dev)
        self.raw = np.array([orc.crc32c(self.host[c]) for c in range(nchunks)], dtype=np.uint32)

    def batch(self, h3c, rng, n, n_invalid=0, stream=None, check=True):
        torch, dev = self.torch, self.dev
        bpc = self.chunk_len // G
        wc = rng.integers(0, self.nchunks, n).astype(np.uint32)
        wb = rng.integers(0, bpc, n).astype(np.uint32)
        bad = rng.choice(n, size=min(n_invalid, n), replace=False) if n_invalid else []
        for k in bad:
            wb[k] = bpc + int(rng.integers(0, 5))  # out of range: no effect, counted
        pay = rng.integers(0, 256, (n, G), dtype=np.uint8)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        raw_out = torch.zeros(self.nchunks, dtype=torch.int32, device=dev)
        ninv = torch.full((1,), -7, dtype=torch.int32, device=dev)
        args = (i32(self.raw, torch, dev), i32(wc, torch, dev), i32(wb, torch, dev), torch.from_numpy(pay).to(dev))
        h3c.update_blocks(self.bases, self.chunk_len, args[0], args[1], args[2], args[3], out, raw_out,
                          n_invalid=ninv, stream=stream)
        if stream is not None:
            stream.synchronize()
        torch.cuda.synchronize()
        for k in range(n):
            if wb[k] < bpc:
                self.host[wc[k], wb[k] * G:(wb[k] + 1) * G] = pay[k]
        fin = raw_out.cpu().numpy().view(np.uint32).copy()
        got = out.cpu().numpy().view(np.uint32)
        if check:
            assert int(ninv.item()) == len(bad)
            want = np.zeros(self.nchunks, dtype=np.uint32)
            orc.lib().orc_batch_crc32c(self.host.ctypes.data, self.chunk_len, self.nchunks, 0xFFFFFFFF, 8, 0,
                                       want.ctypes.data)
            assert np.array_equal(fin, want), np.nonzero(fin != want)[0][:8]
            for c in range(self.nchunks):
                ks = np.nonzero((wc == c) & (wb < bpc))[0]
                if len(ks):
                    assert int(got[ks[-1]]) == int(want[c]), c
            assert np.array_equal(self.d.cpu().numpy(), self.host)
        self.raw = fin
        return int(ninv.item())


def test_scratch_many_batches_sizes_and_invalid(h3c, torch_dev, hooks):
    """260 batches on one stream (past the 240-batch re-zero), sizes crossing hash-size powers of two
    (a new layout each time), every fifth batch with invalid entries."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(501)
    st = Store(torch, dev, rng, 8, 256 << 10)
    sizes = [1, 5, 64, 300, 255, 257, 1000, 3000, 511, 513, 2048, 4100]
    for b in range(260):
        n = sizes[b % len(sizes)] if b < 36 else int(rng.integers(200, 700))
        st.batch(h3c, rng, n, n_invalid=(3 if b % 5 == 0 else 0))


def test_scratch_void_batch_then_good_batches(h3c, torch_dev, hooks):
    """A batch whose look-back gives up (H3C_HOOK_UPD_LOOKBACK) reports void; the next batches on the
    same scratch are exact (the timeout flag and the counts were put back)."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(502)
    st = Store(torch, dev, rng, 8, 256 << 10)
    st.batch(h3c, rng, 3000)
    hooks(h3c.HOOK_UPD_LOOKBACK, 1)
    assert st.batch(h3c, rng, 20000, check=False) == -1
    hooks(h3c.HOOK_UPD_LOOKBACK, 0)
    st.raw = np.array([orc.crc32c(st.host[c]) for c in range(st.nchunks)], dtype=np.uint32)  # recomputed
    for n in (20000, 3000, 20000):
        st.batch(h3c, rng, n, n_invalid=2)


def test_scratch_two_streams_interleaved(h3c, torch_dev, hooks):
    """Two streams (two scratches), batches alternating between them on disjoint chunk sets."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(503)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    stores = [Store(torch, dev, rng, 4, 128 << 10), Store(torch, dev, rng, 6, 128 << 10)]
    for b in range(40):
        k = b % 2
        stores[k].batch(h3c, rng, int(rng.integers(1, 2500)), n_invalid=b % 3, stream=streams[k])


def test_scratch_more_streams_than_the_table_and_release(h3c, torch_dev, hooks):
    """72 streams, each one batch then another round (more than the 64 scratches the library keeps: the
    least recently used idle one is evicted and reused), then every stream released before it goes
    (h3c_stream_release); all batches exact.  (scratches were never freed, a 65th stream fell
    back to the workspace for good, and a recycled stream handle inherited a live scratch.)"""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(505)
    streams = [torch.cuda.Stream() for _ in range(72)]
    store = Store(torch, dev, rng, 4, 128 << 10)
    for rnd in range(2):
        for k, s in enumerate(streams):
            store.batch(h3c, rng, int(rng.integers(100, 1200)), n_invalid=k % 2, stream=s)
    for s in streams:
        h3c.stream_release(s)
    h3c.stream_release(streams[0])  # (again: nothing left to release)
    store.batch(h3c, rng, 2000, stream=streams[3])  # a released stream gets a fresh scratch


def test_scratch_threads_on_one_stream(h3c, torch_dev, hooks):
    """Four threads issue batches on the same (default) stream without waiting on each other: each
    call's launches are enqueued whole, so each thread's chunks end exact."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    seeds = np.random.SeedSequence(504).spawn(4)
    stores = [Store(torch, dev, np.random.default_rng(s), 4, 128 << 10) for s in seeds]
    errors = []

    def work(i):
        try:
            torch.cuda.set_device(dev)
            rng = np.random.default_rng(seeds[i])
            for _ in range(12):
                stores[i].batch(h3c, rng, int(rng.integers(100, 3000)), n_invalid=1)
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append((i, repr(e)))

    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_fused_path_chunk_boundaries_inside_cache_lines(h3c, torch_dev, hooks):
    """Chunks laid out 64 bytes past a 128-byte line boundary, so every chunk boundary falls inside a cache
    line: writes to the last block of chunk c and the first block of chunk c+1 touch the same lines from
    different workgroups (the fused path's write-back is by plain stores since round 5, held in each XCD's
    L2 until the launch ends).  Bytes and checksums against the oracle."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(505)
    nchunks, clen = 16, 64 << 10
    bpc = clen // G
    host = rng.integers(0, 256, (nchunks, clen), dtype=np.uint8)
    buf = torch.zeros(nchunks * clen + 256, dtype=torch.uint8, device=dev)
    off = 64 + (-buf.data_ptr()) % 128  # every chunk starts 64 bytes into a 128-byte line
    assert (buf.data_ptr() + off) % 128 == 64 and off + nchunks * clen <= buf.numel()
    view = buf[off: off + nchunks * clen].view(nchunks, clen)
    view.copy_(torch.from_numpy(host))
    bases = torch.tensor([view[c].data_ptr() for c in range(nchunks)], dtype=torch.int64, device=dev)
    raw = np.array([orc.crc32c(host[c]) for c in range(nchunks)], dtype=np.uint32)
    for it in range(3):
        wc, wb = [], []
        for c in range(nchunks):  # each chunk's first and last block, in an order that spreads them apart
            wc += [c, c]
            wb += [0, bpc - 1]
        extra = 3000
        wc += list(rng.integers(0, nchunks, extra))
        wb += list(rng.integers(0, bpc, extra))
        order = rng.permutation(len(wc))
        wc = np.array(wc, dtype=np.uint32)[order]
        wb = np.array(wb, dtype=np.uint32)[order]
        n = len(wc)
        pay = rng.integers(0, 256, (n, G), dtype=np.uint8)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        raw_out = torch.zeros(nchunks, dtype=torch.int32, device=dev)
        h3c.update_blocks(bases, clen, i32(raw, torch, dev), i32(wc, torch, dev), i32(wb, torch, dev),
                          torch.from_numpy(pay).to(dev), out, raw_out)
        torch.cuda.synchronize()
        for k in range(n):
            host[wc[k], wb[k] * G:(wb[k] + 1) * G] = pay[k]
        want = np.array([orc.crc32c(host[c]) for c in range(nchunks)], dtype=np.uint32)
        got = raw_out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), (it, np.nonzero(got != want)[0][:8])
        assert np.array_equal(view.cpu().numpy(), host), it
        assert int(buf[:off].sum().item()) == 0 and int(buf[off + nchunks * clen:].sum().item()) == 0  # no stray bytes
        raw = want


def test_fused_path_captured_into_a_caller_graph(h3c, torch_dev, hooks):
    """A caller that captures h3c_update_blocks into its own graph gets the workspace form (the per-stream
    scratch is never baked into a capture): three replays of [update; raw_in <- raw_out] against the oracle."""
    torch, dev = torch_dev
    hooks(h3c.HOOK_UPD_SCAN, h3c.UPD_SCAN_PATHS["fused"])
    rng = np.random.default_rng(506)
    st = Store(torch, dev, rng, 8, 256 << 10)
    st.batch(h3c, rng, 500)  # (the shift table is cached before the capture)
    n = 3000
    bpc = st.chunk_len // G
    wc = rng.integers(0, st.nchunks, n).astype(np.uint32)
    wb = rng.integers(0, bpc, n).astype(np.uint32)
    pay = rng.integers(0, 256, (n, G), dtype=np.uint8)
    d_wc, d_wb, d_pay = i32(wc, torch, dev), i32(wb, torch, dev), torch.from_numpy(pay).to(dev)
    raw_in = i32(st.raw, torch, dev)
    raw_out = torch.zeros_like(raw_in)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ws = torch.empty(h3c.update_workspace_bytes(n, st.nchunks, st.chunk_len, G), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        h3c.update_blocks(st.bases, st.chunk_len, raw_in, d_wc, d_wb, d_pay, out, raw_out, workspace=ws)
        raw_in.copy_(raw_out)
    torch.cuda.synchronize()
    for rep in range(3):
        g.replay()
        torch.cuda.synchronize()
        for k in range(n):
            st.host[wc[k], wb[k] * G:(wb[k] + 1) * G] = pay[k]
        want = np.zeros(st.nchunks, dtype=np.uint32)
        orc.lib().orc_batch_crc32c(st.host.ctypes.data, st.chunk_len, st.nchunks, 0xFFFFFFFF, 8, 0, want.ctypes.data)
        got = raw_out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), (rep, np.nonzero(got != want)[0][:8])
        assert np.array_equal(st.d.cpu().numpy(), st.host), rep
