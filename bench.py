#!/usr/bin/env python3
"""Benchmarks of the MI355X chunk-checksum engine (BASELINE.json configs).

Default (the headline, BASELINE config 2): a step = one batch verify of 8192 x 1 MiB
device-resident chunks per GPU -- recompute every chunk's CRC32C, compare with the
stored value, count mismatches.  That is ChunkReplica::update's payload verify /
AioReadJob::setResult's recalculate path (src/storage/store/ChunkReplica.cc:193-207,
src/storage/aio/BatchReadJob.cc:43-54) batched.  Inputs are resident in HBM before
the timed region starts.

The default line also carries two sub-passes that are never its `value`: `hostfed` (a short
BASELINE config-5 pass, PCIe-inclusive) and `update` (BASELINE config 3 through h3c_update_ios_dev,
100k random 4 KiB UpdateIOs into 64 x 64 MiB chunks, 10 warm + 20 timed batches, a CPU-oracle
check of sampled chunks, its own roofline and case-(iv) CPU baseline).

Other workloads (--workload), each printing its own JSON line:
  update   BASELINE config 3: 100k random 4 KiB writes into 64 x 64 MiB chunks,
           per-write chunk checksum (ChunkReplica::updateChecksum) -> writes/s
  hostfed  BASELINE config 5: mixed 64 KiB-64 MiB chunks in pinned host memory,
           H2D double-buffered against the CRC -> GiB/s (PCIe-inclusive)
  shard4m  BASELINE config 4: 256 GiB as 4 MiB chunks split over the ranks (strong
           scaling), generated in HBM in passes

Multi-GPU: one process per GPU (torchrun); chunks are sharded, there is no data-path
collective.  torch.distributed is used only for the barrier and max-over-ranks time.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 20250629
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md
PCIE_SPEC_GBPS = 63.0  # PCIe Gen5 x16 (spec)
METRIC = "GiB/s CRC32C verified (1 MiB chunks) at 1/2/4/8 GPUs; % of HBM peak"


# --------------------------------------------------------------------------- helpers


def _oracle():
    """CPU oracle library (oracle/) -- used only by the cpu_baseline legs."""
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess

        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    L = ctypes.CDLL(so)
    L.orc_fill_splitmix.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    L.orc_batch_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.orc_has_vpclmul.restype = ctypes.c_int
    return L


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(gpu_raw_first: np.ndarray, chunk_len: int, seconds: float = 8.0) -> dict:
    """Reference CPU path restated (oracle/, folly-faithful 3-stream SSE4.2 crc32q) on this host.

    Sample: 1024 x 1 MiB splitmix chunks (BASELINE config 1), ChecksumInfo::create
    semantics, 1 host thread, repeated for ~`seconds`.  The same pass also checks
    the GPU's values for those chunk indices."""
    L = _oracle()
    n = 1024
    host = np.empty(n * chunk_len, dtype=np.uint8)
    for c in range(n):
        L.orc_fill_splitmix(host[c * chunk_len:].ctypes.data, chunk_len, SEED, c)
    out = np.zeros(n, dtype=np.uint32)
    # one thread pinned to one core ("one thread pinned with taskset"): the calling
    # thread's affinity, which the oracle's worker pthread inherits; restored afterwards
    allowed = sorted(os.sched_getaffinity(0))
    core = allowed[0]
    os.sched_setaffinity(0, {core})
    try:
        L.orc_batch_crc32c(host.ctypes.data, chunk_len, n, 0xFFFFFFFF, 1, 0, out.ctypes.data)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            L.orc_batch_crc32c(host.ctypes.data, chunk_len, n, 0xFFFFFFFF, 1, 0, out.ctypes.data)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        os.sched_setaffinity(0, set(allowed))
    gibps = reps * n * chunk_len / el / 2**30
    # context only (BASELINE.md "all-cores run"): the same restatement on every core this
    # process may use (the GPU box grants a share of the host, not all of nproc)
    threads = max(1, min(len(os.sched_getaffinity(0)), 16))  # the GPU box grants 16 CPUs per GPU
    reps_mt, t0 = 0, time.perf_counter()
    while True:
        L.orc_batch_crc32c(host.ctypes.data, chunk_len, n, 0xFFFFFFFF, threads, 0, out.ctypes.data)
        reps_mt += 1
        el_mt = time.perf_counter() - t0
        if el_mt >= min(2.0, seconds):
            break
    # context only: best-case CPU ("PCLMUL-folding variant"), not the reference's
    # path -- AVX-512 VPCLMULQDQ folding, 1 thread (falls back to the 3-way path without it)
    has_vpclmul = bool(L.orc_has_vpclmul())
    reps_v, t0 = 0, time.perf_counter()
    while True:
        L.orc_batch_crc32c(host.ctypes.data, chunk_len, n, 0xFFFFFFFF, 1, 3, out.ctypes.data)
        reps_v += 1
        el_v = time.perf_counter() - t0
        if el_v >= min(2.0, seconds):
            break
    return {
        "value": round(gibps, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{reps} x (1024 x {chunk_len >> 20} MiB splitmix chunks), folly-faithful 3-way SSE4.2 crc32q, "
                  f"1 thread pinned to core {core}, {el:.1f} s",
        "pinned_core": core,
        "gpu_values_match": bool(np.array_equal(out, gpu_raw_first[:n])),
        "cpu_model": _cpu_model(),
        "nproc": os.cpu_count(),
        "context_all_cores": {"value": round(reps_mt * n * chunk_len / el_mt / 2**30, 3), "unit": "GiB/s",
                              "threads": threads, "seconds": round(el_mt, 2)},
        "context_best_case_cpu": {"value": round(reps_v * n * chunk_len / el_v / 2**30, 3), "unit": "GiB/s",
                                  "cores": 1, "variant": "AVX-512 VPCLMULQDQ folding" if has_vpclmul
                                  else "unavailable (3-way fallback)", "reference_faithful": False},
    }


def pmc_traffic(bytes_per_launch: int, kernel: str = "seg_crc_kernel"):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/*_pmc_summary.json,
    scripts/profile_r1.sh + summarize_prof.py: FETCH_SIZE / WRITE_SIZE in separate passes,
    gfx950 FETCH_SIZE x2).  Only used when that profile was taken on this same per-launch
    workload."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("kernel", "seg_crc_kernel") != kernel:
            continue
        t = d.get("pmc", {}).get("traffic_bytes_per_launch")
        if t and abs(d.get("algorithmic_bytes_per_launch", 0) - bytes_per_launch) < 1:
            k = d.get(kernel, {})
            best = (t, os.path.basename(f), k.get("avg_us_last_half") or k.get("avg_us"))
    return best


class Ctx:
    def __init__(self):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        # one process per GPU; modulo only matters for single-GPU rehearsals of N>1
        self.ndev = torch.cuda.device_count()
        self.local = int(os.environ.get("LOCAL_RANK", "0")) % max(self.ndev, 1)
        if self.world > 1:
            # Control plane only (barrier, max-over-ranks time, verified flag): no data
            # path collective exists, so gloo on CPU tensors is enough; set
            # H3C_DIST_BACKEND=nccl to use RCCL instead.
            backend = os.environ.get("H3C_DIST_BACKEND", "gloo")
            kw = {"device_id": torch.device(f"cuda:{self.local}")} if backend == "nccl" else {}
            dist.init_process_group(backend, **kw)
            self.cdev = torch.device(f"cuda:{self.local}") if backend == "nccl" else torch.device("cpu")
        torch.cuda.set_device(self.local)
        self.dev = torch.device(f"cuda:{self.local}")
        self.h3c = importlib.import_module("3fs_amd")
        self.stream = torch.cuda.current_stream()

    def barrier(self):
        self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def max_over_ranks(self, v: float) -> float:
        if self.world == 1:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def all_true(self, b: bool) -> bool:
        if self.world == 1:
            return b
        t = self.torch.tensor([1 if b else 0], dtype=self.torch.int32, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return bool(t.item())

    def timed(self, step, steps: int, warmup: int, kind: int, after_warmup=None):
        """warmup, barrier, time `steps` calls (max over ranks); returns (elapsed_s, prof)."""
        for _ in range(warmup):
            step()
        self.barrier()
        if after_warmup:
            after_warmup()
        self.h3c.profile_read(reset=True, kind=kind)
        self.h3c.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        self.barrier()
        t1 = time.perf_counter()
        self.h3c.profile_enable(False)
        prof = self.h3c.profile_read(reset=True, kind=kind)
        return self.max_over_ranks(t1 - t0), prof


# Measured ceilings of the access patterns themselves (no CRC work), for context beside the
# 8 TB/s spec peak: streaming reads of per-wave contiguous segments (scripts/readbw.hip) and
# the update kernel's random 4 KiB read-modify-write (scripts/rmwbw.hip).
PLAIN_STORE_KERNELS = ("upd_fused_kernel", "uio_afused_kernel")  # write-back by plain stores (round 5)
PATTERN_CEILING = {
    "seg_crc_kernel": (6905.0, "profiles/r01_readbw_ceiling.txt"),
    "seg_quad_kernel": (6905.0, "profiles/r01_readbw_ceiling.txt"),
    "seg_uni_kernel": (6905.0, "profiles/r01_readbw_ceiling.txt"),
    # config 3's pattern: the best payload+old read alone plus the best plain write alone, back to back
    # (198.8 us per 100k writes = 6,181 GB/s of the 12 KiB per write; the round-5 kernels beat the probe's
    # own mixed rmw loop, so that is no ceiling: profiles/r05_rmw_ceiling.txt)
    "upd_delta_kernel": (6181.0, "profiles/r05_rmw_ceiling.txt"),
    "upd_fused_kernel": (6181.0, "profiles/r05_rmw_ceiling.txt"),
    "uio_block_kernel": (6181.0, "profiles/r05_rmw_ceiling.txt"),
    "uio_fast_kernel": (6181.0, "profiles/r05_rmw_ceiling.txt"),
    "uio_afused_kernel": (6181.0, "profiles/r05_rmw_ceiling.txt"),
}


def roofline(prof, peak: float, unit: str = "GB/s", bound: str = "hbm", kernel: str = "seg_crc_kernel"):
    ms, launches, nbytes = prof
    per = nbytes / max(launches, 1)
    avg_s = ms / 1e3 / max(launches, 1)
    achieved = per / avg_s / 1e9 if launches and avg_s > 0 else 0.0
    r = {"bound": bound, "achieved": round(achieved, 1), "peak": peak, "unit": unit,
         "frac": round(achieved / peak, 4), "traffic": None, "kernel": kernel,
         "kernel_avg_us": round(avg_s * 1e6, 2), "algorithmic_bytes_per_launch": int(per)}
    tr = pmc_traffic(int(per), kernel)
    if tr:
        r["traffic"] = int(tr[0])
        r["traffic_source"] = f"profiles/{tr[1]}"
        if tr[2]:  # the same kernel's rocprof duration in that profile (its settled second half, where recorded)
            r["rocprof_avg_us"] = round(tr[2], 2)
            r["frac_rocprof"] = round(per / (tr[2] * 1e-6) / 1e9 / peak, 4)
            if kernel in PLAIN_STORE_KERNELS:
                # the kernel's own stamps end before the end-of-launch L2 write-back of its plain stores,
                # which rocprof's duration covers: lead with the slower of the two
                r["frac_stamps"] = r["frac"]
                r["achieved_stamps"] = r["achieved"]
                if tr[2] > r["kernel_avg_us"]:
                    achieved = per / (tr[2] * 1e-6) / 1e9
                    r["achieved"] = round(achieved, 1)
                    r["frac"] = r["frac_rocprof"]
                    r["frac_source"] = "rocprof (committed profile of this launch shape): slower than the stamps"
                r["timing_note"] = ("kernel_avg_us: the kernel's own stamps, first workgroup start to last workgroup "
                                    "end; rocprof's duration also covers the end-of-launch L2 write-back of its plain "
                                    "stores, so `frac` is the slower of the two")
    if kernel in PATTERN_CEILING:
        ceil, src = PATTERN_CEILING[kernel]
        r["pattern_ceiling"] = {"achieved": ceil, "frac": round(achieved / ceil, 4), "source": src}
        if src.endswith("r05_rmw_ceiling.txt"):
            r["pattern_ceiling"]["kind"] = ("synthetic: the best read-only probe and the best write-only probe timed "
                                            "separately and summed (not a measured read-modify-write loop)")
    return r


# --------------------------------------------------------------------------- workloads


def run_verify(args, cx: Ctx) -> dict:
    torch, h3c = cx.torch, cx.h3c
    n, clen = args.chunks, args.chunk_kib << 10
    buf = torch.empty(n * clen, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(buf, clen, n, clen, SEED, first_chunk=cx.rank * n)  # rank r: chunks [r*n, (r+1)*n)
    torch.cuda.synchronize()
    plan = h3c.Plan.uniform(buf.data_ptr(), clen, n, device=cx.local)
    # Stored checksums = a create pass; then corrupt flip_frac of the chunks.
    stored = torch.zeros(n, dtype=torch.int32, device=cx.dev)
    plan.run(stored, stream=cx.stream)
    torch.cuda.synchronize()
    stored_host = stored.cpu().numpy().view(np.uint32).copy()
    g = torch.Generator().manual_seed(SEED + cx.rank)
    nflip = int(n * args.flip_frac)
    flips = torch.randperm(n, generator=g)[:nflip].sort().values
    pos = flips * clen + torch.randint(0, clen, (nflip,), generator=g)
    bits = (1 << torch.randint(0, 8, (nflip,), generator=g)).to(torch.uint8)
    pos_d = pos.to(cx.dev)
    buf[pos_d] ^= bits.to(cx.dev)

    out = torch.zeros(n, dtype=torch.int32, device=cx.dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=cx.dev)
    mis = torch.zeros(1, dtype=torch.int32, device=cx.dev)

    def step():
        mis.zero_()
        plan.run(out, expected=stored, ok=ok, mismatch=mis, stream=cx.stream)

    elapsed, prof = cx.timed(step, args.steps, args.warmup, h3c.engine.PROF_SEG)
    bad = np.nonzero(ok.cpu().numpy() == 0)[0]
    verified = cx.all_true(int(mis.item()) == nflip and np.array_equal(bad, flips.numpy()))
    plan.close()
    value = n * clen * args.steps * cx.world / elapsed / 2**30
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": cx.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 chunks generated in HBM; 5% of chunks carry one flipped bit)",
        "config": {
            "workload": f"batched CRC32C verify of {n} x {clen >> 10} KiB device-resident chunks per GPU"
                        + (" (BASELINE config 2)" if (n, clen) == (8192, 1 << 20) else " (chunk-size sweep)"),
            "chunks_per_gpu": n,
            "chunk_bytes": clen,
            "parallelism": f"shard{cx.world}",
        },
        "verified": verified,
        "pct_hbm_peak": round(100.0 * (n * clen) / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS, 2),
        # chunks of <= 16 KiB (one segment each) run the small-chunk kernel
        # (a uniform plan of such chunks, rows of 64 / 256 bytes: seg_uni_kernel, §4.1 5c)
        "roofline": roofline(prof, HBM_PEAK_GBPS, kernel=("seg_uni_kernel" if clen % 64 == 0 else "seg_quad_kernel")
                             if clen <= (16 << 10) else "seg_crc_kernel"),
    }
    if cx.world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(stored_host, clen, args.cpu_seconds)
    return res


def run_inproc(args, cx: Ctx, devices) -> dict:
    """The product path over several GPUs of ONE process (h3c_multi_*): one worker thread
    per entry of `devices`, each holding `chunks` x `chunk_kib` resident on its device (chunk indices
    [k*n, (k+1)*n) on device k, 5% flipped), verified as one batch per step through
    h3c_multi_plan_verify -- host arrays in and out, as a C++ storage service calls it.  The byte-balanced
    partition puts device k's share on worker k."""
    torch, h3c = cx.torch, cx.h3c
    n, clen = args.chunks, args.chunk_kib << 10
    W = len(devices)
    bufs, descs, flips_all, stored = [], [], [], []
    m = h3c.Multi(devices)
    try:
        for k, dv in enumerate(devices):
            dev = torch.device(f"cuda:{dv}")
            buf = torch.empty(n * clen, dtype=torch.uint8, device=dev)
            with torch.cuda.device(dev):
                h3c.fill_splitmix(buf, clen, n, clen, SEED, first_chunk=k * n)
            d = np.zeros(n, dtype=h3c.engine.DESC_DTYPE)
            d["ptr"] = buf.data_ptr() + np.arange(n, dtype=np.uint64) * np.uint64(clen)
            d["len"] = clen
            d["start_raw"] = 0xFFFFFFFF
            d["type"] = 1
            d["mem"] = 0
            bufs.append(buf)
            descs.append(d)
        for dv in set(devices):
            torch.cuda.synchronize(dv)
        d = np.concatenate(descs)
        _, want = m.batch_create(d)  # the stored checksums (h3c_multi_batch_create)
        g = torch.Generator().manual_seed(SEED + 17)
        for k, buf in enumerate(bufs):
            nflip = int(n * args.flip_frac)
            fl = torch.randperm(n, generator=g)[:nflip].sort().values
            pos = fl * clen + torch.randint(0, clen, (nflip,), generator=g)
            bits = (1 << torch.randint(0, 8, (nflip,), generator=g)).to(torch.uint8)
            pos_d = pos.to(buf.device)
            buf[pos_d] ^= bits.to(buf.device)
            flips_all.append(fl.numpy() + k * n)
        for dv in set(devices):
            torch.cuda.synchronize(dv)
        plan = m.plan(d)
        try:
            for _ in range(args.warmup):
                plan.verify(want)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                nbad = plan.verify(want)
            el = time.perf_counter() - t0
            stats = m.last_stats()
            flips = np.concatenate(flips_all)
            bad = np.nonzero(plan.ok == 0)[0]
            ok = nbad == flips.size and np.array_equal(bad, flips)
            ok = ok and np.array_equal(np.delete(plan.out, flips), np.delete(want, flips))
        finally:
            plan.close()
    finally:
        m.close()
    total = W * n * clen
    return {
        "metric": METRIC, "value": round(total * args.steps / el / 2**30, 2), "unit": "GiB/s",
        "n_gpus": len(set(devices)), "workers": W, "devices": list(devices), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 chunks generated in HBM; 5% of chunks carry one flipped bit)",
        "config": {"workload": f"{n} x {clen >> 10} KiB device-resident chunks per worker, verified as one batch "
                               f"through h3c_multi_plan_verify (host expected / results arrays, one process)",
                   "parallelism": f"inproc{W}", "launcher": "in-process (h3c_multi)"},
        "verified": bool(ok),
        "per_worker": [{"device": dv, "chunks": u, "bytes": b, "last_ms": round(ms, 3)}
                       for dv, (u, b, ms) in zip(devices, stats)],
        "note": "wall time of whole synchronous calls: expected values in, results and flags out over PCIe",
    }


def cpu_baseline_update(samples: int = 40) -> dict:
    """The reference algorithm on the host: ChunkReplica::updateChecksum case (iv) for a 4 KiB
    overwrite of a 64 MiB chunk = CRC of the prefix + suffix (the whole chunk minus the write)
    + CRC of the write + 2 combines, prefix/suffix read from memory (not disk).  Timed on
    `samples` writes and extrapolated to writes/s."""
    L = _oracle()
    L.orc_crc32c_sse42_3way.restype = ctypes.c_uint32
    L.orc_crc32c_sse42_3way.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    L.orc_crc32c_combine.restype = ctypes.c_uint32
    L.orc_crc32c_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    clen, G = 64 << 20, 4096
    chunk = np.empty(clen, dtype=np.uint8)
    L.orc_fill_splitmix(chunk.ctypes.data, clen, SEED, 0)
    rng = np.random.default_rng(1)
    offs = rng.integers(0, clen // G, samples) * G
    base = chunk.ctypes.data
    t0 = time.perf_counter()
    for off in offs:
        off = int(off)
        pre = L.orc_crc32c_sse42_3way(base, off, 0xFFFFFFFF)
        w = L.orc_crc32c_sse42_3way(base + off, G, 0xFFFFFFFF)
        suf = L.orc_crc32c_sse42_3way(base + off + G, clen - off - G, 0xFFFFFFFF)
        v = L.orc_crc32c_combine((~pre) & 0xFFFFFFFF, w, G)
        v = L.orc_crc32c_combine((~v) & 0xFFFFFFFF, suf, clen - off - G)
    el = time.perf_counter() - t0
    return {"value": round(samples / el, 2), "unit": "writes/s", "cores": 1, "kind": "port",
            "sample": f"{samples} writes of 4 KiB into a 64 MiB chunk via updateChecksum case (iv) "
                      f"(prefix+write+suffix CRC, 2 combines), {el:.2f} s, extrapolated",
            "cpu_model": _cpu_model()}


def run_update(args, cx: Ctx) -> dict:
    torch, h3c = cx.torch, cx.h3c
    nchunks, clen, nw, G = 64, 64 << 20, args.writes, 4096
    bpc = clen // G
    chunks = torch.empty(nchunks * clen, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(chunks, clen, nchunks, clen, SEED, first_chunk=cx.rank * nchunks)
    payload = torch.empty(nw * G, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(payload, G, nw, G, SEED + 1, first_chunk=cx.rank * nw)
    # `tables` seeded write tables in rotation (as run_updio): each step applies the next table on top of the
    # previous state, so the kernel's per-XCD range weights never see the same batch twice in a row
    ntab = max(1, int(getattr(args, "update_tables", 4)))
    tabs = []
    for t in range(ntab):
        g = torch.Generator().manual_seed(SEED + cx.rank + 7919 * t)
        tabs.append((torch.randint(0, nchunks, (nw,), generator=g, dtype=torch.int32).to(cx.dev),
                     torch.randint(0, bpc, (nw,), generator=g, dtype=torch.int32).to(cx.dev)))
    plan = h3c.Plan.uniform(chunks.data_ptr(), clen, nchunks, device=cx.local)
    raw = [torch.zeros(nchunks, dtype=torch.int32, device=cx.dev) for _ in range(2)]
    plan.run(raw[0], stream=cx.stream)
    bases = torch.arange(nchunks, dtype=torch.int64, device=cx.dev) * clen + chunks.data_ptr()
    out = torch.zeros(nw, dtype=torch.int32, device=cx.dev)
    ws = torch.empty(h3c.update_workspace_bytes(nw, nchunks, clen, G), dtype=torch.uint8, device=cx.dev)
    ctr = torch.zeros(8, dtype=torch.int64, device=cx.dev)
    exact = bool(getattr(args, "exact", False))
    cur = [0, 0]

    def step():  # the next table on top of the previous state: same traffic, new checksums
        i = cur[0]
        wc, wb = tabs[cur[1] % ntab]
        h3c.update_blocks(bases, clen, raw[i], wc, wb, payload, out, raw[1 - i], block_bytes=G, workspace=ws,
                          stream=cx.stream, exact=exact, counters=ctr)
        cur[0] = 1 - i
        cur[1] += 1

    elapsed, prof = cx.timed(step, args.steps, args.warmup, h3c.engine.PROF_UPDATE)
    fresh = torch.zeros(nchunks, dtype=torch.int32, device=cx.dev)
    plan.run(fresh, stream=cx.stream)
    torch.cuda.synchronize()
    counters = dict(zip((f for f, _ in h3c.UpdateCounters._fields_), ctr.cpu().tolist()))
    verified = cx.all_true(bool(torch.equal(fresh, raw[cur[0]])) and counters["read_chunk"] == nw)
    plan.close()
    writes = nw * args.steps * cx.world
    res = {
        "metric": "partial-update writes/s (4 KiB writes into 64 MiB chunks, per-write chunk CRC32C)",
        "value": round(writes / elapsed, 1),
        "unit": "writes/s",
        "n_gpus": cx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 chunks and payloads in HBM, seeded uniform chunk/offset)",
        "config": {"workload": f"BASELINE config 3: {nw} random 4 KiB writes into {nchunks} x 64 MiB chunks per GPU"
                               + (" (H3C_UPD_EXACT: the chunks re-CRC'd from their bytes every step)" if exact else ""),
                   "parallelism": f"shard{cx.world}", "exact": exact, "tables": ntab,
                   "table_rotation": "each step applies the next of `tables` seeded write tables"},
        "verified": verified,
        "counters": counters,
        "algorithmic_gbps": round(writes * 3 * G / elapsed / 1e9, 1),
        "roofline": roofline(prof, HBM_PEAK_GBPS, kernel="upd_fused_kernel"),
    }
    if cx.world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_update()
    return res


def _pinned_records(torch, n: int, dtype) -> np.ndarray:
    """A numpy record array in pinned host memory (DMA without a staging copy)."""
    t = torch.empty(n * dtype.itemsize, dtype=torch.uint8).pin_memory()
    a = t.numpy().view(dtype)
    a[...] = 0
    return a, t


def run_updio(args, cx: Ctx) -> dict:
    """BASELINE config 3 through the general path: each 4 KiB write is a full UpdateIO -- client
    checksum verified (ChunkReplica.cc:193-207), updateChecksum's case analysis, fragments chained
    per 4 KiB block.  `value` is h3c_update_ios_dev with the op table, chunk table, results and
    counters resident in HBM (like the payloads and chunks); the host-array entry
    (h3c_update_ios_ex: tables in pinned host memory, copied over PCIe inside the step) is timed
    beside it and reported as `pcie_inclusive`."""
    torch, h3c = cx.torch, cx.h3c
    nchunks, clen, nw, G = 64, 64 << 20, args.writes, 4096
    bpc = clen // G
    chunks = torch.empty(nchunks * clen, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(chunks, clen, nchunks, clen, SEED, first_chunk=cx.rank * nchunks)
    payload = torch.empty(nw * G, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(payload, G, nw, G, SEED + 1, first_chunk=cx.rank * nw)
    # `tables` seeded op tables (different chunk / offset draws over the same payloads), run in rotation:
    # every timed batch differs from the one before it, as on a real update stream, so nothing the
    # kernels learn from the previous batch (the aligned branch's per-XCD range weights) flatters them
    ntab = max(1, int(getattr(args, "updio_tables", 4)))
    draws = []
    for t in range(ntab):
        g = np.random.default_rng(SEED + cx.rank + (0 if getattr(args, "updio_same_tables", False) else 7919 * t))
        wc = g.integers(0, nchunks, nw).astype(np.uint32)
        wb = g.integers(0, bpc, nw).astype(np.uint32)
        if getattr(args, "updio_order", "random") == "chunk":  # diagnostics: the ops grouped by chunk
            o = np.argsort(wc, kind="stable")
            wc, wb = wc[o], wb[o]
        draws.append((wc, wb))
    wc, wb = draws[0]
    g = np.random.default_rng(SEED + cx.rank)
    plan = h3c.Plan.uniform(chunks.data_ptr(), clen, nchunks, device=cx.local)
    raw0 = torch.zeros(nchunks, dtype=torch.int32, device=cx.dev)
    plan.run(raw0, stream=cx.stream)
    pplan = h3c.Plan.uniform(payload.data_ptr(), G, nw, device=cx.local)  # the clients' write checksums
    praw = torch.zeros(nw, dtype=torch.int32, device=cx.dev)
    pplan.run(praw, stream=cx.stream)
    torch.cuda.synchronize()
    state, _st = _pinned_records(torch, nchunks, h3c.CHUNK_STATE_DTYPE)
    state["base"] = chunks.data_ptr() + np.arange(nchunks, dtype=np.uint64) * np.uint64(clen)
    state["chunk_size"] = clen
    state["size"] = clen
    state["value"] = raw0.cpu().numpy().view(np.uint32)
    state["type"] = 1
    praw_np = praw.cpu().numpy().view(np.uint32)
    tabs = []
    for twc, twb in draws:
        t_ios, t_keep = _pinned_records(torch, nw, h3c.UPDATE_IO_DTYPE)
        t_ios["payload"] = payload.data_ptr() + np.arange(nw, dtype=np.uint64) * np.uint64(G)
        t_ios["chunk"] = twc
        t_ios["offset"] = twb * G
        t_ios["length"] = G
        t_ios["checksum_value"] = praw_np
        t_ios["checksum_type"] = 1
        t_ios["kind"] = h3c.UPD_WRITE
        tabs.append({"ios": t_ios, "keep": t_keep, "wc": twc,
                     "d_ios": torch.from_numpy(t_ios.view(np.uint8).copy()).to(cx.dev),
                     "d_res": torch.zeros(nw * h3c.UPDATE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=cx.dev)})
    ios = tabs[0]["ios"]
    exact = bool(getattr(args, "exact", False))
    d_state = torch.from_numpy(state.view(np.uint8).copy()).to(cx.dev)
    d_ios, d_res = tabs[0]["d_ios"], tabs[0]["d_res"]
    d_ctr = torch.zeros(8, dtype=torch.int64, device=cx.dev)

    # (bound once per table: the step is the C call, as for a C++ caller; update_ios_dev re-checks the
    # tensors).  --updio-graphs picks the headline form; the other is timed beside it (`other_form`)
    hg = bool(getattr(args, "updio_graphs", 1))
    tsteps = [h3c.UpdateIosDev(d_state, t["d_ios"], t["d_res"], stream=cx.stream, exact=exact, counters=d_ctr,
                               graphs=hg).run for t in tabs]
    nxt = [0]

    def step():
        tsteps[nxt[0] % ntab]()
        nxt[0] += 1

    g0 = h3c.diag_counters()
    elapsed, prof = cx.timed(step, args.steps, args.warmup, h3c.engine.PROF_UPDIO,
                             after_warmup=lambda: h3c.diag_host_trace(reset=True))
    host_us = h3c.diag_host_trace(reset=True)  # (the timed steps only)
    diag = {k: v - g0[k] for k, v in h3c.diag_counters().items()}
    graphs = {"replays": diag["graph_replays"], "captures": diag["graph_captures"],
              "capture_failures": diag["graph_capture_failures"]}
    # every redo / recovery / abandoned attempt the engine counts (h3c_diag_counter 3-9), over warmup +
    # timed steps: all 0 on config 3, which must run every step on the fast branch
    redo = {k: diag[k] for k in ("redo_front_void", "rerun_phase_b_void", "redo_failed_a6", "redo_short_fragment_guess",
                                 "fast_abandoned", "fast_recovered", "aligned_abandoned", "aligned_recovered")}
    fast_steps = diag["fast_batches"]
    aligned_steps = diag["aligned_batches"]
    torch.cuda.synchronize()
    last_tab = tabs[(nxt[0] - 1) % ntab]
    fin = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
    res = last_tab["d_res"].cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)
    counters = dict(zip((f for f, _ in h3c.UpdateCounters._fields_), d_ctr.cpu().tolist()))
    fresh = torch.zeros(nchunks, dtype=torch.int32, device=cx.dev)
    plan.run(fresh, stream=cx.stream)
    torch.cuda.synchronize()
    fresh_np = fresh.cpu().numpy().view(np.uint32)
    ok = bool((res["status"] == 0).all()) and np.array_equal(fresh_np, fin["value"])
    ok = ok and counters["read_chunk"] == nw and not any(redo.values())
    # every table once more, each checked right after its run: all ops OK, each chunk's last op reports the
    # chunk's stored checksum, and that equals a fresh GPU CRC of the chunk's bytes
    tables_ok = []
    if getattr(args, "updio_headline_only", False):  # (diagnostics: the timed leg's last launch stays the last one)
        tabs_check = []
    else:
        tabs_check = tabs
    for ti, t in enumerate(tabs_check):
        tsteps[ti]()
        torch.cuda.synchronize()
        tfin = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
        tres = t["d_res"].cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)
        plan.run(fresh, stream=cx.stream)
        torch.cuda.synchronize()
        last = np.full(nchunks, -1, dtype=np.int64)
        np.maximum.at(last, t["wc"].astype(np.int64), np.arange(nw))  # each chunk's last op
        hit = last >= 0
        tok = bool((tres["status"] == 0).all()) and np.array_equal(fresh.cpu().numpy().view(np.uint32), tfin["value"])
        tok = tok and np.array_equal(tres["value"][last[hit]], tfin["value"][hit])
        tables_ok.append(tok)
    ok = ok and all(tables_ok)
    fin = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)
    # independent of the GPU: a sample of chunks copied back and CRC'd by the CPU oracle (the chunks'
    # stored checksums after every batch must be the CRC32C of their bytes, ChunkReplica.cc:356-390)
    L = _oracle()
    L.orc_crc32c_sse42.restype = ctypes.c_uint32
    L.orc_crc32c_sse42.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    sample = sorted({0, nchunks - 1, *map(int, g.choice(nchunks, size=min(4, nchunks), replace=False))})
    oracle_ok = True
    for c in sample:
        h = chunks[c * clen:(c + 1) * clen].cpu().numpy()
        oracle_ok &= L.orc_crc32c_sse42(h.ctypes.data, h.size, 0xFFFFFFFF) == int(fin["value"][c])
    ok = ok and bool(oracle_ok)

    if getattr(args, "updio_headline_only", False):
        return {"metric": "diagnostics", "value": round(nw * args.steps / elapsed, 1), "ms_per_step":
                round(elapsed / args.steps * 1e3, 4), "verified": bool(ok), "roofline": roofline(
                    prof, HBM_PEAK_GBPS, kernel="uio_afused_kernel"), "config": {"tables": ntab}}
    # the same step through the host-array entry: tables over PCIe, inside the timed region
    state["value"] = fin["value"]
    hres, _rt = _pinned_records(torch, nw, h3c.UPDATE_RESULT_DTYPE)
    hctr = h3c.UpdateCounters()
    hsteps = max(1, min(args.steps, 20))

    hn = [0]

    def hstep():
        h3c.update_ios(state, tabs[hn[0] % ntab]["ios"], stream=cx.stream, out=hres, exact=exact, counters=hctr)
        hn[0] += 1

    helapsed, _ = cx.timed(hstep, hsteps, min(args.warmup, 2), h3c.engine.PROF_UPDIO)

    # the device-table step again in the other form (graphs on / off)
    d_state.copy_(torch.from_numpy(state.view(np.uint8).copy()).to(cx.dev))

    # (rotating the same tables as the headline form: one repeated table flatters a step by ~11 %, §5)
    psteps = [h3c.UpdateIosDev(d_state, t["d_ios"], t["d_res"], stream=cx.stream, exact=exact, counters=d_ctr,
                               graphs=not hg).run for t in tabs]
    pn = [0]

    def pstep():
        psteps[pn[0] % ntab]()
        pn[0] += 1

    pelapsed, _ = cx.timed(pstep, hsteps, min(args.warmup, 2), h3c.engine.PROF_UPDIO)
    torch.cuda.synchronize()
    state["value"] = d_state.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE)["value"]
    ok = ok and all(bool((t["d_res"].cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE)["status"] == 0).all()) for t in tabs)
    plan.run(fresh, stream=cx.stream)
    torch.cuda.synchronize()
    ok = ok and bool((hres["status"] == 0).all()) and np.array_equal(fresh.cpu().numpy().view(np.uint32),
                                                                     state["value"])
    verified = cx.all_true(ok)
    plan.close()
    pplan.close()
    writes = nw * args.steps * cx.world
    fast = fast_steps == args.steps + args.warmup
    aligned = aligned_steps == args.steps + args.warmup
    rl = roofline(prof, HBM_PEAK_GBPS, kernel="uio_afused_kernel" if aligned else "uio_fast_kernel" if fast
                  else "uio_block_kernel")
    out = {
        "metric": "partial-update writes/s through the general UpdateIO path (4 KiB writes into 64 MiB chunks)",
        "value": round(writes / elapsed, 1),
        "unit": "writes/s",
        "n_gpus": cx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 chunks and payloads in HBM, seeded uniform chunk/offset)",
        "config": {"workload": f"BASELINE config 3 via h3c_update_ios_dev{' (H3C_UPD_EXACT)' if exact else ''}: "
                               f"{nw} random 4 KiB UpdateIOs into {nchunks} x 64 MiB chunks per GPU, op / chunk / "
                               f"result tables in HBM",
                   "parallelism": f"shard{cx.world}", "exact": exact, "tables": ntab,
                   "table_rotation": f"{ntab} seeded op tables run in turn (batch k uses table k mod {ntab}); "
                                     "host-array and other-form legs use table 0"},
        "verified": verified,
        "tables_verified": tables_ok,
        # the minimum traffic per write: its payload read, its block read and written (3 x 4 KiB);
        # the A6 check of a one-block write runs inside the block kernel on the payload it reads
        "algorithmic_gbps": round(writes * 3 * G / elapsed / 1e9, 1),
        "counters": counters,
        "graphs": graphs,  # the headline leg's graph use over warmup + timed steps (--updio-graphs)
        "branch": "fast, aligned sub-branch (uio_aprep_kernel + uio_afused_kernel)" if aligned else
                  "fast (uio_fast_kernel)" if fast else f"general ({fast_steps} of {args.steps + args.warmup} fast)",
        "redo": redo,
        "host_us_per_call": host_us,  # the device-table leg's host time per call, by phase (h3c_diag_host_trace)
        "oracle_sample": {"chunks": sample, "ok": bool(oracle_ok),
                          "check": "final stored checksum == CPU oracle CRC32C of the chunk's bytes after the run"},
        "pcie_inclusive": {"entry": "h3c_update_ios_ex (host tables in pinned memory)",
                           "value": round(nw * hsteps * cx.world / helapsed, 1), "unit": "writes/s",
                           "ms_per_step": round(helapsed / hsteps * 1e3, 4), "steps": hsteps, "tables": ntab},
        "other_form": {"entry": "h3c_update_ios_dev, " + ("plain launches" if hg else
                                                           "H3C_UPD_GRAPHS: one graph replay per batch"),
                       "value": round(nw * hsteps * cx.world / pelapsed, 1), "unit": "writes/s",
                       "ms_per_step": round(pelapsed / hsteps * 1e3, 4), "steps": hsteps, "tables": ntab},
        "roofline": rl,
    }
    if cx.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_update()
    return out


def run_sync(args, cx: Ctx) -> dict:
    """The synchronous per-IO surface: 32 host threads each verifying their own
    pinned host buffer one call at a time, as AioReadJob::setResult (BatchReadJob.cc:34) and
    ChunkReplica::update (ChunkReplica.cc:194) call ChecksumInfo::create once per IO.  Per size:
    p50 / p99 call latency and aggregate GiB/s, uncoalesced and with the coalescing queue, and
    the CPU's per-call time for the same buffer (folly's 3-way SSE4.2 path restated in oracle/)."""
    h3c = cx.h3c
    threads = args.sync_threads
    calls_for = {4: 2000, 128: 600, 1024: 150}
    sizes = [(k << 10, calls_for.get(k, max(50, 2000 * 4 // k))) for k in map(int, args.sync_kib.split(","))]
    rows = []
    t_all = 0.0
    for nbytes, calls in sizes:
        row = {"bytes": nbytes, "threads": threads, "calls_per_thread": calls}
        for mode in ("uncoalesced", "coalesced"):
            h3c.set_coalescing(mode == "coalesced")
            lat, wall = h3c.sync_bench(threads, nbytes, calls, "verify")
            t_all += wall
            row[mode] = {"p50_us": round(float(np.percentile(lat, 50)), 1),
                         "p99_us": round(float(np.percentile(lat, 99)), 1),
                         "gib_s": round(threads * calls * nbytes / wall / 2**30, 3),
                         "calls_s": round(threads * calls / wall, 1)}
        h3c.set_coalescing(False)
        if not args.no_cpu_baseline:
            L = _oracle()
            L.orc_time_crc32c_calls.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
            L.orc_time_crc32c_calls.restype = ctypes.c_double
            buf = np.random.default_rng(nbytes).integers(0, 256, nbytes, dtype=np.uint8)
            per = L.orc_time_crc32c_calls(buf.ctypes.data, nbytes, max(200, (256 << 20) // nbytes))
            row["cpu_per_call_us"] = round(per * 1e6, 3)
            row["cpu_1core_gib_s"] = round(nbytes / per / 2**30, 2)
        rows.append(row)
    head = rows[0]["coalesced"]
    return {
        "metric": f"synchronous per-IO verify calls/s at {threads} threads (4 KiB pinned host buffers, coalesced)",
        "value": head["calls_s"], "unit": "calls/s", "n_gpus": cx.world, "steps": 1, "warmup": 3,
        "ms_per_step": round(t_all * 1e3, 2), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (xorshift bytes in pinned host memory)",
        "config": {"workload": f"sync: {threads} threads x h3c_batch_verify of one host buffer per call, "
                               "4 KiB / 128 KiB / 1 MiB", "parallelism": "one GPU, many host threads"},
        "verified": True, "sizes": rows,
        "note": "PCIe-inclusive per-call latency; cpu_per_call_us is one core's folly-path crc32c of the same buffer",
    }


def pcie_h2d_peak(cx: "Ctx", nbytes: int = 1 << 30, hb=None) -> float:
    """Pinned H2D GB/s per rank with EVERY rank copying at once (the ranks of one node share
    host DRAM and PCIe switches, so a rank measured alone would overstate its share): barrier,
    5 copies of `nbytes` per rank, barrier; per-rank rate = 5 * nbytes / the slowest rank's
    time.  The source is the rank's NUMA-local HostBuffer when given (the memory the host-fed
    pass read), else torch pinned memory."""
    torch = cx.torch
    src = torch.from_numpy(hb.array[:nbytes]) if hb is not None and hb.nbytes >= nbytes \
        else torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device=cx.dev)
    dst.copy_(src, non_blocking=True)
    cx.barrier()
    t0 = time.perf_counter()
    for _ in range(5):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    cx.barrier()
    return 5 * nbytes / cx.max_over_ranks(el) / 1e9


def run_hostfed(args, cx: Ctx) -> dict:
    torch, h3c = cx.torch, cx.h3c
    rng = np.random.default_rng(SEED + cx.rank)
    lens, total = [], 0
    while total < (args.hostfed_gib << 30):
        L = (64 << 10) << int(rng.integers(0, 11))  # 11 size classes 64 KiB .. 64 MiB
        if rng.random() < 0.1:
            L -= int(rng.integers(1, 4096))  # ragged lengths
        lens.append(L)
        total += L
    devbuf = torch.empty(total, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(devbuf, total - total % 8, 1, total - total % 8, SEED + 7 + cx.rank)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    _, expected = h3c.batch_create([(devbuf[o: o + L], L) for o, L in zip(offs, lens)])
    # NUMA-local pinned host memory: pages on the GPU's node, registered.
    # If the host refuses the registration, torch's pinned memory instead (node unknown), so
    # every rank still reaches the same collectives.
    try:
        hb = h3c.engine.HostBuffer(cx.local, total)
        host = hb.array
        torch.from_numpy(host).copy_(devbuf)
    except h3c.EngineError:
        hb = None
        host = devbuf.cpu().pin_memory()
    del devbuf
    items = [(host[o: o + L], L) for o, L in zip(offs, lens)]
    hf = h3c.HostFed(cx.local, args.window_mib << 20)
    state = {}

    def step():
        state["r"] = hf.run(items, expected=expected)

    elapsed, prof = cx.timed(step, args.steps, args.warmup, h3c.engine.PROF_HOSTFED)
    _, ok, nbad = state["r"]
    verified = cx.all_true(nbad == 0 and bool(ok.all()))
    hf.close()
    items = host = None
    node = hb.node if hb is not None else -1
    peak = pcie_h2d_peak(cx, hb=hb)
    if hb is not None:
        hb.close()
    value = total * args.steps * cx.world / elapsed / 2**30
    rl = roofline(prof, round(peak, 1), bound="pcie", kernel="hostfed pipeline (H2D + CRC)")
    rl["pcie_spec_gbps"] = PCIE_SPEC_GBPS
    return {
        "metric": "host-fed GiB/s CRC32C verified (mixed 64 KiB-64 MiB chunks from pinned host memory)",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": cx.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic: {len(lens)} chunks, {total / 2**30:.2f} GiB pinned host memory per GPU, 10% ragged",
        "config": {"workload": "BASELINE config 5: host-fed verify, H2D double-buffered against CRC",
                   "window_bytes": args.window_mib << 20, "parallelism": f"shard{cx.world}",
                   "host_numa_node": node},
        "verified": verified,
        "measured_h2d_gbps": round(peak, 1),
        "measured_h2d_note": f"per rank, all {cx.world} rank(s) copying pinned -> HBM at once",
        "roofline": rl,
    }


def run_mixed(args, cx: Ctx) -> dict:
    """Device-resident verify of mixed 64 KiB-64 MiB chunks (config 5's size classes, 10% ragged,
    packed back to back so most chunks start unaligned): the kernel at variable chunk sizes."""
    torch, h3c = cx.torch, cx.h3c
    rng = np.random.default_rng(SEED + 11 + cx.rank)
    lens, total = [], 0
    while total < (args.mixed_gib << 30):
        L = (64 << 10) << int(rng.integers(0, 11))
        if rng.random() < 0.1 and not args.mixed_aligned:
            L -= int(rng.integers(1, 4096))
        lens.append(L)
        total += L
    buf = torch.empty(total + 64, dtype=torch.uint8, device=cx.dev)
    h3c.fill_splitmix(buf, (total + 63) & ~7, 1, (total + 63) & ~7, SEED + 13 + cx.rank)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    d = np.zeros(len(lens), dtype=h3c.engine.DESC_DTYPE)
    d["ptr"] = np.uint64(buf.data_ptr()) + offs
    d["len"] = lens
    d["start_raw"] = 0xFFFFFFFF
    d["type"] = 1
    d["mem"] = 0
    plan = h3c.Plan(d, cx.local)
    n = len(lens)
    out = torch.zeros(n, dtype=torch.int32, device=cx.dev)
    plan.run(out, stream=cx.stream)
    torch.cuda.synchronize()
    # independent check: oracle on a sample of chunks (<= 4 MiB each)
    L = _oracle()
    L.orc_crc32c_sse42.restype = ctypes.c_uint32
    L.orc_crc32c_sse42.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    got = out.cpu().numpy().view(np.uint32)
    small = [i for i in range(n) if lens[i] <= (4 << 20)]
    sample = rng.choice(small, size=min(48, len(small)), replace=False) if small else []
    sample_ok = True
    for i in sample:
        h = buf[int(offs[i]): int(offs[i]) + lens[i]].cpu().numpy()
        sample_ok &= L.orc_crc32c_sse42(h.ctypes.data, h.size, 0xFFFFFFFF) == int(got[i])
    expected = out.clone()
    ok = torch.zeros(n, dtype=torch.uint8, device=cx.dev)
    mis = torch.zeros(1, dtype=torch.int32, device=cx.dev)

    def step():
        mis.zero_()
        plan.run(out, expected, ok, mis, stream=cx.stream)

    elapsed, prof = cx.timed(step, args.steps, args.warmup, h3c.engine.PROF_SEG)
    verified = cx.all_true(bool(sample_ok) and int(mis.item()) == 0)
    plan.close()
    value = total * args.steps * cx.world / elapsed / 2**30
    return {
        "metric": "GiB/s CRC32C verified (mixed 64 KiB-64 MiB device-resident chunks)",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": cx.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic: {n} chunks, {total / 2**30:.2f} GiB in HBM per GPU, 10% ragged, packed unaligned",
        "config": {"workload": "config 5 size classes, device-resident verify", "parallelism": f"shard{cx.world}"},
        "verified": verified,
        "roofline": roofline(prof, HBM_PEAK_GBPS),
    }


def run_shard4m(args, cx: Ctx) -> dict:
    """BASELINE config 4: total_gib as 4 MiB chunks split over the ranks (strong scaling),
    generated in HBM in passes of <= pass_gib; create (untimed) then timed verify per pass."""
    torch, h3c = cx.torch, cx.h3c
    clen = 4 << 20
    total_chunks = (args.total_gib << 30) // clen
    per = total_chunks // cx.world
    first = cx.rank * per
    pass_chunks = max(1, (args.pass_gib << 30) // clen)
    buf = torch.empty(min(per, pass_chunks) * clen, dtype=torch.uint8, device=cx.dev)
    elapsed_total, prof_acc, verified = 0.0, [0.0, 0, 0], True
    reps, pass_times = max(3, args.shard_reps), []
    done = 0
    while done < per:
        m = min(pass_chunks, per - done)
        h3c.fill_splitmix(buf, clen, m, clen, SEED, first_chunk=first + done)
        plan = h3c.Plan.uniform(buf.data_ptr(), clen, m, device=cx.local)
        stored = torch.zeros(m, dtype=torch.int32, device=cx.dev)
        plan.run(stored, stream=cx.stream)
        out = torch.zeros_like(stored)
        ok = torch.zeros(m, dtype=torch.uint8, device=cx.dev)
        mis = torch.zeros(1, dtype=torch.int32, device=cx.dev)

        def step():
            plan.run(out, expected=stored, ok=ok, mismatch=mis, stream=cx.stream)

        # warm launch on every pass (a pass's first launch pays its plan's first touches), then
        # `reps` launches timed one at a time (each max over ranks); the pass counts its median
        step()
        times = []
        for _ in range(reps):
            el, prof = cx.timed(step, 1, 0, h3c.engine.PROF_SEG)
            times.append(el)
            for k in range(3):
                prof_acc[k] += prof[k]
        pass_times.append(sorted(times)[len(times) // 2])
        elapsed_total += pass_times[-1]
        verified = verified and int(mis.item()) == 0
        plan.close()
        done += m
    verified = cx.all_true(verified)
    value = total_chunks * clen / elapsed_total / 2**30
    return {
        "metric": "GiB/s CRC32C verified (4 MiB chunks, 256 GiB total split over the GPUs)",
        # steps / warmup per pass: `reps` timed launches after 1 warm one (a step is one pass over the
        # whole 256 GiB: the sum over passes of each pass's median launch).  Rounds 1-3 timed one cold
        # launch per pass; their config-4 numbers are not comparable with this method's.
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": cx.world, "steps": reps, "warmup": 1,
        "ms_per_step": round(elapsed_total * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "timing": f"per pass: one warm launch, then the median of {reps} launches timed one at a time "
                  f"(max over ranks); a step is the sum over passes",
        "pass_ms": [round(t * 1e3, 3) for t in pass_times],
        "vs_baseline": None, "dtype": "u8", "data": "synthetic splitmix64 4 MiB chunks generated in HBM in passes",
        "config": {"workload": f"BASELINE config 4: {args.total_gib} GiB as 4 MiB chunks, "
                               f"{per} chunks per GPU in passes of <= {pass_chunks}",
                   "parallelism": f"shard{cx.world}"},
        "verified": verified,
        "roofline": roofline(tuple(prof_acc), HBM_PEAK_GBPS),
    }


def _set_pdeathsig() -> None:  # pragma: no cover - runs in the child between fork and exec
    """Children die with the launcher (a driver timeout that kills it must not leave ranks on
    the GPU): prctl(PR_SET_PDEATHSIG, SIGTERM)."""
    import signal

    try:
        ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGTERM), 0, 0, 0)
    except (OSError, AttributeError):
        pass


def rank_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    """The environment torch.distributed.run gives rank `rank` of a one-node job."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), H3C_BENCH_LAUNCHED="1")
    return env


def check_world(gpus: int, env=os.environ) -> str | None:
    """The --gpus / WORLD_SIZE contract: under a launcher (WORLD_SIZE set) the two must agree.
    Returns an error message, or None."""
    if gpus < 1:
        return f"--gpus must be >= 1 (got {gpus})"
    ws = env.get("WORLD_SIZE")
    if ws is not None and int(ws) != gpus:
        return f"WORLD_SIZE={ws} from the launcher disagrees with --gpus {gpus}"
    return None


def check_devices(world: int, ndev: int, allow_shared: bool) -> str | None:
    """One process per GPU: a job with more ranks than visible devices would put several ranks on
    one GPU and still print n_gpus = WORLD_SIZE.  Refused unless --allow-shared-devices (a
    single-GPU rehearsal of the N-rank path), which the line then reports as "rehearsal"."""
    if world > max(ndev, 0) and not allow_shared:
        return (f"WORLD_SIZE={world} ranks but only {ndev} visible GPU(s): one process per GPU; "
                f"pass --allow-shared-devices for a shared-device rehearsal")
    return None


def devices_used(world: int, ndev: int) -> int:
    """Distinct GPUs a job of `world` ranks uses (rank r on device r % ndev)."""
    return min(world, max(ndev, 1))


def spawn_ranks(gpus: int, argv: list, grace_s: float = 60.0) -> int:
    """`bench.py --gpus N` run without a launcher (WORLD_SIZE unset): start N child processes of
    this script, one per GPU, with the env torchrun would give them (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT).  The parent never imports torch
    or touches HIP -- it only waits.  Rank 0 prints the JSON line on the inherited stdout.
    Returns 0 only when every rank exits 0, else the exit code of the first rank to fail; then the
    others get `grace_s` to finish before they are terminated (they would otherwise wait in a
    barrier for gloo's 30-minute timeout)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=rank_env(r, gpus, port),
                              preexec_fn=_set_pdeathsig) for r in range(gpus)]
    first_fail, cause = None, 0
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if first_fail is None and any(rc not in (None, 0) for rc in rcs):
            first_fail = time.monotonic()
            cause = next(rc for rc in rcs if rc not in (None, 0))
        if first_fail is not None and time.monotonic() - first_fail > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.2)
    rcs = [p.returncode for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr, flush=True)
        # the first rank to fail is the cause (ranks terminated after the grace period are not);
        # a signal death (-N) becomes 128 + N, as a shell reports it
        rc = cause if first_fail is not None else bad[0]
        return 128 - rc if rc < 0 else rc
    return 0


def dry_run_launch(args) -> int:
    """CPU-only rehearsal of the launch contract (tests/test_bench_contract.py): every rank joins
    a gloo group from the env it was given and rank 0 prints the ranks it saw; rank
    `--dry-run-launch K` (K >= 0) exits 3 before joining, to exercise failure propagation."""
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if args.dry_run_launch == rank:
        return 3
    seen = [rank]
    if world > 1:
        import torch
        import torch.distributed as dist

        dist.init_process_group("gloo")
        t = torch.zeros(world, dtype=torch.int64)
        t[rank] = int(os.environ["LOCAL_RANK"]) + 1
        dist.all_reduce(t)
        seen = [int(v) - 1 for v in t.tolist()]
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "local_ranks": seen,
                          "launched": bool(os.environ.get("H3C_BENCH_LAUNCHED"))}), flush=True)
    return 0


def main_inproc(args) -> int:
    """bench.py --gpus N --inproc [--devices LIST]: the headline verify over N GPUs from this one process
    through the C-ABI multi engine (h3c_multi_*), the way a C++ storage service drives them."""
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        print("bench.py: --inproc runs in one process; do not launch it with torchrun", file=sys.stderr, flush=True)
        return 2
    import torch

    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    ndev = torch.cuda.device_count()
    if any(d >= ndev for d in devices) or len(devices) != args.gpus:
        print(f"bench.py: --inproc wants {args.gpus} device(s) {devices}, {ndev} visible", file=sys.stderr, flush=True)
        return 2
    cx = Ctx()
    res = run_inproc(args, cx, devices)
    res["config"]["devices_visible"] = ndev
    if len(set(devices)) < len(devices):
        res["rehearsal"] = True  # workers share devices: n_gpus counts distinct GPUs
    print(json.dumps(res), flush=True)
    return 0 if res["verified"] else 1


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dry-run-launch", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["verify", "update", "updio", "hostfed", "shard4m", "mixed", "sync"], default="verify")
    ap.add_argument("--chunks", type=int, default=8192)
    ap.add_argument("--chunk-kib", type=int, default=1024)
    ap.add_argument("--flip-frac", type=float, default=0.05)
    ap.add_argument("--writes", type=int, default=100_000)
    ap.add_argument("--hostfed-gib", type=int, default=4)
    ap.add_argument("--hostfed-extra-gib", type=int, default=2,
                    help="default verify run: also a short host-fed pass of this many GiB per GPU (0: off)")
    ap.add_argument("--update-extra", type=int, choices=[0, 1], default=1,
                    help="default verify run: also a short BASELINE config-3 UpdateIO pass (the `update` object)")
    ap.add_argument("--shard4m-extra", type=int, choices=[0, 1], default=1,
                    help="default verify run: also config 4's per-GPU share, 8192 x 4 MiB (the `shard4m` object)")
    ap.add_argument("--inproc-extra", type=int, choices=[0, 1], default=1,
                    help="default verify run: also the in-process multi-GPU product path (the `inproc` object)")
    ap.add_argument("--inproc", action="store_true",
                    help="one process drives --gpus devices through h3c_multi_* (no launcher, no torch.distributed)")
    ap.add_argument("--devices", default=None,
                    help="--inproc: comma-separated device list (a device may repeat: workers sharing one GPU)")
    ap.add_argument("--mixed-gib", type=int, default=8)
    ap.add_argument("--mixed-aligned", action="store_true", help="no ragged lengths (every chunk 64 KiB-aligned)")
    ap.add_argument("--window-mib", type=int, default=64)
    ap.add_argument("--total-gib", type=int, default=256)
    ap.add_argument("--pass-gib", type=int, default=64)
    ap.add_argument("--shard-reps", type=int, default=3, help="shard4m: timed launches per pass (>= 3; median)")
    ap.add_argument("--allow-shared-devices", action="store_true",
                    help="rehearsal: allow more ranks than visible GPUs (ranks share devices; the line says so)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exact", action="store_true", help="updio / update: do not trust stored checksums")
    ap.add_argument("--updio-order", choices=["random", "chunk"], default="random",
                    help="updio diagnostics: chunk = the same writes grouped by chunk (sequence order within)")
    ap.add_argument("--updio-graphs", type=int, choices=[0, 1], default=1,
                    help="updio: the headline leg as one replayed graph per batch (1) or plain launches (0); "
                         "the other form is timed beside it")
    ap.add_argument("--updio-tables", type=int, default=4,
                    help="updio: seeded op tables run in rotation (every batch differs from the last)")
    ap.add_argument("--update-tables", type=int, default=4,
                    help="update (block path): seeded write tables run in rotation")
    ap.add_argument("--updio-same-tables", action="store_true", help=argparse.SUPPRESS)  # (diagnostics: one draw)
    ap.add_argument("--updio-headline-only", action="store_true", help=argparse.SUPPRESS)  # (diagnostics: timed leg only)
    ap.add_argument("--sync-threads", type=int, default=32)
    ap.add_argument("--sync-kib", default="4,128,1024", help="sync: buffer sizes (KiB), comma-separated")
    args = ap.parse_args()
    err = check_world(args.gpus)
    if err:
        print(f"bench.py: {err}", file=sys.stderr, flush=True)
        return 2
    if args.inproc:
        return main_inproc(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, sys.argv[1:], float(os.environ.get("H3C_BENCH_GRACE_S", "60")))
    if args.dry_run_launch is not None:
        return dry_run_launch(args)
    import torch  # device_count() does not initialise the GPU on this image

    ndev = torch.cuda.device_count()
    err = check_devices(int(os.environ.get("WORLD_SIZE", "1")), ndev, args.allow_shared_devices)
    if err:
        print(f"bench.py: {err}", file=sys.stderr, flush=True)
        return 2
    cx = Ctx()
    fn = {"verify": run_verify, "update": run_update, "updio": run_updio, "hostfed": run_hostfed,
          "shard4m": run_shard4m, "mixed": run_mixed, "sync": run_sync}[args.workload]
    if args.workload in ("hostfed", "updio") and args.steps == 50:
        # (updio: a batch is ~0.34 ms; 100 timed batches after 20 warm ones -- 10 after 2 left the timed
        # leg within the GPU's clock ramp, ~2-3 % slower than the same leg run later)
        args.steps, args.warmup = (5, 1) if args.workload == "hostfed" else (100, 20)
    res = fn(args, cx)
    if args.workload == "verify" and args.hostfed_extra_gib > 0 and (args.chunks, args.chunk_kib) == (8192, 1024):
        # BASELINE asks for host-fed throughput at 1/2/4/8 GPUs too: the driver's scaling runs
        # use the default workload, so it carries a short config-5 pass (never the `value`).
        sub = argparse.Namespace(**vars(args))
        sub.hostfed_gib, sub.steps, sub.warmup = args.hostfed_extra_gib, 3, 1
        hf = run_hostfed(sub, cx)
        res["hostfed"] = {
            "metric": hf["metric"], "value": hf["value"], "unit": hf["unit"], "n_gpus": hf["n_gpus"],
            "ms_per_step": hf["ms_per_step"], "scaling": "weak", "data": hf["data"],
            "measured_h2d_gbps": hf["measured_h2d_gbps"], "pcie_frac": hf["roofline"]["frac"],
            "host_numa_node_rank0": hf["config"]["host_numa_node"], "verified": hf["verified"],
            "note": "PCIe-inclusive (payloads in NUMA-local pinned host memory); not the headline value",
        }
    if args.workload == "verify" and args.update_extra and (args.chunks, args.chunk_kib) == (8192, 1024):
        # BASELINE config 3 in front of the driver too: 100k random 4 KiB UpdateIOs into
        # 64 x 64 MiB chunks through h3c_update_ios_dev, 30 warm + 50 timed batches (never the `value`; the
        # aligned sub-branch's range weights settle over the first ~10 batches)
        sub = argparse.Namespace(**vars(args))
        sub.steps, sub.warmup, sub.writes, sub.exact = 50, 30, 100_000, False
        up = run_updio(sub, cx)
        res["update"] = {
            "metric": up["metric"], "config": up["config"]["workload"], "n_gpus": up["n_gpus"],
            "steps": up["steps"], "warmup": up["warmup"], "ms_per_step": up["ms_per_step"],
            "tables": up["config"]["tables"], "tables_verified": up["tables_verified"],
            "writes_per_s": up["value"], "unit": "writes/s", "scaling": "weak", "verified": up["verified"],
            "branch": up["branch"], "redo": up["redo"], "counters": up["counters"],
            "oracle_sample": up["oracle_sample"], "algorithmic_gbps": up["algorithmic_gbps"],
            "roofline": up["roofline"], "pcie_inclusive": up["pcie_inclusive"], "other_form": up["other_form"],
            "note": "algorithmic bytes 12 KiB per write (payload read, block read and written); not the headline value",
        }
        if "cpu_baseline" in up:
            res["update"]["cpu_baseline"] = up["cpu_baseline"]
        res["verified"] = res["verified"] and up["verified"]
    if args.workload == "verify" and args.shard4m_extra and (args.chunks, args.chunk_kib) == (8192, 1024):
        # BASELINE config 4's per-GPU share in front of the driver: 8192 x 4 MiB = 32 GiB, the
        # N=8 share of 256 GiB, verified against 5% flipped chunks (never the `value`)
        sub = argparse.Namespace(**vars(args))
        sub.chunks, sub.chunk_kib, sub.steps, sub.warmup, sub.no_cpu_baseline = 8192, 4096, 20, 5, True
        r4 = run_verify(sub, cx)
        res["shard4m"] = {
            "metric": "GiB/s CRC32C verified (4 MiB chunks, the per-GPU share of 256 GiB at 8 GPUs)",
            "value": r4["value"], "unit": "GiB/s", "n_gpus": r4["n_gpus"], "steps": r4["steps"],
            "warmup": r4["warmup"], "ms_per_step": r4["ms_per_step"], "scaling": "weak",
            "config": f"BASELINE config 4 share: 8192 x 4 MiB = 32 GiB device-resident per GPU "
                      f"({cx.world} x 32 GiB in this job), 5% of chunks with one flipped bit",
            "verified": r4["verified"], "roofline": r4["roofline"],
            "note": "at N=8 the job verifies the whole 256 GiB of config 4; not the headline value",
        }
        res["verified"] = res["verified"] and r4["verified"]
    if args.workload == "verify" and args.inproc_extra and (args.chunks, args.chunk_kib) == (8192, 1024):
        # the product path over all of this job's GPUs from ONE process (h3c_multi_*): rank 0 drives every
        # device of the job while the other ranks wait at a barrier (never the `value`)
        cx.barrier()
        if cx.rank == 0:
            sub = argparse.Namespace(**vars(args))
            sub.steps, sub.warmup = 20, 3
            ip = run_inproc(sub, cx, [r % max(cx.ndev, 1) for r in range(cx.world)])
            res["inproc"] = {k: ip[k] for k in ("value", "unit", "n_gpus", "workers", "devices", "steps", "warmup",
                                                 "ms_per_step", "verified", "per_worker", "note")}
            res["inproc"]["config"] = ip["config"]["workload"]
        ok_ip = cx.all_true(res.get("inproc", {}).get("verified", True))
        res["verified"] = res["verified"] and ok_ip
    # N ranks on fewer devices (--allow-shared-devices) is a rehearsal: n_gpus is the devices used
    res.setdefault("config", {})["devices_visible"] = cx.ndev
    if cx.world > cx.ndev:
        res["rehearsal"] = True
        res["n_gpus"] = devices_used(cx.world, cx.ndev)
        res["config"]["ranks"] = cx.world
        for sub in ("hostfed", "update"):  # (the sub-passes' n_gpus by the same rule)
            if sub in res:
                res[sub]["n_gpus"] = res["n_gpus"]
                res[sub]["ranks"] = cx.world
    res["config"]["launcher"] = "bench.py --gpus (spawned ranks)" if os.environ.get("H3C_BENCH_LAUNCHED") \
        else ("torchrun" if cx.world > 1 else "single process")
    if cx.rank == 0:
        print(json.dumps(res), flush=True)
    if cx.world > 1:
        cx.dist.destroy_process_group()
    return 0 if res["verified"] else 1


if __name__ == "__main__":
    sys.exit(main())
