#!/usr/bin/env python3
"""Headline bench: GiB/s of CRC32C-verified 1 MiB chunks (BASELINE.json config 2).

A step = one batch verify of 8192 x 1 MiB device-resident chunks per GPU
(recompute every chunk's CRC32C, compare against the stored value, count
mismatches) -- the ChunkReplica::update / AioReadJob::setResult recalculate
path (src/storage/store/ChunkReplica.cc:193-207, src/storage/aio/BatchReadJob.cc:43-54)
batched.  Inputs are resident in HBM before the timed region starts.

Multi-GPU: one process per GPU (torchrun), each verifies its own 8192-chunk
shard; there is no data-path collective (weak scaling).  torch.distributed is
used only for the barrier and the max-over-ranks time.

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


def cpu_baseline(gpu_raw_first: np.ndarray, chunk_len: int, seconds: float = 8.0) -> dict:
    """Reference CPU path restated (oracle/, folly-faithful 3-stream SSE4.2 crc32q) on this host.

    Sample: 1024 x 1 MiB splitmix chunks (BASELINE config 1), ChecksumInfo::create
    semantics, 1 host thread, repeated for ~`seconds`.  The same pass also checks
    the GPU's values for those chunk indices."""
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        import subprocess

        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    L = ctypes.CDLL(so)
    L.orc_fill_splitmix.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    L.orc_batch_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    n = 1024
    host = np.empty(n * chunk_len, dtype=np.uint8)
    for c in range(n):
        L.orc_fill_splitmix(host[c * chunk_len:].ctypes.data, chunk_len, SEED, c)
    out = np.zeros(n, dtype=np.uint32)
    L.orc_batch_crc32c(host.ctypes.data, chunk_len, n, 0xFFFFFFFF, 1, 0, out.ctypes.data)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        L.orc_batch_crc32c(host.ctypes.data, chunk_len, n, 0xFFFFFFFF, 1, 0, out.ctypes.data)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gibps = reps * n * chunk_len / el / 2**30
    match = bool(np.array_equal(out, gpu_raw_first[:n]))
    return {
        "value": round(gibps, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{reps} x (1024 x {chunk_len >> 20} MiB splitmix chunks), folly-faithful 3-way SSE4.2 crc32q, "
                  f"1 thread, {el:.1f} s",
        "gpu_values_match": match,
        "cpu_model": _cpu_model(),
        "nproc": os.cpu_count(),
    }


def pmc_traffic(bytes_per_launch: int):
    """HBM bytes per seg_crc_kernel launch from the committed rocprofv3 PMC summary
    (profiles/*_pmc_summary.json, made by scripts/profile_r1.sh + summarize_prof.py,
    FETCH_SIZE/WRITE_SIZE in separate passes, gfx950 FETCH_SIZE x2 correction).
    Only used when that profile was taken on this same per-launch workload."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        t = d.get("pmc", {}).get("traffic_bytes_per_launch")
        if t and abs(d.get("algorithmic_bytes_per_launch", 0) - bytes_per_launch) < 1:
            best = (t, os.path.basename(f))
    return best


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=8192)
    ap.add_argument("--chunk-kib", type=int, default=1024)
    ap.add_argument("--flip-frac", type=float, default=0.05)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    h3c = importlib.import_module("3fs_amd")

    n, clen = args.chunks, args.chunk_kib << 10
    buf = torch.empty(n * clen, dtype=torch.uint8, device=dev)
    # Rank r holds chunk indices [r*n, (r+1)*n): distinct data per GPU.
    h3c.fill_splitmix(buf, clen, n, clen, SEED, first_chunk=rank * n)
    torch.cuda.synchronize()
    plan = h3c.Plan.uniform(buf.data_ptr(), clen, n, device=local)
    stream = torch.cuda.current_stream()

    # Stored checksums = a create pass; then corrupt flip_frac of the chunks.
    stored = torch.zeros(n, dtype=torch.int32, device=dev)
    plan.run(stored, stream=stream)
    torch.cuda.synchronize()
    stored_host = stored.cpu().numpy().view(np.uint32).copy()
    g = torch.Generator().manual_seed(SEED + rank)
    nflip = int(n * args.flip_frac)
    flips = torch.randperm(n, generator=g)[:nflip].sort().values
    pos = flips * clen + torch.randint(0, clen, (nflip,), generator=g)
    bits = (1 << torch.randint(0, 8, (nflip,), generator=g)).to(torch.uint8)
    pos_d = pos.to(dev)
    buf[pos_d] ^= bits.to(dev)

    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    mis = torch.zeros(1, dtype=torch.int32, device=dev)

    def step():
        mis.zero_()
        plan.run(out, expected=stored, ok=ok, mismatch=mis, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    h3c.profile_read(reset=True)
    h3c.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    h3c.profile_enable(False)
    kern_ms, launches, kbytes = h3c.profile_read(reset=True)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Correctness of the timed work: exactly the flipped chunks fail.
    bad = np.nonzero(ok.cpu().numpy() == 0)[0]
    verified = int(mis.item()) == nflip and np.array_equal(bad, flips.numpy())
    if world > 1:
        vt = torch.tensor([1 if verified else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(vt, op=dist.ReduceOp.MIN)
        verified = bool(vt.item())

    total_bytes = n * clen * args.steps * world
    value = total_bytes / elapsed / 2**30
    bytes_per_launch = kbytes / max(launches, 1)
    avg_kernel_s = kern_ms / 1e3 / max(launches, 1)
    achieved = bytes_per_launch / avg_kernel_s / 1e9 if launches else 0.0

    if rank == 0:
        res = {
            "metric": "GiB/s CRC32C verified (1 MiB chunks) at 1/2/4/8 GPUs; % of HBM peak",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 chunks generated in HBM; 5% of chunks carry one flipped bit)",
            "config": {
                "workload": f"batched CRC32C verify of {n} x {clen >> 10} KiB device-resident chunks per GPU "
                            f"(BASELINE config 2)",
                "chunks_per_gpu": n,
                "chunk_bytes": clen,
                "parallelism": f"shard{world}",
            },
            "verified": verified,
            "pct_hbm_peak": round(100.0 * (n * clen) / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBPS, 2),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": None,
                "kernel": "seg_crc_kernel",
                "kernel_avg_us": round(avg_kernel_s * 1e6, 2),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
            },
        }
        tr = pmc_traffic(int(bytes_per_launch))
        if tr:
            res["roofline"]["traffic"] = int(tr[0])
            res["roofline"]["traffic_source"] = f"profiles/{tr[1]}"
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(stored_host, clen, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()
    return 0 if verified else 1


if __name__ == "__main__":
    sys.exit(main())
