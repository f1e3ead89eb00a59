"""Concurrent stress of the engine against the oracle (GPU box; not part of the test suite).

Several host threads, each on its own HIP stream, loop for --seconds over seeded random
work and compare every result with the CPU oracle:
  * create / verify batches mixing polynomials, starts, memory kinds, lengths, alignments
    (tests/test_gpu_fuzz.py's generator), through the synchronous and the plan paths;
  * general UpdateIO batches (tests/test_gpu_updio.py's scenario generator), some past the
    parallel host-pass threshold;
  * (round 5) aligned one-block UpdateIO batches (the aligned sub-branch, with failed checks at times) and
    block-aligned updates through h3c_update_blocks on the thread's stream (its per-stream scratch).
Prints one line per thread and a summary; exits non-zero on the first mismatch.
usage: python scripts/stress.py [--seconds 120] [--threads 4]
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_lib as orc  # noqa: E402
import test_gpu_fuzz as fz  # noqa: E402
import test_gpu_updio as up  # noqa: E402
import test_gpu_update_scratch as us  # noqa: E402
import test_gpu_updio_aligned as al  # noqa: E402


def worker(tid, h3c, torch, dev, deadline, stats, errors):
    stream = torch.cuda.Stream(device=dev)
    rng = np.random.default_rng(7000 + tid)
    pool = 16 << 20
    host = rng.integers(0, 256, pool, dtype=np.uint8)
    dbuf = torch.from_numpy(host).to(dev)
    pinned = torch.from_numpy(host).pin_memory()
    it = 0
    store = us.Store(torch, dev, rng, 6, 256 << 10)
    with torch.cuda.stream(stream):
        while time.time() < deadline and not errors:
            it += 1
            kind = it % 5
            try:
                if kind in (0, 1):
                    small = [0, 4096, 8192][int(rng.integers(0, 3))]
                    batch = fz.random_batch(rng, int(rng.integers(1, 400)), pool, small)
                    items, want = [], []
                    for off, ln, t, start, mem in batch:
                        if mem == "null":
                            items.append((None, ln, start, t))
                            want.append(orc.create(t, None, ln, start))
                            continue
                        src = {"dev": dbuf, "pinned": pinned, "pageable": host}[mem]
                        items.append((src[off: off + ln], ln, start, t))
                        want.append(orc.create(t, host[off: off + ln], ln, start))
                    types, vals = h3c.batch_create(items, stream=stream)
                    got = [(int(a), int(b)) for a, b in zip(types, vals)]
                    if got != want:
                        errors.append(f"thread {tid} iter {it}: create mismatch")
                    stats[tid]["create"] += len(items)
                elif kind == 2:
                    nops = int(rng.choice([200, 2000, 20000]))
                    sc = up.random_scenario(h3c, torch, dev, rng, nchunks=int(rng.integers(4, 32)),
                                            chunk_size=64 << 10, nops=nops)
                    sc.check(*sc.run())
                    stats[tid]["updio"] += nops
                elif kind == 3:
                    nops = int(rng.choice([500, 5000, 20000]))
                    sc = al.aligned_scenario(h3c, torch, dev, rng, nchunks=int(rng.integers(4, 64)),
                                             chunk_size=256 << 10, nops=nops, bad=float(rng.choice([0.0, 0.0, 0.02])))
                    sc.check(*sc.run(dev_api=True))
                    stats[tid]["updio"] += nops
                else:
                    nw = int(rng.integers(1, 6000))
                    store.batch(h3c, rng, nw, n_invalid=int(rng.integers(0, 3)), stream=stream)
                    stats[tid]["blocks"] += nw
            except AssertionError as e:
                errors.append(f"thread {tid} iter {it}: {str(e)[:200]}")
            except Exception as e:  # noqa: BLE001
                errors.append(f"thread {tid} iter {it}: {type(e).__name__}: {str(e)[:200]}")
    stats[tid]["iters"] = it


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--threads", type=int, default=4)
    args = ap.parse_args()
    import importlib

    import torch

    h3c = importlib.import_module("3fs_amd")
    dev = torch.device("cuda:0")
    deadline = time.time() + args.seconds
    stats = [{"create": 0, "updio": 0, "blocks": 0, "iters": 0} for _ in range(args.threads)]
    errors = []
    ths = [threading.Thread(target=worker, args=(t, h3c, torch, dev, deadline, stats, errors))
           for t in range(args.threads)]
    t0 = time.time()
    for t in ths:
        t.start()
    while any(t.is_alive() for t in ths):  # progress line every 30 s (keeps the box's watchdog fed)
        time.sleep(min(30.0, max(0.1, deadline - time.time() + 1)))
        print(f"[stress] {time.time() - t0:.0f} s, errors {len(errors)}", flush=True)
    for t in ths:
        t.join()
    for tid, s in enumerate(stats):
        print(f"thread {tid}: {s['iters']} iterations, {s['create']} checksums, {s['updio']} UpdateIOs, "
              f"{s['blocks']} block writes", flush=True)
    print(f"stress: {time.time() - t0:.0f} s, {len(errors)} errors", flush=True)
    for e in errors[:10]:
        print("  " + e)
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main())
