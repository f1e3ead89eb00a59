import importlib, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
h3c = importlib.import_module("3fs_amd")
dev = torch.device("cuda:0")
total = 4 << 30
pinned = torch.empty(total, dtype=torch.uint8).pin_memory()
dst = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
for off in range(0, total, 64 << 20):
    dst.copy_(pinned[off: off + (64 << 20)], non_blocking=True)
torch.cuda.synchronize()
print("torch 64MiB slice copies: %.1f GB/s" % (total / (time.perf_counter() - t0) / 1e9), flush=True)
for win in (64, 256):
    hf = h3c.HostFed(0, win << 20)
    for label, items in (("one 4GiB chunk", [(pinned, total)]),
                         ("64 x 64MiB chunks", [(pinned[o: o + (64 << 20)], 64 << 20) for o in range(0, total, 64 << 20)]),
                         ("4096 x 1MiB chunks", [(pinned[o: o + (1 << 20)], 1 << 20) for o in range(0, total, 1 << 20)])):
        hf.run(items)
        t0 = time.perf_counter()
        for _ in range(3):
            hf.run(items)
        el = (time.perf_counter() - t0) / 3
        print("hostfed win %d MiB %-20s %.1f GB/s (%.1f ms)" % (win, label, total / el / 1e9, el * 1e3), flush=True)
    hf.close()
