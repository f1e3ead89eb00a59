"""Diagnostic: which sizes / segment sizes / code paths disagree with the oracle."""
import importlib, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle_lib as orc
h3c = importlib.import_module("3fs_amd")
rng = np.random.default_rng(1)
sizes = [4096, 5120, 6144, 7168, 8192, 9216, 12288, 16384, 16385, 32768, 65536, 65543, 1 << 20]
host = [rng.integers(0, 256, n, dtype=np.uint8) for n in sizes]
dev = [torch.from_numpy(h).cuda() for h in host]
_, v = h3c.batch_create(dev)
print("seg", os.environ.get("H3C_SEG_BYTES"), "dbg", os.environ.get("H3C_DEBUG_FLAGS"),
      " ".join(f"{n}:{'ok' if int(g) == orc.crc32c(h) else 'BAD'}" for n, h, g in zip(sizes, host, v)), flush=True)
