"""Where does an update_ios step spend its time? (phase clock inside + wall clock outside)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib

import torch

h3c = importlib.import_module("3fs_amd")
dev = torch.device("cuda:0")
nchunks, clen, nw, G = 64, 64 << 20, 100_000, 4096
chunks = torch.empty(nchunks * clen, dtype=torch.uint8, device=dev)
h3c.fill_splitmix(chunks, clen, nchunks, clen, 1)
payload = torch.empty(nw * G, dtype=torch.uint8, device=dev)
h3c.fill_splitmix(payload, G, nw, G, 2)
g = np.random.default_rng(3)
wc = g.integers(0, nchunks, nw).astype(np.uint32)
wb = g.integers(0, clen // G, nw).astype(np.uint32)
raw0 = torch.zeros(nchunks, dtype=torch.int32, device=dev)
h3c.Plan.uniform(chunks.data_ptr(), clen, nchunks).run(raw0)
praw = torch.zeros(nw, dtype=torch.int32, device=dev)
h3c.Plan.uniform(payload.data_ptr(), G, nw).run(praw)
torch.cuda.synchronize()
state = np.zeros(nchunks, dtype=h3c.CHUNK_STATE_DTYPE)
state["base"] = chunks.data_ptr() + np.arange(nchunks, dtype=np.uint64) * np.uint64(clen)
state["chunk_size"] = clen
state["size"] = clen
state["value"] = raw0.cpu().numpy().view(np.uint32)
state["type"] = 1
ios = np.zeros(nw, dtype=h3c.UPDATE_IO_DTYPE)
ios["payload"] = payload.data_ptr() + np.arange(nw, dtype=np.uint64) * np.uint64(G)
ios["chunk"] = wc
ios["offset"] = wb * G
ios["length"] = G
ios["checksum_value"] = praw.cpu().numpy().view(np.uint32)
ios["checksum_type"] = 1
ios["kind"] = 1
for k in range(6):
    t0 = time.perf_counter()
    r = h3c.update_ios(state, ios)
    t1 = time.perf_counter()
    print(f"step {k}: {1e3 * (t1 - t0):.3f} ms wall", file=sys.stderr, flush=True)
