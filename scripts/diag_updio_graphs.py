"""Diagnostic: the same device-resident UpdateIO batch run repeatedly on restored state; prints,
per run, how many op results / chunk states differ from run 0 (run 1 captures the pipeline
graphs, later runs replay them)."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_gpu_updio as T  # noqa: E402

h3c = importlib.import_module("3fs_amd")
dev = torch.device("cuda:0")
if len(sys.argv) > 1:
    h3c.set_test_hook(h3c.HOOK_UPD_GRAPHS, int(sys.argv[1]))
rng = np.random.default_rng(91)
sc = T.random_scenario(h3c, torch, dev, rng, nchunks=10, chunk_size=64 << 10, nops=2500)
chunks, ios = sc.device_ios()
d_chunks0 = torch.from_numpy(chunks.view(np.uint8).copy()).to(dev)
d_chunks = d_chunks0.clone()
d_ios = torch.from_numpy(ios.view(np.uint8).copy()).to(dev)
d_res = torch.zeros(len(ios) * h3c.UPDATE_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
d_ctr = torch.zeros(8, dtype=torch.int64, device=dev)
slab0 = sc.slab.clone()
ref = None
for it in range(5):
    sc.slab.copy_(slab0)
    d_chunks.copy_(d_chunks0)
    d_res.fill_(0xA5)
    torch.cuda.synchronize()
    h3c.update_ios_dev(d_chunks, d_ios, d_res, counters=d_ctr)
    torch.cuda.synchronize()
    res = d_res.cpu().numpy().view(h3c.UPDATE_RESULT_DTYPE).copy()
    ch = d_chunks.cpu().numpy().view(h3c.CHUNK_STATE_DTYPE).copy()
    want = np.array([(e["status"], e["size"], e["type"], e["value"] & 0xFFFFFFFF) for e in sc.expect])
    got = np.stack([res["status"], res["size"], res["type"], res["value"]], 1).astype(np.int64)
    bad_oracle = int((got != want).any(1).sum())
    if ref is None:
        ref = (res, ch)
    d_res_bad = int((res != ref[0]).sum())
    diff_fields = {f: int((res[f] != ref[0][f]).sum()) for f in ("status", "size", "value", "type")}
    print(f"run {it}: vs oracle {bad_oracle} ops wrong; vs run 0: {diff_fields}, chunks differ "
          f"{int((ch != ref[1]).sum())}, counters {d_ctr.cpu().tolist()}, graphs (replays, captures, failures) "
          f"{[h3c.diag_counter(k) for k in range(3)]}; last error: {h3c.engine.lib.h3c_last_error()}", flush=True)
