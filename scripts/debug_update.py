import importlib, sys, os, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
h3c = importlib.import_module("3fs_amd")
print("cuda", torch.cuda.is_available(), "h3c devices", h3c.device_count(), flush=True)
print("ws bytes", h3c.update_workspace_bytes(1000, 4, 128 << 10), "err:", h3c.lib.h3c_last_error(), flush=True)
x = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
t, v = h3c.batch_create([x])
print("create ok", hex(int(v[0])), flush=True)
print("ws bytes after init", h3c.update_workspace_bytes(1000, 4, 128 << 10), flush=True)
