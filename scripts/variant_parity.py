"""Quick parity of each variant .so (H3C_LIB_PATH) vs the oracle across segment sizes."""
import importlib, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle_lib as orc
h3c = importlib.import_module("3fs_amd")
rng = np.random.default_rng(3)
sizes = [1, 17, 1024, 4096, 6144, 9216, 12345, 16385, 65543, 262144 + 1000, (1 << 20) + 3, 3 << 20]
host = rng.integers(0, 256, sum(sizes) + 64, dtype=np.uint8)
buf = torch.from_numpy(host).cuda()
bad = 0
for seg in (1024, 16384, 262144, 1 << 20):
    os.environ["H3C_SEG_BYTES"] = str(seg)
    items, want, off = [], [], 5
    for n in sizes:
        items.append((buf[off: off + n], n)); want.append(orc.crc32c(host[off: off + n])); off += n
    _, got = h3c.batch_create(items)
    bad += sum(int(g) != w for g, w in zip(got, want))
print(os.path.basename(os.environ.get("H3C_LIB_PATH", "default")), "PARITY", "OK" if bad == 0 else f"BAD({bad})", flush=True)
sys.exit(1 if bad else 0)
