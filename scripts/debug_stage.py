import importlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import oracle_lib as orc
h3c = importlib.import_module("3fs_amd")
rng = np.random.default_rng(1)
for n in (1, 100, 4096, 65536, 1 << 20, (3 << 20) + 123):
    a = rng.integers(0, 256, n, dtype=np.uint8)
    for start in (0xFFFFFFFF, 0x1234):
        t, v = h3c.batch_create([(a, n, start)])
        d = torch.from_numpy(a).cuda()
        t2, v2 = h3c.batch_create([(d, n, start)])
        w = orc.crc32c(a, start)
        print(n, hex(start), "host", int(v[0]) == w, "dev", int(v2[0]) == w, hex(int(v[0])), hex(w), flush=True)
