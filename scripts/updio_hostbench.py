# Host-pass timing of h3c_update_ios without device work (h3c_diag_updio_host_ms): 100k random
# 4 KiB UpdateIOs into 64 x 64 MiB chunks.  usage: python scripts/updio_hostbench.py [lib.so]
import ctypes, numpy as np, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3fs_amd", "_lib", "libh3c_crc.so"))
CS = np.dtype([("base", "<u8"), ("chunk_size", "<u4"), ("size", "<u4"), ("value", "<u4"), ("type", "u1"), ("r", "u1", 3)])
IO = np.dtype([("payload", "<u8"), ("chunk", "<u4"), ("offset", "<u4"), ("length", "<u4"), ("checksum_value", "<u4"),
               ("checksum_type", "u1"), ("kind", "u1"), ("r", "u1", 6)])
nch, clen, nw, G = 64, 64 << 20, 100000, 4096
st = np.zeros(nch, CS); st["base"] = (1 << 40) + np.arange(nch, dtype=np.uint64) * clen; st["chunk_size"] = clen
st["size"] = clen; st["type"] = 1
g = np.random.default_rng(5)
ios = np.zeros(nw, IO); ios["payload"] = (1 << 44) + np.arange(nw, dtype=np.uint64) * G
ios["chunk"] = g.integers(0, nch, nw); ios["offset"] = g.integers(0, clen // G, nw) * G; ios["length"] = G
ios["checksum_type"] = 1; ios["kind"] = 1
f = lib.h3c_diag_updio_host_ms; f.restype = ctypes.c_double
f.argtypes = [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
f(1, st.ctypes.data, nch, ios.ctypes.data, nw, 3)
print("host ms per 100k ops:", round(f(1, st.ctypes.data, nch, ios.ctypes.data, nw, 200), 3))
