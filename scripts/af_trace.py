"""Per-workgroup phases of uio_afused_kernel (an H3C_AF_TRACE=1 build: scripts/build_variant.sh aftrace
-DH3C_AF_TRACE=1): runs config-3 UpdateIO batches and prints, per ticket-ordered workgroup, its start, table
fill, main loop, look-back and tail in microseconds from the first start (quantiles over workgroups).
usage: H3C_LIB_PATH=.../diag/aftrace/libh3c_crc.so python scripts/af_trace.py"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0], "--workload", "updio", "--no-cpu-baseline", "--steps", "5", "--warmup", "30", "--updio-tables", os.environ.get("AF_TABLES", "4"), "--updio-headline-only",
            "--updio-graphs", "0"]
bench = importlib.import_module("bench")
h3c = importlib.import_module("3fs_amd")
rc = bench.main()
lib = h3c.engine.lib
lib.h3c_diag_af_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
nwg = 250
buf = (ctypes.c_ulonglong * (5 * 1024))()
assert lib.h3c_diag_af_trace(buf, 1024) == 0
a = np.array(buf[:5 * nwg], dtype=np.float64).reshape(nwg, 5)
khz = 100000.0  # the wall clock's 100 MHz
t0 = a[:, 0].min()
us = (a - t0) / (khz / 1000.0)
names = ["start", "filled", "loop_end", "lookback_end", "end"]
lib.h3c_diag_af_entry.argtypes = [ctypes.c_void_p, ctypes.c_int]
ent = (ctypes.c_ulonglong * (2 * 1024))()
assert lib.h3c_diag_af_entry(ent, 1024) == 0
e = np.array(ent[:2 * nwg], dtype=np.float64).reshape(nwg, 2)
e0 = e[:, 0].min()
eu = (e - e0) / (khz / 1000.0)
print("kernel entry -> post-fill sync (us): first entry 0; entry q0/q50/q100 = %.1f/%.1f/%.1f; ticket taken "
      "q0/q50/q100 = %.1f/%.1f/%.1f; sync passed q0/q100 = %.1f/%.1f" % (
          *np.percentile(eu[:, 0], [0, 50, 100]), *np.percentile(eu[:, 1], [0, 50, 100]),
          (a[:, 0].min() - e0) / (khz / 1000.0), (a[:, 0].max() - e0) / (khz / 1000.0)))
print("entry order vs ticket wait (us), first 8 by entry:", [(round(float(x), 1), round(float(y - x), 1))
                                                          for x, y in sorted(eu.tolist())[:8]])
for q in (0, 50, 90, 99, 100):
    print(f"q{q:3d} " + " ".join(f"{n}={np.percentile(us[:, i], q):7.1f}" for i, n in enumerate(names)))
print("per-wg loop time (loop_end - filled): median %.1f max %.1f" % (np.median(us[:, 2] - us[:, 1]), (us[:, 2] - us[:, 1]).max()))
print("look-back wait (lookback_end - loop_end): median %.1f max %.1f" % (np.median(us[:, 3] - us[:, 2]), (us[:, 3] - us[:, 2]).max()))
print("tail (end - lookback_end): median %.1f max %.1f" % (np.median(us[:, 4] - us[:, 3]), (us[:, 4] - us[:, 3]).max()))
order = np.argsort(us[:, 2])[-5:]
print("latest loop ends (ticket, us):", [(int(i), round(float(us[i, 2]), 1)) for i in order])
corr = np.corrcoef(np.arange(nwg), us[:, 2] - us[:, 1])[0, 1]
print("corr(ticket, loop time) = %.2f" % corr)
lib.h3c_diag_af_waves.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
wv = (ctypes.c_ulonglong * (16 * 1024))()
bk = (ctypes.c_uint32 * (4 * 1024))()
fn = (ctypes.c_uint32 * (16 * 1024))()
assert lib.h3c_diag_af_waves(wv, bk, fn, 1024) == 0
fin = np.array(fn[:16 * nwg]).reshape(nwg, 16)
w = (np.array(wv[:16 * nwg], dtype=np.float64).reshape(nwg, 16) - t0) / (khz / 1000.0)
blk = np.array(bk[:4 * nwg]).reshape(nwg, 4)
ops = (blk[:, 3] - blk[:, 2]).astype(np.float64)
loop = us[:, 2] - us[:, 1]
spread = w.max(1) - w.min(1)
print("per-wg wave spread (max - min wave end): median %.1f max %.1f" % (np.median(spread), spread.max()))
print("wave ends: q0 %.1f q50 %.1f q90 %.1f q100 %.1f" % tuple(np.percentile(w, [0, 50, 90, 100])))
for x in range(8):
    m = blk[:, 1] == x
    if m.any():
        print("xcc %d: %3d wgs, loop_end median %.1f max %.1f, mean wave end %.1f, mean ticket %.0f, fin ops/wave %.2f, "
              "ops/wg %.1f, loop %.1f us, ops/us %.3f" % (
            x, m.sum(), np.median(us[m, 2]), us[m, 2].max(), w[m].mean(), np.arange(nwg)[m].mean(), fin[m].mean(),
            ops[m].mean(), loop[m].mean(), (ops[m] / loop[m]).mean()))
wl = (w - us[:, 1:2]).ravel()
print("corr(wave time, fin ops) = %.2f; fin ops/wave by ticket quartile:" % np.corrcoef(wl, fin.ravel())[0, 1],
      [round(float(fin[q * nwg // 4:(q + 1) * nwg // 4].mean()), 2) for q in range(4)])
# the look-back's own latency: from the moment every ticket up to L (itself included) has ended its loop
pre = np.maximum.accumulate(us[:, 2])
exc = us[:, 3] - pre
print("look-back latency after the last predecessor's loop end: q50 %.1f q90 %.1f max %.1f (ticket %d)" % (
    np.median(exc), np.percentile(exc, 90), exc.max(), int(exc.argmax())))
lo = np.argsort(us[:, 3])[-8:]
print("latest look-back ends (ticket, loop_end, predecessors' last loop end, lookback_end):",
      [(int(i), round(float(us[i, 2]), 1), round(float(pre[i]), 1), round(float(us[i, 3]), 1)) for i in lo])
# per-workgroup loop time against its ops and its fin-path ops (a block's first of several writes)
finw = fin.sum(1).astype(np.float64)
A = np.stack([ops, finw], 1)
coef, *_ = np.linalg.lstsq(A, loop, rcond=None)
print("loop time ~ %.4f us/op + %.4f us/fin-op (fin-op extra cost = %.2f ops); residual std %.1f us" % (
    coef[0], coef[1], coef[1] / coef[0], np.std(loop - A @ coef)))
q4 = [slice(q * nwg // 4, (q + 1) * nwg // 4) for q in range(4)]
print("by ticket quartile: ops", [round(float(ops[s_].mean()), 1) for s_ in q4], "fin ops", [round(float(finw[s_].mean()), 1) for s_ in q4],
      "loop us", [round(float(loop[s_].mean()), 1) for s_ in q4], "loop_end", [round(float(us[s_, 2].mean()), 1) for s_ in q4])
print("blockIdx -> xcc:", [(int(blk[i, 0]), int(blk[i, 1])) for i in range(12)])
# which waves are late: their op ranges (ticket * 16 + wave) -> position in the batch
late = np.argsort(w.ravel())[-20:]
print("latest waves (ticket, wave, end):", [(int(i // 16), int(i % 16), round(float(w.ravel()[i]), 1)) for i in late[-8:]])
sys.exit(rc)
