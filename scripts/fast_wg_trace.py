"""Per-workgroup start / end of uio_fast_kernel on config 3 (the H3C_FAST_TRACE=3 diag build, loaded through
H3C_LIB_PATH): runs bench.py's updio workload briefly, then reads the last launch's stamps."""
import argparse
import ctypes
import statistics
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

args = argparse.Namespace(steps=5, warmup=2, writes=100000, exact=False, updio_order="random", updio_graphs=0,
                          no_cpu_baseline=True)
cx = bench.Ctx()
bench.run_updio(args, cx)
lib = cx.h3c.engine.lib
n = cx.h3c.engine.device_num_cu(0) if hasattr(cx.h3c.engine, "device_num_cu") else 256
buf = (ctypes.c_ulonglong * (2 * 1024))()
assert lib.h3c_diag_fast_wg(buf, 1024) == 0
st = [buf[2 * b] for b in range(256)]
en = [buf[2 * b + 1] for b in range(256)]
t0 = min(st)
e = sorted((x - t0) / 100.0 for x in en)  # 100 MHz wall clock -> us
print("workgroups 256; start spread %.1f us" % ((max(st) - t0) / 100.0))
print("end us: min %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f" % (e[0], e[25], e[128], e[230], e[253], e[-1]))
by = {}
for b in range(256):
    by.setdefault(b % 8, []).append((en[b] - t0) / 100.0)
print("per XCD (b % 8) mean / max end:", "  ".join("%.1f/%.1f" % (statistics.mean(v), max(v)) for _, v in sorted(by.items())))
