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
lib = cx.h3c.engine.lib
runs, rots = [], [0, 0, 97]
for rep in range(3):  # the same batch each time (bench.run_updio regenerates it from the same seed)
    assert lib.h3c_diag_fast_rot(ctypes.c_uint32(rots[rep])) == 0  # (run 2: workgroup b takes range b + 97)
    bench.run_updio(args, cx)
    buf = (ctypes.c_ulonglong * (2 * 1024))()
    assert lib.h3c_diag_fast_wg(buf, 1024) == 0
    st = [buf[2 * b] for b in range(256)]
    en = [buf[2 * b + 1] for b in range(256)]
    t0 = min(st)
    ends = [(x - t0) / 100.0 for x in en]  # 100 MHz wall clock -> us
    runs.append(ends)
    e = sorted(ends)
    print("run %d: start spread %.1f us; end us: min %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f"
          % (rep, (max(st) - t0) / 100.0, e[0], e[25], e[128], e[230], e[253], e[-1]))
    by = {}
    for b in range(256):
        by.setdefault(b % 8, []).append(ends[b])
    print("   per XCD (b % 8) mean / max end:",
          "  ".join("%.1f/%.1f" % (statistics.mean(v), max(v)) for _, v in sorted(by.items())))
# is a workgroup's lateness a property of its CU (stable from batch to batch)?  rank correlation of the ends
skip = {0, 1, 128, 255}  # (the FAST_TRACE printfs slow these)
def ranks(v):
    o = sorted(range(len(v)), key=lambda i: v[i])
    r = [0] * len(v)
    for k, i in enumerate(o):
        r[i] = k
    return r
def spear(xa, xb):
    ra, rb = ranks(xa), ranks(xb)
    m = len(ra)
    return 1 - 6 * sum((x - y) ** 2 for x, y in zip(ra, rb)) / (m * (m * m - 1))
keep = [i for i in range(256) if i not in skip and (i - 97) % 256 not in skip]
print("same mapping, by workgroup: spearman(run 0, run 1) = %.3f" % spear([runs[0][i] for i in keep], [runs[1][i] for i in keep]))
# run 2 rotated: workgroup b took range b + 97; compare by workgroup (the CU side) and by range (the data side)
print("rotated, by workgroup:       spearman(run 1, run 2) = %.3f" % spear([runs[1][i] for i in keep], [runs[2][i] for i in keep]))
print("rotated, by range:           spearman(run 1, run 2) = %.3f" % spear([runs[1][(i + 97) % 256] for i in keep], [runs[2][i] for i in keep]))
# what in a range makes it late: the ops its waves run (its chain starts and their later ops), and how many of
# those are later ops of a chain (their rows load with nothing else in flight)
import numpy as np  # noqa: E402
g = np.random.default_rng(bench.SEED + 0)
wc = g.integers(0, 64, 100000).astype(np.int64)
wb = g.integers(0, (64 << 20) // 4096, 100000).astype(np.int64)
key = wc * (1 << 20) + wb
first = {}
length = np.zeros(100000, dtype=np.int64)
for i, k in enumerate(key.tolist()):
    h = first.setdefault(k, i)
    length[h] += 1
nw = 256 * 16
work = np.zeros(256)
conts = np.zeros(256)
for r in range(256):
    lo, hi = r * 16 * 100000 // nw, (r + 1) * 16 * 100000 // nw
    seg = length[lo:hi]
    work[r] = seg.sum()
    conts[r] = (seg - 1).clip(min=0).sum()
ends_by_range = [runs[1][(r - 0) % 256] for r in range(256)]  # run 1: workgroup b took range b
keepr = [r for r in range(256) if r not in skip]
print("ops run per range: mean %.1f sd %.1f; later ops per range: mean %.1f sd %.1f" % (work.mean(), work.std(), conts.mean(), conts.std()))
print("spearman(end, ops run) = %.3f; spearman(end, later ops) = %.3f" % (
    spear([ends_by_range[r] for r in keepr], [work[r] for r in keepr]),
    spear([ends_by_range[r] for r in keepr], [conts[r] for r in keepr])))
