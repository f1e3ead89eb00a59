"""Per-kernel summary of a scripts/profile.sh output directory: kernel-trace stats plus
HBM bytes per launch from the separate FETCH_SIZE / WRITE_SIZE passes (KiB; FETCH_SIZE
doubled on gfx950 per MI355X_MICROARCH.md §HBM -- exact for wide coalesced streaming reads)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]


def one(pattern):
    f = glob.glob(f"{d}/{pattern}", recursive=True)
    return f[0] if f else None


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if "rocprim" in name:
        for key in ("onesweep_histogram", "onesweep_iteration", "onesweep_scan", "radix_sort_block_sort",
                    "radix_sort_merge", "scan_by_key", "init_lookback", "lookback_scan", "scan"):
            if key in name:
                return "rocprim::" + key
        return "rocprim::" + name[:40]
    return name.split("(")[0].split("<")[0][:60]


stats = one("kt/**/kt_kernel_stats.csv")
print(f"{'kernel':62s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'pct':>6s}")
for r in csv.DictReader(open(stats)):
    print(f"{short(r['Name']):62s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.2f} "
          f"{float(r['MinNs'])/1e3:10.2f} {float(r['Percentage']):6.2f}")


def pmc(pattern, counter):
    f = one(pattern)
    acc = collections.defaultdict(list)
    if not f:
        return acc
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


fetch = pmc("fetch/**/fetch_counter_collection.csv", "FETCH_SIZE")
write = pmc("write/**/write_counter_collection.csv", "WRITE_SIZE")
print()
print(f"{'kernel':62s} {'read_B/launch(x2)':>18s} {'write_B/launch':>16s}")
for k in sorted(set(fetch) | set(write)):
    fr = fetch.get(k, [])
    wr = write.get(k, [])
    rb = 2 * 1024 * sum(fr) / len(fr) if fr else float("nan")
    wb = 1024 * sum(wr) / len(wr) if wr else float("nan")
    print(f"{k:62s} {rb:18.0f} {wb:16.0f}")
