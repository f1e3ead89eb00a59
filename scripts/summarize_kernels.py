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
    if name.startswith("void "):  # template kernels carry their return type
        name = name[5:]
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

# --json KERNEL ALG_BYTES WORKLOAD: also write the profiles/*_pmc_summary.json form that
# bench.py's roofline() reads for `traffic` (per launch, same corrections).
if len(sys.argv) > 2 and sys.argv[2] == "--json":
    import json

    kern, alg, workload, out = sys.argv[3], int(sys.argv[4]), sys.argv[5], sys.argv[6]
    row = next(r for r in csv.DictReader(open(stats)) if short(r["Name"]) == kern)
    fr, wr = fetch.get(kern, []), write.get(kern, [])
    rb = 2 * 1024 * sum(fr) / len(fr)
    wb = 1024 * sum(wr) / len(wr)
    # the last half of the kernel's dispatches (kernels whose per-XCD range weights settle over the first
    # batches of a stream: the steady state the bench's timed steps see)
    durs = []
    trace = one("kt/**/kt_kernel_trace.csv")
    if trace:
        for r in csv.DictReader(open(trace)):
            if short(r["Kernel_Name"]) == kern:
                durs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    durs = [x for _, x in sorted(durs)]
    tail = durs[len(durs) // 2:]
    json.dump({
        "kernel": kern,
        kern: {"calls": int(row["Calls"]), "avg_us": float(row["AverageNs"]) / 1e3,
               "min_us": float(row["MinNs"]) / 1e3, "pct_gpu_time": float(row["Percentage"]),
               "avg_us_last_half": (sum(tail) / len(tail) / 1e3) if tail else None},
        "pmc": {"FETCH_SIZE_kib_raw": sum(fr) / len(fr), "WRITE_SIZE_kib": sum(wr) / len(wr),
                "hbm_read_bytes_per_launch": rb, "hbm_write_bytes_per_launch": wb,
                "correction": "FETCH_SIZE x1024 x2 (gfx950 reports half of a wide streaming read); WRITE_SIZE x1024",
                "traffic_bytes_per_launch": rb + wb},
        "algorithmic_bytes_per_launch": alg,
        "workload": workload,
        "command": "scripts/profile.sh (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE) + "
                   "scripts/summarize_kernels.py --json",
    }, open(out, "w"), indent=1)
