"""Timeline of one UpdateIO batch from a rocprofv3 --kernel-trace CSV: the kernels of the last
complete batch (from the last uio_prep_kernel on), with start / end in microseconds from that
kernel's start, plus the batch span.  usage: python3 scripts/updio_timeline.py <kernel_trace.csv>"""
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if "rocprim" in name:
        for key in ("scan_by_key", "init_lookback", "lookback_scan", "merge", "block_sort", "scan"):
            if key in name:
                return "rocprim::" + key
        return "rocprim"
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].split("<")[0][:48]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
preps = [k for k, r in enumerate(rows) if "uio_prep_kernel" in r["Kernel_Name"]]
if len(preps) < 2:
    sys.exit("fewer than two batches in the trace")
a, b = preps[-2], preps[-1]  # the second-to-last batch is complete
t0 = int(rows[a]["Start_Timestamp"])
end = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    end = max(end, e)
    print(f"{short(r['Kernel_Name']):50s} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
print(f"batch span {end / 1e3:.1f} us; next batch starts at {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")
