"""Per-batch kernel timelines from a rocprofv3 kernel trace: each batch starts at a kernel whose
name contains the first argument (default uio_zero_kernel); prints every batch's kernels as
name start-end (us from the batch start) and the gap to the next batch.
Usage: python3 scripts/ktimeline.py kt_kernel_trace.csv [first-kernel] [max-batches]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "uio_zero_kernel"
mx = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
for a, i in enumerate(starts[:mx]):
    j = starts[a + 1] if a + 1 < len(starts) else len(rows)
    t0 = int(rows[i]["Start_Timestamp"])
    parts = []
    for r in rows[i:j]:
        nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        nm = nm.split("(")[0].split("<")[0].replace("uio_", "").replace("_kernel", "")
        parts.append(f"{nm} {(int(r['Start_Timestamp']) - t0) / 1e3:.1f}-{(int(r['End_Timestamp']) - t0) / 1e3:.1f}")
    nxt = f" | next {(int(rows[j]['Start_Timestamp']) - t0) / 1e3:.1f}" if j < len(rows) else ""
    print(f"{a:3d}: " + " | ".join(parts) + nxt)
