"""Host + device timeline of UpdateIO batches from a rocprofv3 --hip-trace --kernel-trace run
(scripts/r04i.sh): per batch, the HIP calls (repeated device queries folded into one line) and the
kernels, in microseconds from the batch's first kernel.
Usage: python3 scripts/host_timeline.py <dir with ht_hip_api_trace.csv / ht_kernel_trace.csv> [batch ...]"""
import csv
import sys

d = sys.argv[1]
api = sorted(csv.DictReader(open(f"{d}/ht_hip_api_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
kt = sorted(csv.DictReader(open(f"{d}/ht_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
zs = [r for r in kt if "uio_prep_kernel" in r["Kernel_Name"]]
picks = [int(x) for x in sys.argv[2:]] or [4, len(zs) - 3]
for b in picks:
    t0 = int(zs[b]["Start_Timestamp"])
    t_next = int(zs[b + 1]["Start_Timestamp"]) if b + 1 < len(zs) else t0 + 10**6
    prev_end = max(int(r["End_Timestamp"]) for r in kt if int(r["End_Timestamp"]) <= t0)
    print(f"batch {b}: previous batch's last kernel ended at {(prev_end - t0) / 1e3:.1f}; next batch at "
          f"{(t_next - t0) / 1e3:.1f}")
    ev = [((int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3, "H " + r["Function"])
          for r in api if prev_end - 20000 <= int(r["Start_Timestamp"]) < t_next]
    ev += [((int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3,
            "K " + r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0])
           for r in kt if t0 <= int(r["Start_Timestamp"]) < t_next]
    ev.sort()
    fold = None
    for s, e, name in ev:
        q = any(x in name for x in ("GetDevice", "DeviceGetAttribute", "CallConfiguration", "GetLastError"))
        if q:
            fold = (fold[0], e, fold[2] + 1) if fold else (s, e, 1)
            continue
        if fold:
            print(f"  {fold[0]:8.1f} {fold[1]:8.1f}  H ({fold[2]} device / launch-config queries)")
            fold = None
        print(f"  {s:8.1f} {e:8.1f}  {name}")
