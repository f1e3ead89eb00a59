"""The durations of one kernel's dispatches in launch order from a rocprofv3 kernel trace, grouped by
position modulo `period` (e.g. the 4 rotating op tables of bench.py --workload updio).
usage: python3 scripts/kseq.py kt_kernel_trace.csv kernel_substring [period] [skip]"""
import csv
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
name = sys.argv[2]
period = int(sys.argv[3]) if len(sys.argv) > 3 else 1
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]])
print(f"{name}: {d.size} dispatches, mean {d.mean():.1f} us")
d = d[skip:]
print("sequence (us):", " ".join(f"{x:.0f}" for x in d[:48]))
for k in range(period):
    x = d[k::period]
    print(f"  position {k} mod {period}: n={x.size} mean {x.mean():.1f} min {x.min():.1f} max {x.max():.1f}")
