"""Summarize scripts/r04_fetchcal.sh: per kernel, the average per-dispatch FETCH_SIZE and the
memory-side read requests by size, against the kernel's known bytes per launch (8 GiB for every
kernel measured).  Usage: python3 scripts/summarize_fetchcal.py gpurun_out/r04cal"""
import csv
import glob
import json
import sys
from collections import defaultdict

BYTES = 8 << 30


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            key = next((k for k in ("fetchcal_rows4_span_plain", "fetchcal_rows4_span", "fetchcal_rows4_plain",
                                    "fetchcal_rows4_b8", "fetchcal_rows4", "fetchcal_rows8", "fetchcal_wide",
                                    "seg_uni_kernel", "seg_crc_kernel") if k in name), None)
            if key:
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


out = {}
for sub in sys.argv[1:]:
    for kern, ctrs in load(sub).items():
        o = out.setdefault(kern, {})
        for c, v in ctrs.items():
            o[c] = sum(v) / len(v)
for kern, o in out.items():
    if "TCC_EA0_RDREQ_sum" in o:
        n32, n64, n128 = (o.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) for s in (32, 64, 128))
        o["request_bytes"] = 32 * n32 + 64 * n64 + 128 * n128
        o["request_bytes_over_8GiB"] = o["request_bytes"] / BYTES
        o["rdreq_x64_over_8GiB"] = o["TCC_EA0_RDREQ_sum"] * 64 / BYTES
    if "FETCH_SIZE" in o:
        o["fetch_x1024_over_8GiB"] = o["FETCH_SIZE"] * 1024 / BYTES
        o["fetch_x2048_over_8GiB"] = o["FETCH_SIZE"] * 2048 / BYTES
print(json.dumps(out, indent=1))
