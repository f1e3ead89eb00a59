"""Per-kernel averages of a rocprofv3 --pmc counter collection (one line per kernel and counter,
averaged over its dispatches).  usage: python3 scripts/summarize_pmc.py <rocprofv3 -d directory>"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
if not f:
    sys.exit("no counter_collection.csv")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f[0])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    name = name.split("(")[0].split("<")[0][:48]
    acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    cs = acc[k]
    n = max(len(v) for v in cs.values())
    print(f"{k:48s} n={n:3d} " + " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
