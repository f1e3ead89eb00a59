"""Short per-kernel table of a rocprofv3 --stats kernel_stats.csv: name, calls, average and min (us)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:44]
    print(f"{n:46s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:9.2f} us  min {float(r['MinNs']) / 1e3:9.2f} us")
