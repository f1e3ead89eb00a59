"""Config 4: the bench's warm per-launch time against rocprofv3's durations in the same process.
usage: python3 scripts/shard4m_warm.py gpurun_out/prof_shard4m
Per pass of 16384 x 4 MiB the bench launches seg_crc_kernel as: create (cold), warm, 3 timed."""
import csv
import json
import sys

d = sys.argv[1]
line = [l for l in open(f"{d}/kt_bench.log") if l.startswith('{"metric"')][-1]
b = json.loads(line)
rows = sorted((r for r in csv.DictReader(open(f"{d}/kt/kt_kernel_trace.csv")) if "seg_crc_kernel" in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
npass = len(b["pass_ms"])
assert len(dur) == 5 * npass, (len(dur), npass)
k = b["roofline"]["kernel_avg_us"]
print("# Config 4 (VERDICT r03 #5): the bench's warm per-launch time against rocprofv3 in the same process (round-4 refresh).")
print("# rocprofv3 --kernel-trace of bench.py --workload shard4m (scripts/profile.sh via scripts/r04_prof.sh): per pass of")
print("# 16384 x 4 MiB, seg_crc_kernel launches in order: create (cold: the pass's first touches), warm, 3 timed.")
print("# The bench line printed by that process (kernel_avg_us: the kernels' own wall-clock stamps over the timed launches):")
print(f"#   pass_ms {b['pass_ms']} kernel_avg_us {k:.2f} frac {b['roofline']['frac']}")
print("# rocprof durations (us), one row per pass:")
timed = []
for p in range(npass):
    c, w, *t = dur[5 * p:5 * p + 5]
    timed += t
    print(f"  create {c:.1f}  warm {w:.1f}  timed " + " ".join(f"{x:.1f}" for x in t))
m = sum(timed) / len(timed)
print(f"# timed launches: rocprof mean {m:.1f} us; the bench {k:.2f} us in the same process: {abs(m - k) / m * 100:.2f} % apart")
