"""The bench line's kernel time (the kernel's own wall-clock stamps) against rocprofv3's durations of the
same launches, in the profiled process of scripts/profile.sh.  usage:
python3 scripts/stamps_vs_rocprof.py gpurun_out/prof_<tag> <kernel name part>
The timed leg is the `steps` launches after the `warmup` ones (one kernel launch per step)."""
import csv
import json
import sys

d, kern = sys.argv[1], sys.argv[2]
line = [l for l in open(f"{d}/kt_bench.log") if l.startswith('{"metric"')][-1]
b = json.loads(line)
rows = sorted((r for r in csv.DictReader(open(f"{d}/kt/kt_kernel_trace.csv")) if kern in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
w, s = b["warmup"], b["steps"]
timed = dur[w:w + s]
m = sum(timed) / len(timed)
k = b["roofline"]["kernel_avg_us"]
print(f"# {kern}: the bench's timed leg ({s} launches after {w} warm) in one rocprofv3 --kernel-trace process")
print(f"#   bench (kernel stamps): {k:.2f} us per launch; rocprof: {m:.2f} us (min {min(timed):.2f}, max {max(timed):.2f});"
      f" {100 * abs(k - m) / m:.2f} % apart")
print(f"#   all {len(dur)} launches of the process (every leg): rocprof mean {sum(dur) / len(dur):.2f} us")
