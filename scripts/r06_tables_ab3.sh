#!/bin/bash
# The aligned kernel's time by launch form and step count (normal build), 4 rotating tables.
set -e
out=gpurun_out/r06_tables_ab3.txt
: > $out
run() {  # label, extra args
  timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline $2 > gpurun_out/r06_tab.json
  python - "$1" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:34s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']} "
      f"other_form_ms={d['other_form']['ms_per_step']} host_us={d['host_us_per_call']}")
PY
}
for rep in 1 2; do
  run "t4 graphs1 steps100 warm20" "--updio-tables 4 --updio-graphs 1"
  run "t4 graphs0 steps100 warm20" "--updio-tables 4 --updio-graphs 0"
  run "t4 graphs0 steps5 warm30" "--updio-tables 4 --updio-graphs 0 --steps 5 --warmup 30"
  run "t1 graphs0 steps100 warm20" "--updio-tables 1 --updio-graphs 0"
done
cat $out
