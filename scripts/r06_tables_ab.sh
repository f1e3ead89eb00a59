#!/bin/bash
# A/B on one box: the config-3 UpdateIO bench with one op table repeated vs 4 seeded tables in rotation.
set -e
out=gpurun_out/r06_tables_ab.txt
: > $out
for rep in 1 2; do
  for t in 1 4; do
    timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline --updio-tables $t > gpurun_out/r06_tab.json
    python - "$t" "$rep" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"tables={sys.argv[1]} rep={sys.argv[2]} ms={d['ms_per_step']} wps={d['value']} verified={d['verified']} "
      f"kernel_us={r['kernel_avg_us']} frac_stamps={r.get('frac_stamps', r['frac'])} branch={d['branch']}")
PY
  done
done
cat $out
