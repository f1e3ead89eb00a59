#!/bin/bash
# Aligned UpdateIO: kernel time with the pipeline captured in a graph (the headline form) and with plain
# launches, 4 rotating op tables, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_graphs_ab.txt
: > $out
for rep in 1 2; do
  for g in 1 0; do
    timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline --updio-tables 4 --updio-graphs $g > gpurun_out/r06_tab.json || exit 1
    python - "graphs=$g" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:10s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']}")
PY
  done
done
cat $out
