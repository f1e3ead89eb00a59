#!/bin/bash
# Block-update path (h3c_update_blocks, upd_fused_kernel): one repeated write table against 4 in rotation.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_update_tables.txt
: > $out
for rep in 1 2; do
  for t in 4 1; do
    timeout -k 10 120 python -u bench.py --workload update --no-cpu-baseline --update-tables $t > gpurun_out/r06_upd.json || exit 1
    python - "tables=$t" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r06_upd.json") if l.startswith("{")][0])
r = d["roofline"]
print(f"{sys.argv[1]:10s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']} frac={r['frac']}")
PY
  done
done
cat $out
cp gpurun_out/r06_upd.json gpurun_out/r06_update_t1.json
