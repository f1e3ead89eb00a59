#!/bin/bash
# Per-XCD weight learning gain with 4 rotating op tables (the honest config-3 loop), same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_gain_t4.txt
: > $out
run() {  # label, lib
  H3C_LIB_PATH=$2 timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline --updio-tables 4 > gpurun_out/r06_tab.json || exit 1
  python - "$1" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:10s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']}")
PY
}
for rep in 1 2 3; do
  run "g0.5" $PWD/3fs_amd/_lib/libh3c_crc.so
  for g in 0.25 0.125 0.0; do run "g$g" $PWD/3fs_amd/_lib/diag/g$g/libh3c_crc.so; done
done
cat $out
