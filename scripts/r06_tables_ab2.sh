#!/bin/bash
# Why rotated op tables run slower than one repeated table: learnt range weights (gain 0 variant) vs the
# same blocks being touched again (4 buffers of one draw).
set -e
out=gpurun_out/r06_tables_ab2.txt
: > $out
run() {  # label, lib, extra args
  H3C_LIB_PATH=$2 timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline $3 > gpurun_out/r06_tab.json
  python - "$1" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:28s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']}")
PY
}
CUR=3fs_amd/_lib/libh3c_crc.so
G0=3fs_amd/_lib/diag/gain0/libh3c_crc.so
for rep in 1 2; do
  run "cur tables=1" $CUR "--updio-tables 1"
  run "cur tables=4" $CUR "--updio-tables 4"
  run "cur tables=4 same-draw" $CUR "--updio-tables 4 --updio-same-tables"
  run "gain0 tables=1" $G0 "--updio-tables 1"
  run "gain0 tables=4" $G0 "--updio-tables 4"
done
cat $out
