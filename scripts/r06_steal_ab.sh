#!/bin/bash
# Aligned UpdateIO kernel with and without work stealing, 4 rotating op tables (and 1 table), same box.
set -e
out=gpurun_out/r06_steal_ab.txt
: > $out
run() {  # label, lib, extra args
  H3C_LIB_PATH=$2 timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline $3 > gpurun_out/r06_tab.json
  python - "$1" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:22s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']} "
      f"redo={sum(d['redo'].values())} branch={d['branch'][:12]}")
PY
}
CUR=3fs_amd/_lib/libh3c_crc.so
NS=3fs_amd/_lib/diag/nosteal/libh3c_crc.so
for rep in 1 2 3; do
  run "steal t4" $CUR "--updio-tables 4"
  run "nosteal t4" $NS "--updio-tables 4"
  run "steal t1" $CUR "--updio-tables 1"
done
cat $out
