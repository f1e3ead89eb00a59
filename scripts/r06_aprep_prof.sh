#!/bin/bash
# The aligned UpdateIO kernels' durations per library (rocprofv3 kernel trace of the timed updio leg, 4 rotating
# tables), appended to gpurun_out/r06_aprep_ab.txt.  usage: scripts/r06_aprep_prof.sh label=lib ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
GRAFT_REPO_ROOT=$PWD
# each library's kernel durations (rocprof kernel trace of the timed updio leg)
for lv in "$@"; do
  label=${lv%%=*}; lib=$PWD/${lv#*=}
  cd /tmp && export TMPDIR=/tmp
  H3C_LIB_PATH=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/aprep_$label -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload updio --no-cpu-baseline --updio-headline-only --steps 60 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/aprep_$label.log 2>&1 || { echo PROF_FAIL $label; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/aprep_$label -name "kt_kernel_stats.csv" | head -1)
  python3 - "$label" "$f" <<'PY' | tee -a gpurun_out/r06_aprep_ab.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if "uio_a" in r["Name"]:
        print(f"{sys.argv[1]:8s} {r['Name'].split('(')[0][-24:]:26s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1e3:.2f} min_us={float(r['MinNs'])/1e3:.2f}")
PY
done
