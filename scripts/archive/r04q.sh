#!/bin/bash
# Kernel traces of bench --workload updio: the in-tree build and diag variants (timing-only variants may fail
# verification; only their kernel durations are read).  usage: scripts/r04q.sh <variant> [<variant> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in cur "$@"; do
  OUT=$R/gpurun_out/r04q_$v
  L=""; [ $v = cur ] || L=$R/3fs_amd/_lib/diag/$v/libh3c_crc.so
  H3C_LIB_PATH=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 $R/bench.py --workload updio --no-cpu-baseline --steps 20 --warmup 2 > $OUT.log 2>&1
  rc=$?; [ $rc -le 1 ] || { echo KT_${v}_FAIL $rc; tail -5 $OUT.log; exit 1; }
  echo "== $v"; python3 $R/scripts/kstats.py $OUT/kt_kernel_stats.csv | grep -E "uio_" || true
done
echo R04Q_OK
