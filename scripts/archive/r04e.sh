#!/bin/bash
# kernel-trace timelines of the config-3 UpdateIO batch: the fast branch and (H3C_UPD_FAST=1) the general
# pipeline; rocprofv3 --kernel-trace --stats summaries.  Outputs: gpurun_out/r04e_*
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in fast general; do
  f1=0; [ $v = general ] && f1=1
  OUT=$R/gpurun_out/r04e_kt_$v
  H3C_UPD_FAST=$f1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- \
    python3 $R/bench.py --workload updio --no-cpu-baseline --steps 20 --warmup 2 > $OUT.log 2>&1 || { echo KT_${v}_FAIL; exit 1; }
  f=$(find $OUT -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/updio_timeline.py $f > $R/gpurun_out/r04e_tl_$v.txt || { echo TL_${v}_FAIL; exit 1; }
done
echo PROF_OK
cat $R/gpurun_out/r04e_tl_fast.txt
cat $R/gpurun_out/r04e_tl_general.txt
