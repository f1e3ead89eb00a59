#!/bin/bash
# Kernel-trace timelines of the config-3 UpdateIO batch for the in-tree library and variants
# (VARIANTS; "scan" = the in-tree library with H3C_UPD_FRONT=1).  Outputs: gpurun_out/<TAG>_tl_<v>.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${TAG:-r03}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in cur ${VARIANTS:-}; do
  lib=$R/3fs_amd/_lib/libh3c_crc.so; front=0
  [ "$v" = scan ] && front=1
  [ "$v" != cur ] && [ "$v" != scan ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
  OUT=$R/gpurun_out/${T}_kt_$v
  H3C_UPD_FRONT=$front H3C_LIB_PATH=$lib timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT -o kt --output-format csv -- \
    python3 $R/bench.py --workload updio --no-cpu-baseline --steps 6 --warmup 2 > $OUT.log 2>&1 || { echo KT_${v}_FAIL; exit 1; }
  f=$(find $OUT -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/updio_timeline.py $f > $R/gpurun_out/${T}_tl_$v.txt || { echo TL_${v}_FAIL; exit 1; }
done
echo PROF_OK
