#!/bin/bash
# host-side timeline of the UpdateIO batches: HIP API trace + kernel trace of bench updio
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/r04i_ht
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace -d $OUT -o ht --output-format csv -- python3 $R/bench.py --workload updio --no-cpu-baseline --steps 10 --warmup 2 > $OUT.log 2>&1 || { echo HT_FAIL; tail -5 $OUT.log; exit 1; }
ls $OUT
echo R04I_OK
