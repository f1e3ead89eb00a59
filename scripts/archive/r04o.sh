#!/bin/bash
# per-workgroup start / end times of uio_fast_kernel (H3C_FAST_TRACE=3 build) over a few config-3 batches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
H3C_LIB_PATH=$R/3fs_amd/_lib/diag/ftrace3/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --steps 4 --warmup 2 > gpurun_out/r04o_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 gpurun_out/r04o_trace.log; exit 1; }
grep -c fastwg gpurun_out/r04o_trace.log
echo R04O_OK
