#!/bin/bash
# wave end-time histograms: the fast kernel (H3C_FAST_TRACE=2) and the general block kernel (H3C_BLOCK_TRACE=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
H3C_LIB_PATH=$R/3fs_amd/_lib/diag/ftrace/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --steps 3 --warmup 1 > $O/r04c_ftrace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/r04c_ftrace.log; exit 1; }
H3C_UPD_FAST=1 H3C_LIB_PATH=$R/3fs_amd/_lib/diag/btrace/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --steps 3 --warmup 1 > $O/r04c_btrace.log 2>&1 || { echo BTRACE_FAIL; tail -20 $O/r04c_btrace.log; exit 1; }
echo R04C_OK
grep "fast waves" $O/r04c_ftrace.log | tail -4
grep "btrace" $O/r04c_btrace.log | tail -2
