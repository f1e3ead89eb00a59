#!/bin/bash
# Per-workgroup traces of the aligned UpdateIO kernel (4 rotating tables): working tree vs base look-back.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
AF_TABLES=4 H3C_LIB_PATH=$PWD/3fs_amd/_lib/diag/aftrace/libh3c_crc.so timeout -k 10 120 python -u scripts/af_trace.py > gpurun_out/r06_aftrace_wide.txt 2>&1 || { echo TRACE_FAIL; tail gpurun_out/r06_aftrace_wide.txt; exit 1; }
AF_TABLES=4 H3C_LIB_PATH=$PWD/3fs_amd/_lib/diag/basetrace/libh3c_crc.so timeout -k 10 120 python -u scripts/af_trace.py > gpurun_out/r06_aftrace_base.txt 2>&1 || { echo TRACE_FAIL; tail gpurun_out/r06_aftrace_base.txt; exit 1; }
for f in wide base; do echo "== $f"; sed -n '3,13p;26,28p' gpurun_out/r06_aftrace_$f.txt; done
