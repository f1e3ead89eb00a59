#!/bin/bash
# tail-kernel step times (trace build) and the fast kernel with every op its own chain (FX 64, timing only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
H3C_LIB_PATH=$R/3fs_amd/_lib/diag/ftrace/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --steps 3 --warmup 1 > $O/r04f_trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/r04f_trace.log; exit 1; }
H3C_LIB_PATH=$R/3fs_amd/_lib/diag/fx64/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline > $O/r04f_fx64.jsonl 2>$O/r04f_fx64.err
tail -1 $O/r04f_fx64.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fx64', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['verified'])"
grep "tail tile" $O/r04f_trace.log | tail -8
