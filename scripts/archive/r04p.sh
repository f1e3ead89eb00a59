#!/bin/bash
# Block-update step (bench --workload update): the shipped build against diag variants, alternating, then a
# kernel trace of the shipped build.  usage: scripts/r04p.sh <variant> [<variant> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
line() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['verified'])"; }
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload update --no-cpu-baseline --steps 100 --warmup 20 > $O/r04p_cur.jsonl 2> $O/r04p_cur.err || { echo BENCH_FAIL; tail -20 $O/r04p_cur.err; exit 1; }
  line $O/r04p_cur.jsonl cur
  for v in "$@"; do
    H3C_LIB_PATH=$R/3fs_amd/_lib/diag/$v/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload update --no-cpu-baseline --steps 100 --warmup 20 > $O/r04p_$v.jsonl 2> $O/r04p_$v.err; rc=$?  # (timing-only variants fail verification: exit 1)
    [ $rc -le 1 ] || { echo BENCH_${v}_FAIL $rc; tail -20 $O/r04p_$v.err; exit 1; }
    line $O/r04p_$v.jsonl $v
  done
done
echo R04P_OK
