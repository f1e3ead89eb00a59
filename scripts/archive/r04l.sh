#!/bin/bash
# same-box sweep of the 4 KiB batch (bench.py --chunks 2097152 --chunk-kib 4) over diag builds, alternating.
# usage: scripts/r04l.sh <variant> [...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
line() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['verified'])"; }
for rep in 1 2; do
  for v in cur "$@"; do
    if [ $v = cur ]; then unset H3C_LIB_PATH; else export H3C_LIB_PATH=$R/3fs_amd/_lib/diag/$v/libh3c_crc.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --chunks 2097152 --chunk-kib 4 --hostfed-extra-gib 0 > $O/r04l_$v.jsonl 2> $O/r04l_$v.err || { echo BENCH_${v}_FAIL; tail -20 $O/r04l_$v.err; exit 1; }
    line $O/r04l_$v.jsonl $v
  done
done
echo R04L_OK
