#!/bin/bash
# fast-branch tests, then an A/B of the shipped build against diag variants (bench updio, alternating),
# then a kernel trace of the shipped build.  usage: scripts/r04h.sh <variant> [<variant> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_updio_fast.py tests/test_gpu_update.py > $O/r04h_fast.log 2>&1 || { echo FAST_TESTS_FAIL; tail -40 $O/r04h_fast.log; exit 1; }
grep -c PASSED $O/r04h_fast.log
line() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['other_form']['ms_per_step'], d['branch'][:4], d['verified'])"; }
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline > $O/r04h_cur.jsonl 2> $O/r04h_cur.err || { echo BENCH_FAIL; tail -20 $O/r04h_cur.err; exit 1; }
  line $O/r04h_cur.jsonl cur
  for v in "$@"; do
    H3C_LIB_PATH=$R/3fs_amd/_lib/diag/$v/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline > $O/r04h_$v.jsonl 2> $O/r04h_$v.err || { echo BENCH_${v}_FAIL; tail -20 $O/r04h_$v.err; exit 1; }
    line $O/r04h_$v.jsonl $v
  done
done
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/r04h_kt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 $R/bench.py --workload updio --no-cpu-baseline --steps 20 --warmup 2 > $OUT.log 2>&1 || { echo KT_FAIL; exit 1; }
python3 $R/scripts/kstats.py $OUT/kt_kernel_stats.csv | grep -E "uio_|csort|piece" || true
python3 $R/scripts/ktimeline.py $OUT/kt_kernel_trace.csv uio_zero_kernel 24 | tail -3 | cut -c1-200
echo R04H_OK
