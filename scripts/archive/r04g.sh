#!/bin/bash
# fast-branch tests + bench + kernel trace timeline + tail trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_updio_fast.py tests/test_gpu_update.py > $O/r04g_fast.log 2>&1 || { echo FAST_TESTS_FAIL; tail -40 $O/r04g_fast.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline > $O/r04g_bench_updio.jsonl 2> $O/r04g_bench_updio.err || { echo BENCH_FAIL; tail -20 $O/r04g_bench_updio.err; exit 1; }
tail -1 $O/r04g_bench_updio.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_avg_us'], d['branch'], d['verified'])"
H3C_LIB_PATH=$R/3fs_amd/_lib/diag/ftrace/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --steps 3 --warmup 1 > $O/r04g_trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/r04g_trace.log; exit 1; }
grep "tail tile" $O/r04g_trace.log | tail -4
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/r04g_kt_fast
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 $R/bench.py --workload updio --no-cpu-baseline --steps 20 --warmup 2 > $OUT.log 2>&1 || { echo KT_FAIL; exit 1; }
python3 $R/scripts/kstats.py $OUT/kt_kernel_stats.csv | grep -E "uio_|csort|piece" || true
echo R04G_OK
