#!/bin/bash
# round 4: fast-branch timing (bench updio) and one traced batch (workgroup step times)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_updio_fast.py > $O/r04b_fast.log 2>&1 || { echo FAST_TESTS_FAIL; tail -40 $O/r04b_fast.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline > $O/r04b_bench_updio.jsonl 2> $O/r04b_bench_updio.err || { echo BENCH_FAIL; tail -20 $O/r04b_bench_updio.err; exit 1; }
H3C_LIB_PATH=$R/3fs_amd/_lib/diag/ftrace/libh3c_crc.so timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --steps 3 --warmup 1 > $O/r04b_trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/r04b_trace.log; exit 1; }
timeout -k 10 60 $R/scripts/graph_probe > $O/r04b_graph_probe.txt 2>&1 || { echo PROBE_FAIL; exit 1; }
echo R04B_OK
tail -1 $O/r04b_bench_updio.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_avg_us'], d['branch'], d['redo'], d['verified'])"
grep "fast wg" $O/r04b_trace.log | tail -8
