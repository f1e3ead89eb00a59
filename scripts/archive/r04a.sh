#!/bin/bash
# round 4: the UpdateIO fast branch on the GPU (tests, then the updio bench), the 4 KiB plain-load A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_updio_fast.py tests/test_gpu_updio.py -k "repeated or graph"  > $O/r04a_fast.log 2>&1 || { echo FAST_TESTS_FAIL; tail -40 $O/r04a_fast.log; exit 1; }
timeout -k 10 900 $T tests/test_gpu_updio.py tests/test_gpu_config3.py > $O/r04a_updio.log 2>&1 || { echo UPDIO_TESTS_FAIL; tail -40 $O/r04a_updio.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline > $O/r04a_bench_updio.jsonl 2> $O/r04a_bench_updio.err || { echo BENCH_FAIL; tail -20 $O/r04a_bench_updio.err; exit 1; }
timeout -k 10 300 python -u bench.py --chunks 2097152 --chunk-kib 4 --hostfed-extra-gib 0 --no-cpu-baseline > $O/r04a_bench_small4k.jsonl 2> $O/r04a_bench_small4k.err || { echo SMALL_FAIL; exit 1; }
echo R04A_OK
tail -1 $O/r04a_bench_updio.jsonl
tail -1 $O/r04a_bench_small4k.jsonl
