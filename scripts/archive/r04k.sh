#!/bin/bash
# same-box A/B of the shipped build against diag variants on the headline verify, the block update and
# the 4 KiB batch (bench.py lines; value, ms per step, kernel average), after the parity tests that cover
# the kernels touched.  usage: scripts/r04k.sh <variant> [...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_update.py -m gpu > $O/r04k_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/r04k_tests.log; exit 1; }
tail -1 $O/r04k_tests.log
line() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['verified'])"; }
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export H3C_LIB_PATH=$lib; else unset H3C_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/r04k_$tag.jsonl 2> $O/r04k_$tag.err || { echo BENCH_${tag}_FAIL; tail -20 $O/r04k_$tag.err; exit 1; }
  line $O/r04k_$tag.jsonl $tag
}
for rep in 1 2; do
  for v in cur "$@"; do
    lib=""; [ $v != cur ] && lib=$R/3fs_amd/_lib/diag/$v/libh3c_crc.so
    run ${v}_verify "$lib" --hostfed-extra-gib 0 || exit 1
    run ${v}_update "$lib" --workload update || exit 1
    run ${v}_small4k "$lib" --chunks 2097152 --chunk-kib 4 --hostfed-extra-gib 0 || exit 1
  done
done
echo R04K_OK
