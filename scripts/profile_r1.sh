#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE / WRITE_SIZE / LDS) for bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --hostfed-extra-gib 0 --steps 20 --warmup 2 > $OUT/kt_bench.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $R/bench.py --no-cpu-baseline --hostfed-extra-gib 0 --steps 3 --warmup 1 > $OUT/fetch_bench.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $R/bench.py --no-cpu-baseline --hostfed-extra-gib 0 --steps 3 --warmup 1 > $OUT/write_bench.log 2>&1 || { echo WRITE_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/lds -o lds --output-format csv -- python3 $R/bench.py --no-cpu-baseline --hostfed-extra-gib 0 --steps 3 --warmup 1 > $OUT/lds_bench.log 2>&1 || { echo LDS_FAIL; exit 1; }
find $OUT -name "*.csv" | head -50
echo PROF_OK
