#!/bin/bash
# rocprofv3 kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes for one bench workload.
# usage: scripts/profile.sh <workload> <tag> [extra bench args...]   (outputs under gpurun_out/prof_<tag>)
set -o pipefail
W=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload $W --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $B --steps ${KT_STEPS:-20} --warmup ${KT_WARMUP:-2} > $OUT/kt_bench.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/fetch_bench.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/write_bench.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python3 $R/scripts/summarize_kernels.py $OUT > $OUT/summary.txt || exit 1
echo PROF_OK
