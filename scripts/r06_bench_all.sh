#!/bin/bash
# Round-6 bench records: the default line (driver form), the in-process multi-engine rehearsal with two
# workers on the one GPU, and the two-rank launcher rehearsal (both ranks on the one GPU).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u bench.py > gpurun_out/r06_bench_default.json 2> gpurun_out/r06_bench_default.err || { echo DEFAULT_FAIL; tail -20 gpurun_out/r06_bench_default.err; exit 1; }
timeout -k 10 200 python -u bench.py --gpus 2 --inproc --devices 0,0 --steps 20 --warmup 3 > gpurun_out/r06_bench_inproc_00.json 2> gpurun_out/r06_bench_inproc_00.err || { echo INPROC_FAIL; tail -20 gpurun_out/r06_bench_inproc_00.err; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --allow-shared-devices --steps 20 --warmup 5 > gpurun_out/r06_bench_n2_shared.json 2> gpurun_out/r06_bench_n2_shared.err || { echo N2_FAIL; tail -20 gpurun_out/r06_bench_n2_shared.err; exit 1; }
echo R06BENCH_OK
