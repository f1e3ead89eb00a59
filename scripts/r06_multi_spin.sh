#!/bin/bash
# h3c_multi spin-then-block dispatch: the multi GPU tests, then the in-process bench with one and two workers.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multi.py > gpurun_out/r06_spin_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r06_spin_tests.log; exit 1; }
timeout -k 10 200 python -u bench.py --gpus 1 --inproc --devices 0 --steps 20 --warmup 3 > gpurun_out/r06_spin_inproc_0.json 2> gpurun_out/r06_spin_inproc_0.err || { echo INPROC1_FAIL; tail -20 gpurun_out/r06_spin_inproc_0.err; exit 1; }
timeout -k 10 200 python -u bench.py --gpus 2 --inproc --devices 0,0 --steps 20 --warmup 3 > gpurun_out/r06_spin_inproc_00.json 2> gpurun_out/r06_spin_inproc_00.err || { echo INPROC2_FAIL; tail -20 gpurun_out/r06_spin_inproc_00.err; exit 1; }
tail -3 gpurun_out/r06_spin_tests.log; cat gpurun_out/r06_spin_inproc_0.json gpurun_out/r06_spin_inproc_00.json
