#!/bin/bash
# The whole GPU test suite, then the round-6 profile pass; each step under its own time limit, stopping at
# the first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06i_gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/r06h_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06i_gpu_tests.log
./scripts/r06_prof.sh || exit 1
