#!/bin/bash
# GPU session script (round 1, first pass). Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "Marketing Name|gfx950" > gpurun_out/device.txt
lscpu > gpurun_out/lscpu.txt 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
