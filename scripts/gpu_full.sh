#!/bin/bash
# Full GPU pass: smoke, GPU parity tests, bench (all workloads), optional rocprofv3 passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
# every workload line carries its own CPU leg (config 3's updateChecksum case (iv) timing for
# update / updio, the per-call CPU time for sync), except where none is defined for the workload
for w in ${WORKLOADS:-}; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { echo BENCH_${w}_FAIL; exit 1; }
done
if [ -n "$PROFILE" ]; then
  bash scripts/profile_r1.sh > gpurun_out/profile.log 2>&1 || { echo PROF_FAIL; exit 1; }
  python scripts/summarize_prof.py gpurun_out/prof > gpurun_out/prof/summary.json || exit 1
fi
echo ALL_OK
