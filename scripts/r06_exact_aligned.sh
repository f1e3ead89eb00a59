#!/bin/bash
# Exact mode on the aligned UpdateIO sub-branch: the aligned / config-3 / fast-branch tests, then the
# config-3 bench in trusted and exact mode (4 rotating tables).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_updio_aligned.py tests/test_gpu_config3.py tests/test_gpu_updio_fast.py tests/test_gpu_updio.py > gpurun_out/r06_exact_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/r06_exact_tests.log; exit 1; }
tail -1 gpurun_out/r06_exact_tests.log
out=gpurun_out/r06_exact_bench.txt
: > $out
for mode in "" "--exact"; do
  timeout -k 10 180 python -u bench.py --workload updio --no-cpu-baseline --updio-tables 4 $mode > gpurun_out/r06_tab.json || exit 1
  python - "updio$mode" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:14s} ms={d['ms_per_step']} verified={d['verified']} branch={d['branch'][:40]} kernel_us={r['kernel_avg_us']} redo={sum(d['redo'].values())}")
PY
done
cat $out
