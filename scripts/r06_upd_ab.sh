#!/bin/bash
# Block-update path (upd_fused_kernel) A/B, 4 rotating write tables, same box; the block-update GPU tests first.
# usage: scripts/r06_upd_ab.sh label=lib ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_upd_ab.txt
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_update.py tests/test_gpu_update_scratch.py > gpurun_out/r06_upd_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06_upd_tests.log; exit 1; }
tail -1 gpurun_out/r06_upd_tests.log
for rep in 1 2 3; do
  for lv in "$@"; do
    label=${lv%%=*}; lib=$PWD/${lv#*=}
    H3C_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --workload update --no-cpu-baseline --update-tables 4 > gpurun_out/r06_upd.json || exit 1
    python - "$label" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r06_upd.json") if l.startswith("{")][0])
r = d["roofline"]
print(f"{sys.argv[1]:8s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']}")
PY
  done
done
cat $out
