#!/bin/bash
# Aligned UpdateIO step A/B over several libraries (uio_aprep_kernel changes; 4 rotating op tables, same box), after the
# aligned / config-3 / fast-branch GPU tests on the working tree.
# usage: scripts/r06_aprep_ab.sh label=lib ...   (lib relative to the repo root)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_aprep_ab.txt
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_updio_aligned.py tests/test_gpu_config3.py tests/test_gpu_updio_fast.py tests/test_gpu_concurrency.py > gpurun_out/r06_af_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06_af_tests.log; exit 1; }
tail -1 gpurun_out/r06_af_tests.log
for rep in 1 2 3; do
  for lv in "$@"; do
    label=${lv%%=*}; lib=$PWD/${lv#*=}
    H3C_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline --updio-tables 4 > gpurun_out/r06_tab.json || exit 1
    python - "$label" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:12s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']} redo={sum(d['redo'].values())}")
PY
  done
done
cat $out
bash scripts/r06_aprep_prof.sh "$@"
