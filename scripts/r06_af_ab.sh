#!/bin/bash
# Aligned UpdateIO kernel: working tree against the committed kernel (base),
# 4 rotating op tables, same box; then the aligned / config-3 GPU tests and a per-workgroup trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
out=gpurun_out/r06_af_ab.txt
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_updio_aligned.py tests/test_gpu_config3.py tests/test_gpu_updio_fast.py tests/test_gpu_concurrency.py > gpurun_out/r06_af_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r06_af_tests.log; exit 1; }
tail -2 gpurun_out/r06_af_tests.log
run() {  # label, lib, extra args
  H3C_LIB_PATH=$2 timeout -k 10 120 python -u bench.py --workload updio --no-cpu-baseline $3 > gpurun_out/r06_tab.json || exit 1
  python - "$1" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/r06_tab.json"))
r = d["roofline"]
print(f"{sys.argv[1]:22s} ms={d['ms_per_step']} verified={d['verified']} kernel_us={r['kernel_avg_us']} "
      f"redo={sum(d['redo'].values())} branch={d['branch'][:12]}")
PY
}
CUR=$PWD/3fs_amd/_lib/libh3c_crc.so
BASE=$PWD/3fs_amd/_lib/diag/base/libh3c_crc.so
for rep in 1 2 3; do
  run "new t4" $CUR "--updio-tables 4"
  run "base t4" $BASE "--updio-tables 4"
done
cat $out
AF_TABLES=4 H3C_LIB_PATH=$PWD/3fs_amd/_lib/diag/aftrace/libh3c_crc.so timeout -k 10 120 python -u scripts/af_trace.py > gpurun_out/r06_aftrace_new.txt 2>&1 || { echo TRACE_FAIL; tail gpurun_out/r06_aftrace_new.txt; exit 1; }
sed -n "3,13p;26,28p" gpurun_out/r06_aftrace_new.txt
