#!/bin/bash
# does the op order (random chunks per wave vs grouped by chunk) move the fast kernel? (TLB locality)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
for ord in random chunk random chunk; do
  timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --updio-order $ord > $O/r04d_$ord.jsonl 2> $O/r04d_$ord.err || { echo BENCH_FAIL; exit 1; }
  tail -1 $O/r04d_$ord.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ord', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['branch'], d['verified'])"
  H3C_UPD_FAST=1 timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --updio-order $ord > $O/r04d_g_$ord.jsonl 2> $O/r04d_g_$ord.err || { echo BENCH_FAIL; exit 1; }
  tail -1 $O/r04d_g_$ord.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('general $ord', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['branch'], d['verified'])"
done
