#!/bin/bash
# same-box A/B of the UpdateIO headline form: graphs on / off, alternating, 3 runs each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out
for rep in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 300 python -u bench.py --workload updio --no-cpu-baseline --updio-graphs $g > $O/r04j_g$g.jsonl 2> $O/r04j_g$g.err || { echo BENCH_FAIL; tail -20 $O/r04j_g$g.err; exit 1; }
    tail -1 $O/r04j_g$g.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graphs=$g', d['ms_per_step'], d['roofline']['kernel_avg_us'], 'other', d['other_form']['ms_per_step'], d['verified'])"
  done
done
echo R04J_OK
