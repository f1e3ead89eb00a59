#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for v in $VARIANTS; do
  echo -n "$v "
  H3C_LIB_PATH=$R/3fs_amd/_lib/variants/lib_$v.so timeout -k 5 120 python bench.py --workload update --no-cpu-baseline --steps 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['achieved'], d['verified'])"
done
