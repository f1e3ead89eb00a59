#!/bin/bash
# Same-box A/B of library variants (scripts/build_variant.sh <name> -D...) on one bench.py workload,
# interleaved over reps; prints ms_per_step and the roofline kernel's average per run.
# usage: VARIANTS="a b" WORKLOAD=updio REPS=3 ARGS="--steps 60 --warmup 20" scripts/ab_variants.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
W=${WORKLOAD:-updio}; A=${ARGS:-}
for rep in $(seq 1 ${REPS:-3}); do
  for v in cur $VARIANTS; do
    lib=$R/3fs_amd/_lib/libh3c_crc.so
    [ "$v" != cur ] && lib=$R/3fs_amd/_lib/diag/$v/libh3c_crc.so
    echo -n "$v rep=$rep "
    H3C_LIB_PATH=$lib timeout -k 5 150 python bench.py --workload $W --no-cpu-baseline $A 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']
print(d['ms_per_step'], d['value'], d['verified'], r.get('kernel'), r.get('kernel_avg_us'), r.get('frac'))" || exit 1
  done
done
