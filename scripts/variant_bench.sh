#!/bin/bash
# A/B kernel variants (built locally into 3fs_amd/_lib/variants) with bench.py, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
for v in $VARIANTS; do
  for seg in $SEGS; do
    echo -n "$v seg=$seg rep=$rep "
    H3C_LIB_PATH=$R/3fs_amd/_lib/variants/lib_$v.so H3C_SEG_BYTES=$seg timeout -k 5 120 python bench.py --no-cpu-baseline --steps 30 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['achieved'], d['roofline']['kernel_avg_us'], d['verified'])" || exit 1
  done
done
done
