#!/bin/bash
# Small-chunk kernel vs the general segment kernel (H3C_DEBUG_FLAGS=2) across chunk sizes,
# 8 GiB per run, to place the small-path threshold.  usage: scripts/ab_small_path.sh [KiB...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for kib in ${@:-4 8 16 32 64}; do
  for f in 0 2; do
    echo -n "${kib}KiB flags=$f "
    H3C_DEBUG_FLAGS=$f timeout -k 5 120 python bench.py --chunks $((8388608 / kib)) --chunk-kib $kib --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['achieved'], d['ms_per_step'], d['verified'])" || exit 1
  done
done
