#!/bin/bash
# A/B of the general update path (bench.py --workload updio) between the in-tree library
# and variants built into 3fs_amd/_lib/variants/lib_<name>.so, interleaved on one box
# (host speed differs between boxes, so only same-box comparisons mean anything).
# usage: VARIANTS="old" scripts/ab_updio.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in cur $VARIANTS; do
    lib=$R/3fs_amd/_lib/libh3c_crc.so
    [ "$v" != cur ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
    echo -n "$v rep=$rep "
    H3C_LIB_PATH=$lib timeout -k 5 120 python bench.py --workload updio --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['verified'])" || exit 1
  done
done
