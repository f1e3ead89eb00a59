#!/bin/bash
# A/B of small-chunk verify (seg_small_kernel) between the in-tree library and variants in
# 3fs_amd/_lib/variants/lib_<name>.so, interleaved on one box: 8 GiB of 4 KiB and of 8 KiB chunks.
# usage: VARIANTS="smallold" scripts/ab_small.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  for kib in ${SIZES:-4 8}; do
    for v in cur $VARIANTS; do
      lib=$R/3fs_amd/_lib/libh3c_crc.so
      [ "$v" != cur ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
      echo -n "$v ${kib}KiB rep=$rep "
      H3C_LIB_PATH=$lib timeout -k 5 120 python bench.py --chunks $((8388608 / kib)) --chunk-kib $kib --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['achieved'], d['roofline']['kernel_avg_us'], d['verified'])" || exit 1
    done
  done
done
