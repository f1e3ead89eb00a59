#!/bin/bash
# A/B of uniform small-chunk verify: seg_uni_kernel (cur, variants) vs seg_quad_kernel (quad: the
# same library with H3C_DEBUG_FLAGS=4), interleaved on one box; 8 GiB of 4 / 8 KiB chunks.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  for kib in ${SIZES:-4 8}; do
    for v in cur quad $VARIANTS; do
      lib=$R/3fs_amd/_lib/libh3c_crc.so; dbg=0
      [ "$v" = quad ] && dbg=4
      [ "$v" != cur ] && [ "$v" != quad ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
      echo -n "$v ${kib}KiB rep=$rep "
      H3C_DEBUG_FLAGS=$dbg H3C_LIB_PATH=$lib timeout -k 5 120 python bench.py --chunks $((8388608 / kib)) --chunk-kib $kib --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['achieved'], d['roofline']['kernel_avg_us'], d['verified'])" || exit 1
    done
  done
done
