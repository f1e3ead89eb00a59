#!/bin/bash
# SQ counters of the 4 KiB uniform small-chunk verify for the in-tree library and variants
# (VARIANTS="uni8 ..."): one rocprofv3 --pmc pass per library, outputs under gpurun_out/pmc_<v>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in cur $VARIANTS; do
  lib=$R/3fs_amd/_lib/libh3c_crc.so
  [ "$v" != cur ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
  H3C_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD} \
    -d $R/gpurun_out/pmc${TAG:-}_$v -o pmc --output-format csv -- python3 $R/bench.py --chunks 2097152 --chunk-kib 4 \
    --hostfed-extra-gib 0 --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pmc${TAG:-}_$v.log 2>&1 || { echo PMC_${v}_FAIL; exit 1; }
done
echo PMC_OK
