#!/bin/bash
# SQ counters of the config-3 UpdateIO batch (bench.py --workload updio) for the in-tree library
# and variants (VARIANTS="a b": 3fs_amd/_lib/variants/lib_<v>.so): one rocprofv3 --pmc pass per
# library (8 SQ counters), outputs under gpurun_out/pmc<TAG>_<v>; summarised per kernel by
# scripts/summarize_pmc.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in cur $VARIANTS; do
  lib=$R/3fs_amd/_lib/libh3c_crc.so
  [ "$v" != cur ] && lib=$R/3fs_amd/_lib/variants/lib_$v.so
  H3C_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD} \
    -d $R/gpurun_out/pmc${TAG:-}_$v -o pmc --output-format csv -- python3 $R/bench.py --workload updio \
    --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pmc${TAG:-}_$v.log 2>&1 || { echo PMC_${v}_FAIL; exit 1; }
  python3 $R/scripts/summarize_pmc.py $R/gpurun_out/pmc${TAG:-}_$v > $R/gpurun_out/pmc${TAG:-}_$v.txt || exit 1
done
echo PMC_OK
