#!/bin/bash
# Per-launch durations of uio_afused_kernel (rocprofv3 kernel trace), working tree vs base, 4 rotating tables.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for v in new base; do
  lib=$PWD/3fs_amd/_lib/libh3c_crc.so; [ $v = base ] && lib=$PWD/3fs_amd/_lib/diag/base/libh3c_crc.so
  H3C_LIB_PATH=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$v -o kt -- python3 -u bench.py --workload updio --no-cpu-baseline --updio-tables 4 > gpurun_out/kt_$v.log 2>&1 || { echo FAIL $v; tail gpurun_out/kt_$v.log; exit 1; }
  f=$(find gpurun_out/kt_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python3 scripts/kseq.py $f uio_afused_kernel 4 2
done
