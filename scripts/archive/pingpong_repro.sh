#!/bin/bash
# Reproducer for the two-buffer ping-pong form of segment_crc0's row loop (h3c_common.hpp,
# H3C_PINGPONG=1): the same source built at -O3 and at -O1, next to the shipped copy form.
#   bash scripts/pingpong_repro.sh build        # here: variants/lib_pp_o3.so, lib_pp_o1.so
#   bash scripts/pingpong_repro.sh run          # GPU box: bench verify + parity tests per library
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
V=3fs_amd/_lib/variants
if [ "${1:-build}" = build ]; then
  for opt in O3 O1; do
    O=$V/obj/pp_$opt
    mkdir -p $O
    for f in h3c_engine h3c_update h3c_hostfed h3c_updio h3c_formats; do
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -$opt -std=c++17 -fPIC -DH3C_PINGPONG=1 -I include \
        -c 3fs_amd/csrc/$f.hip -o $O/$f.o &
    done
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $V/lib_pp_$(echo $opt | tr O o).so $O/*.o
  done
  exit 0
fi
for v in cur pp_o3 pp_o1; do
  lib=$R/3fs_amd/_lib/libh3c_crc.so
  [ "$v" != cur ] && lib=$R/$V/lib_$v.so
  echo "== $v"
  H3C_LIB_PATH=$lib timeout -k 5 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], 'verified', d['verified'])"
  set +e
  H3C_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -m gpu > gpurun_out/pp_$v.log 2>&1
  rc=$?
  set -e
  tail -n 12 gpurun_out/pp_$v.log
  # test failures (1) are the expected outcome for a miscompiled library; anything else ends the run
  [ $rc -le 1 ] || exit $rc
done
