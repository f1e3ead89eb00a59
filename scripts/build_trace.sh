#!/bin/bash
# A diagnostics build of the engine with extra -D flags (e.g. -DH3C_FAST_TRACE=1) into
# 3fs_amd/_lib/diag/<name>/libh3c_crc.so; use it with H3C_LIB_PATH.
set -e
name=$1; shift
R=$(cd $(dirname $0)/.. && pwd)
O=$R/3fs_amd/_lib/diag/$name
mkdir -p $O/obj
for f in h3c_engine h3c_update h3c_hostfed h3c_updio h3c_formats; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall "$@" -I $R/include -c $R/3fs_amd/csrc/$f.hip -o $O/obj/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libh3c_crc.so $O/obj/*.o
echo $O/libh3c_crc.so
