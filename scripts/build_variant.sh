#!/bin/bash
# Builds the working tree's engine with extra compile flags into 3fs_amd/_lib/diag/<name>/ for same-box
# A/Bs (H3C_LIB_PATH).  usage: scripts/build_variant.sh <name> [-DFLAG=V ...]
set -e
name=$1; shift
R=$(cd $(dirname $0)/.. && pwd)
O=$R/3fs_amd/_lib/diag/$name
mkdir -p $O/obj
for f in h3c_engine h3c_update h3c_hostfed h3c_updio h3c_formats h3c_multi; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I $R/include "$@" -c $R/3fs_amd/csrc/$f.hip -o $O/obj/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libh3c_crc.so $O/obj/*.o
echo $O/libh3c_crc.so
