#!/bin/bash
# Builds the engine of a git revision (default HEAD) into 3fs_amd/_lib/diag/<name>/ for same-box A/Bs
# against the working tree (H3C_LIB_PATH).  usage: scripts/build_head_variant.sh <name> [rev]
set -e
name=$1; rev=${2:-HEAD}
R=$(cd $(dirname $0)/.. && pwd)
T=$(mktemp -d)
mkdir -p $T/csrc $T/include
for f in $(git -C $R ls-tree --name-only $rev 3fs_amd/csrc/ include/); do git -C $R show $rev:$f > $T/${f#3fs_amd/}; done
O=$R/3fs_amd/_lib/diag/$name
mkdir -p $O/obj
for f in h3c_engine h3c_update h3c_hostfed h3c_updio h3c_formats; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I $T/include -c $T/csrc/$f.hip -o $O/obj/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libh3c_crc.so $O/obj/*.o
rm -rf $T
echo $O/libh3c_crc.so
