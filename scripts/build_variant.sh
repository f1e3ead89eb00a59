#!/bin/bash
# Build the engine with extra defines into 3fs_amd/_lib/variants/lib_<name>.so (A/B runs).
#   bash scripts/build_variant.sh <name> -DFOO=1 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
name=$1; shift
O=3fs_amd/_lib/variants/obj/$name
mkdir -p $O
for f in h3c_engine h3c_update h3c_hostfed h3c_updio h3c_formats; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -I include -c 3fs_amd/csrc/$f.hip -o $O/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o 3fs_amd/_lib/variants/lib_$name.so $O/*.o
