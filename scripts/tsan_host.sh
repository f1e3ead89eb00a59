#!/bin/bash
# Host-side ThreadSanitizer run of the engine's shared host state (lease pools, coalescing
# queue, aux streams, caches, profiling records): the library's host code and
# tests/cpp/tsan_stress.cpp instrumented with -fsanitize=thread (GPU code built normally: GPU
# sanitizers and xnack are not available on the pool).  Build here, run on the GPU box:
#   bash scripts/tsan_host.sh build
#   TSAN_OPTIONS="suppressions=scripts/tsan.supp halt_on_error=0" ./scripts/tsan_stress 16 12
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
if [ "${1:-build}" = build ]; then
  O=/tmp/h3c_tsan_obj
  mkdir -p $O
  for f in h3c_engine h3c_update h3c_hostfed h3c_updio h3c_formats; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -Xarch_host -fsanitize=thread \
      -I include -c 3fs_amd/csrc/$f.hip -o $O/$f.o &
  done
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -Xarch_host -fsanitize=thread -I include -c tests/cpp/tsan_stress.cpp \
    -o $O/tsan_stress.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=thread -fno-gpu-sanitize -o scripts/tsan_stress $O/*.o -lpthread
fi
