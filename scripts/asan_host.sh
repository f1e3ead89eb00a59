#!/bin/bash
# Host-side AddressSanitizer run of the engine (GPU code is built normally: GPU ASan and
# xnack are not available on the pool).  Builds an ASan variant of libh3c_crc.so and the C++
# storage-path test against it (build here, run the binary on the GPU box):
#   bash scripts/asan_host.sh build
#   ASAN_OPTIONS=detect_leaks=0 ./scripts/storage_path_test_asan gpu
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
if [ "${1:-build}" = build ]; then
  mkdir -p 3fs_amd/_lib/variants
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -Xarch_host -fsanitize=address \
    -Xarch_host -fno-omit-frame-pointer -I include -o 3fs_amd/_lib/variants/lib_asan.so \
    3fs_amd/csrc/h3c_engine.hip 3fs_amd/csrc/h3c_update.hip 3fs_amd/csrc/h3c_hostfed.hip \
    3fs_amd/csrc/h3c_updio.hip 3fs_amd/csrc/h3c_formats.hip
  make -C oracle -s
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -Xarch_host -fsanitize=address -I include -o scripts/storage_path_test_asan \
    tests/cpp/storage_path_test.cpp -L3fs_amd/_lib/variants -l:lib_asan.so -Loracle/build -loracle \
    -Wl,-rpath,'$ORIGIN/../3fs_amd/_lib/variants' -Wl,-rpath,'$ORIGIN/../oracle/build'
fi
