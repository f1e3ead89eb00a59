// C++ mirror test: h3c::ChecksumInfo (include/h3c_checksum_info.hpp) vs the CPU oracle.
// usage: checksum_info_test cpu|gpu     (gpu mode needs a HIP device)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/h3c_checksum_info.hpp"
#include "../../oracle/crc_oracle.h"

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                \
    }                                                         \
  } while (0)

using h3c::ChecksumInfo;
using h3c::ChecksumType;

static void cpu_tests() {
  const char *a = "hello ", *b = "3fs world";
  const size_t na = std::strlen(a), nb = std::strlen(b);
  std::string ab = std::string(a) + b;
  ChecksumInfo x{ChecksumType::CRC32C, orc_crc32c_table((const uint8_t *)a, na, ~0U)};
  CHECK(x.combine({ChecksumType::CRC32C, orc_crc32c_table((const uint8_t *)b, nb, ~0U)}, nb) == 0);
  CHECK(x.value == orc_crc32c_table((const uint8_t *)ab.data(), ab.size(), ~0U));
  ChecksumInfo y{ChecksumType::CRC32, orc_crc32_table((const uint8_t *)a, na, ~0U)};
  CHECK(y.combine({ChecksumType::CRC32, orc_crc32_table((const uint8_t *)b, nb, ~0U)}, nb) == 0);
  CHECK(y.value == orc_crc32_table((const uint8_t *)ab.data(), ab.size(), ~0U));
  ChecksumInfo n;
  CHECK(n.combine({ChecksumType::CRC32C, 7}, 3) == 0 && n == (ChecksumInfo{ChecksumType::CRC32C, 7}));
  ChecksumInfo z{ChecksumType::CRC32C, 5};
  CHECK(z.combine({ChecksumType::CRC32C, 9}, 0) == 0 && z.value == 5);
  CHECK(z.combine({ChecksumType::CRC32, 9}, 4) == 4080);
  // TestFolly.cc:9-18
  uint32_t c1 = orc_crc32c_table((const uint8_t *)"hello", 5, 0), c2 = orc_crc32c_table((const uint8_t *)"world", 5, 0);
  CHECK(h3c_crc32c_combine(c1, c2, 5) == orc_crc32c_table((const uint8_t *)"world", 5, c1));
}

static void gpu_tests() {
  std::mt19937_64 rng(7);
  const size_t n = (3u << 20) + 123;
  std::vector<uint8_t> host(n);
  for (auto &c : host) c = (uint8_t)rng();
  uint8_t *dev = nullptr;
  CHECK(hipMalloc(&dev, n) == hipSuccess);
  CHECK(hipMemcpy(dev, host.data(), n, hipMemcpyHostToDevice) == hipSuccess);
  int rc = -1;
  ChecksumInfo g = ChecksumInfo::create(ChecksumType::CRC32C, dev + 3, n - 3, ~0U, H3C_MEM_DEVICE, nullptr, &rc);
  CHECK(rc == 0);
  CHECK(g == (ChecksumInfo{ChecksumType::CRC32C, orc_crc32c_sse42(host.data() + 3, n - 3, ~0U)}));
  ChecksumInfo h = ChecksumInfo::create(ChecksumType::CRC32C, host.data(), n, 0x1234, H3C_MEM_HOST_PAGEABLE);
  CHECK(h.value == orc_crc32c_sse42(host.data(), n, 0x1234));
  ChecksumInfo i = ChecksumInfo::create(ChecksumType::CRC32, dev, 1000);
  CHECK(i.type == ChecksumType::CRC32 && i.value == orc_crc32_table(host.data(), 1000, ~0U));
  CHECK(ChecksumInfo::create(ChecksumType::NONE, dev, 10) == ChecksumInfo{});
  CHECK((ChecksumInfo::create(ChecksumType::CRC32C, nullptr, 10) == ChecksumInfo{}));
  CHECK((ChecksumInfo::create(ChecksumType::CRC32C, nullptr, 0) == ChecksumInfo{ChecksumType::CRC32C, ~0U}));
  // split + combine == whole (Common.h:191 semantics)
  ChecksumInfo p = ChecksumInfo::create(ChecksumType::CRC32C, dev, 1 << 20);
  ChecksumInfo q = ChecksumInfo::create(ChecksumType::CRC32C, dev + (1 << 20), n - (1 << 20));
  CHECK(p.combine(q, n - (1 << 20)) == 0);
  CHECK(p.value == orc_crc32c_sse42(host.data(), n, ~0U));
  std::vector<h3c_desc> ds;
  for (int k = 0; k < 64; ++k) ds.push_back(h3c_desc{dev + k * 4096, 4096 + (uint64_t)k, ~0U, 1, H3C_MEM_DEVICE, 0});
  std::vector<ChecksumInfo> out;
  CHECK(ChecksumInfo::createBatch(ds, out) == 0);
  for (int k = 0; k < 64; ++k) CHECK(out[k].value == orc_crc32c_sse42(host.data() + k * 4096, 4096 + k, ~0U));
  (void)hipFree(dev);
}

int main(int argc, char **argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  cpu_tests();
  if (gpu) gpu_tests();
  std::printf("%s checksum_info_test %s\n", fails ? "FAILED" : "OK", gpu ? "gpu" : "cpu");
  return fails ? 1 : 0;
}
