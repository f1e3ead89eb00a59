// C++ mirror test: h3c::ChecksumInfo (include/h3c_checksum_info.hpp) vs the CPU oracle.
// usage: checksum_info_test cpu|gpu     (gpu mode needs a HIP device)
#include <hip/hip_runtime.h>

#include <algorithm>
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
  // serde (TestCommonStruct.cc:46-56): 1 + 1 + 4 bytes, round trip
  {
    ChecksumInfo ser{ChecksumType::CRC32, 0xff};
    const std::string out = ser.serialize();
    CHECK(out.size() == 1 + 1 + 4);
    ChecksumInfo des;
    CHECK(ChecksumInfo::deserialize(des, out.data(), out.size()) == 0 && des == ser);
    CHECK(ChecksumInfo::deserialize(des, out.data(), 3) != 0);
  }
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
  CHECK((ChecksumInfo::create(ChecksumType::CRC32C, (const uint8_t *)nullptr, 10) == ChecksumInfo{}));
  CHECK((ChecksumInfo::create(ChecksumType::CRC32C, (const uint8_t *)nullptr, 0) == ChecksumInfo{ChecksumType::CRC32C, ~0U}));
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
  // Repeated synchronous calls under /opt/rocm's runtime (the storage service's runtime):
  // pageable and device payloads, null and own streams.  Guards the scratch-allocation
  // path (hipMallocAsync pools handed kernels stale bytes here; profiles/r01b_hip_alloc_coherence.txt).
  hipStream_t own;
  CHECK(hipStreamCreate(&own) == hipSuccess);
  for (int it = 0; it < 200; ++it) {
    const size_t len = 1 + rng() % (1u << 20);
    const size_t off = rng() % 64;
    void *st = (it & 1) ? (void *)own : nullptr;
    const bool host_src = (it & 2) != 0;
    h3c_desc d{host_src ? (const void *)(host.data() + off) : (const void *)(dev + off), len, ~0U, 1,
               (uint8_t)(host_src ? H3C_MEM_HOST_PAGEABLE : H3C_MEM_DEVICE), 0};
    uint8_t t = 0;
    uint32_t v = 0;
    CHECK(h3c_batch_create(&d, 1, &t, &v, st) == 0);
    CHECK(v == orc_crc32c_sse42(host.data() + off, len, ~0U));
  }
  // h3c_update_ios from C++: appends and overwrites, then the chunk checksum equals a fresh CRC.
  {
    const uint32_t cs = 1u << 20;
    uint8_t *chunk = nullptr, *pay = nullptr;
    CHECK(hipMalloc(&chunk, cs) == hipSuccess);
    CHECK(hipMalloc(&pay, 64 * 8192) == hipSuccess);
    std::vector<uint8_t> model(cs, 0), hp(64 * 8192);
    for (auto &c : hp) c = (uint8_t)rng();
    CHECK(hipMemcpy(pay, hp.data(), hp.size(), hipMemcpyHostToDevice) == hipSuccess);
    h3c_chunk_state cst{(uint64_t)(uintptr_t)chunk, cs, 0, 0, 1, {0, 0, 0}};
    std::vector<h3c_update_io> ios;
    uint32_t size = 0;
    for (int k = 0; k < 64; ++k) {
      const uint32_t len = 1 + rng() % 8192;
      const uint32_t o = (k % 3 == 0 || size == 0) ? size : (uint32_t)(rng() % size);
      const uint8_t *p = hp.data() + k * 8192;
      ios.push_back(h3c_update_io{(uint64_t)(uintptr_t)(pay + k * 8192), 0, o, len, orc_crc32c_sse42(p, len, ~0U), 1,
                                  H3C_UPD_WRITE, 0, 0, 0});
      std::memcpy(model.data() + o, p, len);
      size = std::max(size, o + len);
    }
    std::vector<h3c_update_result> res(ios.size());
    CHECK(h3c_update_ios(H3C_TYPE_CRC32C, &cst, 1, ios.data(), (uint32_t)ios.size(), res.data(), 0, own) == 0);
    for (auto &r : res) CHECK(r.status == 0);
    CHECK(cst.size == size && cst.type == 1);
    CHECK(cst.value == orc_crc32c_sse42(model.data(), size, ~0U));
    CHECK(res.back().value == cst.value);
    (void)hipFree(chunk);
    (void)hipFree(pay);
  }
  (void)hipStreamDestroy(own);
  (void)hipFree(dev);
}

int main(int argc, char **argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  cpu_tests();
  if (gpu) gpu_tests();
  std::printf("%s checksum_info_test %s\n", fails ? "FAILED" : "OK", gpu ? "gpu" : "cpu");
  return fails ? 1 : 0;
}
