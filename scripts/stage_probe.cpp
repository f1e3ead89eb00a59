// Does the synchronous batch path stage pageable host payloads correctly under
// /opt/rocm's HIP runtime (no torch in the process)?  Null stream and a created stream.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <vector>
#include "../include/h3c_crc.h"
#include "../oracle/crc_oracle.h"
int main() {
  std::mt19937_64 rng(7);
  int bad = 0;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (void *st : {(void *)nullptr, (void *)s}) {
    for (size_t n : {1ul, 4096ul, 65536ul, 1ul << 20, (3ul << 20) + 123}) {
      std::vector<uint8_t> host(n);
      for (auto &c : host) c = (uint8_t)rng();
      h3c_desc d{host.data(), n, 0x1234, 1, H3C_MEM_HOST_PAGEABLE, 0};
      uint8_t t = 0;
      uint32_t v = 0;
      int rc = h3c_batch_create(&d, 1, &t, &v, st);
      uint32_t w = orc_crc32c_sse42(host.data(), n, 0x1234);
      std::printf("stream=%s n=%zu rc=%d got=%08x want=%08x %s\n", st ? "own" : "null", n, rc, v, w,
                  v == w ? "ok" : "BAD");
      bad += v != w;
    }
  }
  return bad ? 1 : 0;
}
