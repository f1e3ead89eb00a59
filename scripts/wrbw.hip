// Store-policy probe for the partial-update pattern (BASELINE config 3): the rmw probe of
// rmwbw.hip (payload read, random 4 KiB slot read, payload written into the slot) and its
// write-only leg, with the write issued as a nontemporal store, a plain store, or a plain
// global_store_dwordx4 carrying the sc0 / sc1 / nt cache-policy bits.  A question the round-1
// probe left open: random 4 KiB nontemporal writes ran at 4.9 TB/s, below the 6.0-6.2 TB/s
// the microarchitecture guide records for plain stores of random rows.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/wrbw scripts/wrbw.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u __attribute__((address_space(1))) *gv4p;

template <int POL>
__device__ __forceinline__ void st16(char *p, v4u w) {
  if constexpr (POL == 0) {
    __builtin_nontemporal_store(w, (gv4p)p);
  } else if constexpr (POL == 1) {
    *(gv4p)p = w;
  } else if constexpr (POL == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(w) : "memory");
  } else if constexpr (POL == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(w) : "memory");
  }
}

// MODE bit0: read payload, bit1: read slot, bit2: write slot.
template <int MODE, int POL>
__global__ __launch_bounds__(1024) void rmw(const char *pay, char *region, const uint32_t *slot, uint32_t n,
                                            uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint32_t lo = (uint32_t)(gw * n / nw), hi = (uint32_t)((gw + 1) * n / nw);
  v4u acc = {0, 0, 0, 0};
  for (uint32_t i = lo; i < hi; ++i) {
    v4u a[4], b[4];
    const char *p = pay + (uint64_t)i * 4096 + 16 * lane;
    char *s = region + (uint64_t)slot[i] * 4096 + 16 * lane;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (MODE & 1) a[u] = __builtin_nontemporal_load((gv4p)(p + 1024 * u));
      if (MODE & 2) b[u] = __builtin_nontemporal_load((gv4p)(s + 1024 * u));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (MODE & 2) acc ^= b[u];
      if (MODE & 4) {
        v4u w = (MODE & 1) ? a[u] : v4u{lane, i, 0, 0};
        st16<POL>(s + 1024 * u, w);
      }
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

int main() {
  const uint32_t n = 100000, nslots = 64u * 16384u;  // 64 x 64 MiB chunks of 4 KiB slots
  char *pay, *region;
  uint32_t *slot, *o;
  hipMalloc(&pay, (size_t)n * 4096);
  hipMalloc(&region, (size_t)nslots * 4096);
  hipMalloc(&slot, 4ull * n);
  hipMalloc(&o, 4);
  hipMemset(pay, 1, (size_t)n * 4096);
  hipMemset(region, 2, (size_t)nslots * 4096);
  std::vector<uint32_t> hs(n);
  std::mt19937 rng(20250629);
  for (auto &x : hs) x = rng() % nslots;
  hipMemcpy(slot, hs.data(), 4ull * n, hipMemcpyHostToDevice);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char *name, double bytes_per_block, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipDeviceSynchronize();
    const int it = 20;
    hipEventRecord(a);
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / it;
    printf("%-44s %8.1f us  %8.1f GB/s\n", name, us, n * bytes_per_block / (us * 1e-6) / 1e9);
  };
  const char *pol[] = {"nontemporal", "plain", "sc1", "sc0 sc1", "sc0 sc1 nt"};
  for (int rep = 0; rep < 2; ++rep)
    for (int wpc : {8, 16}) {
      char nm[96];
#define P(POL)                                                                                           \
  snprintf(nm, sizeof nm, "[%2d w/CU] write only  %s", wpc, pol[POL]);                                   \
  run(nm, 4096, [&] { rmw<4, POL><<<dim3(cus), dim3(64 * wpc)>>>(pay, region, slot, n, o); });           \
  snprintf(nm, sizeof nm, "[%2d w/CU] rmw         %s", wpc, pol[POL]);                                   \
  run(nm, 12288, [&] { rmw<7, POL><<<dim3(cus), dim3(64 * wpc)>>>(pay, region, slot, n, o); });
      P(0) P(1) P(2) P(3) P(4)
    }
  return 0;
}
