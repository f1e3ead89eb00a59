// Phased read-modify-write probe for the config-3 update pattern (VERDICT r2 "do this" #4):
// per 4 KiB block write, read the payload (sequential over the batch) and the old slot (random
// 4 KiB in a 4 GiB chunk set), then write the payload into the slot.  The reads alone take
// ~123 us and the writes alone ~72-84 us (profiles/r01_update_pattern_ceiling.txt,
// r02_store_policy.txt), but mixed they take 232-247 us.  This asks whether separating the
// two in time wins any of that back:
//   mixed      each wave reads its INF blocks and writes them back, block after block (today)
//   wg-phased  every wave of a workgroup reads INF blocks, workgroup barrier, all write, barrier
//   grid-phased  the same with a grid-wide barrier between the read and write halves of every
//              round (one workgroup per CU, all resident; spins are bounded: a run whose barrier
//              gives up is reported as void)
// Stores: nontemporal (what the kernels use) and plain.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/rmwphase scripts/rmwphase.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u __attribute__((address_space(1))) *gv4p;

enum { kMixed = 0, kWg = 1, kGrid = 2 };

__device__ __forceinline__ void st(v4u v, char *p, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, (gv4p)p);
  else
    *(gv4p)p = v;
}

// Grid barrier on a monotonically increasing counter: arrival k of round r waits for the count
// to reach (r + 1) * gridDim.x.  Bounded: gives up (and flags) after ~2^22 polls.
__device__ __forceinline__ void grid_sync(unsigned *ctr, unsigned target, unsigned *fail) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(ctr, 1u);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        atomicExch(fail, 1u);
        break;
      }
    }
    __threadfence();
  }
  __syncthreads();
}

template <int MODE, int INF>
__global__ __launch_bounds__(1024) void rmw(const char *pay, char *region, const uint32_t *slot, uint32_t n,
                                            uint32_t *out, bool nt, unsigned *ctr, unsigned *fail) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x / 64;
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * wpb;
  v4u acc = {0, 0, 0, 0};
  if (MODE == kMixed) {
    const uint32_t lo = (uint32_t)(gw * n / nw), hi = (uint32_t)((gw + 1) * n / nw);
    for (uint32_t i = lo; i < hi; i += INF) {
      v4u a[INF][4], b[INF][4];
#pragma unroll
      for (int f = 0; f < INF; ++f) {
        const uint32_t k = min(i + f, hi - 1);
        const char *p = pay + (uint64_t)k * 4096 + 16 * lane;
        const char *s = region + (uint64_t)slot[k] * 4096 + 16 * lane;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[f][u] = __builtin_nontemporal_load((gv4p)(p + 1024 * u));
          b[f][u] = __builtin_nontemporal_load((gv4p)(s + 1024 * u));
        }
      }
#pragma unroll
      for (int f = 0; f < INF; ++f) {
        if (i + f >= hi) break;
        char *s = region + (uint64_t)slot[i + f] * 4096 + 16 * lane;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc ^= b[f][u];
          st(a[f][u], s + 1024 * u, nt);
        }
      }
    }
  } else {
    // rounds: round r, wave w handles blocks (r * nw + w) * INF + f
    const uint32_t per_round = (uint32_t)nw * INF;
    const uint32_t rounds = (n + per_round - 1) / per_round;
    for (uint32_t r = 0; r < rounds; ++r) {
      v4u a[INF][4], b[INF][4];
      const uint32_t i0 = (uint32_t)((r * nw + gw) * INF);
#pragma unroll
      for (int f = 0; f < INF; ++f) {
        const uint32_t k = min(i0 + f, n - 1);
        const char *p = pay + (uint64_t)k * 4096 + 16 * lane;
        const char *s = region + (uint64_t)slot[k] * 4096 + 16 * lane;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[f][u] = __builtin_nontemporal_load((gv4p)(p + 1024 * u));
          b[f][u] = __builtin_nontemporal_load((gv4p)(s + 1024 * u));
        }
      }
#pragma unroll
      for (int f = 0; f < INF; ++f)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= b[f][u];
      if (MODE == kWg)
        __syncthreads();
      else
        grid_sync(ctr, (2 * r + 1) * gridDim.x, fail);
#pragma unroll
      for (int f = 0; f < INF; ++f) {
        if (i0 + f >= n) break;
        char *s = region + (uint64_t)slot[i0 + f] * 4096 + 16 * lane;
#pragma unroll
        for (int u = 0; u < 4; ++u) st(a[f][u], s + 1024 * u, nt);
      }
      if (MODE == kWg)
        __syncthreads();
      else
        grid_sync(ctr, (2 * r + 2) * gridDim.x, fail);
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

int main() {
  const uint32_t n = 100000, nslots = 64u * 16384u;  // 64 x 64 MiB chunks of 4 KiB slots
  char *pay, *region;
  uint32_t *slot, *o;
  unsigned *ctr, *fail;
  hipMalloc(&pay, (size_t)n * 4096);
  hipMalloc(&region, (size_t)nslots * 4096);
  hipMalloc(&slot, 4ull * n);
  hipMalloc(&o, 4);
  hipMalloc(&ctr, 4);
  hipMalloc(&fail, 4);
  hipMemset(pay, 1, (size_t)n * 4096);
  hipMemset(region, 2, (size_t)nslots * 4096);
  hipMemset(fail, 0, 4);
  std::vector<uint32_t> hs(n);
  std::mt19937 rng(20250629);
  for (auto &x : hs) x = rng() % nslots;
  hipMemcpy(slot, hs.data(), 4ull * n, hipMemcpyHostToDevice);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char *name, auto launch) {
    for (int w = 0; w < 3; ++w) {
      hipMemsetAsync(ctr, 0, 4);
      launch();
    }
    hipDeviceSynchronize();
    const int it = 20;
    float total = 0;
    for (int k = 0; k < it; ++k) {  // the barrier counter is reset outside the timed launch
      hipMemsetAsync(ctr, 0, 4);
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      total += ms;
    }
    unsigned f = 0;
    hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
    const double us = total * 1e3 / it;
    printf("%-46s %8.1f us  %8.1f GB/s%s\n", name, us, n * 12288.0 / (us * 1e-6) / 1e9, f ? "  (barrier gave up: void)" : "");
    fflush(stdout);
    hipMemset(fail, 0, 4);
  };
  for (int ntv : {1, 0}) {
    const bool nt = ntv;
    const char *sn = nt ? "nt" : "plain";
    char nm[96];
#define RUN(MODE, INF, WPC, LABEL)                                                                   \
  snprintf(nm, sizeof nm, "%-12s %2d w/CU inf%d %s", LABEL, WPC, INF, sn);                            \
  run(nm, [&] { rmw<MODE, INF><<<dim3(cus), dim3(64 * (WPC))>>>(pay, region, slot, n, o, nt, ctr, fail); });
    RUN(kMixed, 1, 16, "mixed")
    RUN(kMixed, 1, 8, "mixed")
    RUN(kWg, 1, 16, "wg-phased")
    RUN(kWg, 2, 16, "wg-phased")
    RUN(kWg, 2, 8, "wg-phased")
    RUN(kWg, 4, 8, "wg-phased")
    RUN(kGrid, 2, 16, "grid-phased")
    RUN(kGrid, 4, 8, "grid-phased")
  }
  return 0;
}
