// Latency / throughput probe for the update path's link hash (upd_tlink_kernel): 100k
// random slot keys inserted into a 256K-entry table by one thread each, with different
// atomic forms.  Prints the average kernel time per form (hipEvents, 50 reps).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/atomic_probe scripts/atomic_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t hsh(uint32_t key, uint32_t mask) { return (key * 0x9E3779B1u >> 7) & mask; }

// MODE 0: load + store only; 1: 64-bit CAS (returning); 2: 32-bit CAS (returning);
// 3: 64-bit atomicMax, result unused; 4: 32-bit atomicExch (returning); 5: plain 64-bit store
template <int MODE>
__global__ __launch_bounds__(256) void ins(const uint32_t *__restrict__ keys, uint32_t n, unsigned long long *tab,
                                           uint32_t mask, uint32_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = keys[i];
  uint32_t h = hsh(key, mask);
  uint32_t r = 0;
  if (MODE == 1) {
    unsigned long long e = ~0ull;
    for (;;) {
      const uint32_t ek = (uint32_t)(e >> 32);
      if (ek == kNone || ek == key) {
        const unsigned long long got = atomicCAS(&tab[h], e, ((unsigned long long)key << 32) | i);
        if (got == e) break;
        e = got;
      } else {
        h = (h + 1) & mask;
        e = ~0ull;
      }
    }
    r = (uint32_t)e;
  } else if (MODE == 2) {
    uint32_t *t32 = reinterpret_cast<uint32_t *>(tab);
    for (;;) {
      const uint32_t k = atomicCAS(&t32[h], kNone, key);
      if (k == kNone || k == key) break;
      h = (h + 1) & mask;
    }
    r = h;
  } else if (MODE == 3) {
    atomicMax(&tab[h], ((unsigned long long)key << 32) | i);
  } else if (MODE == 4) {
    r = atomicExch(reinterpret_cast<uint32_t *>(tab) + h, i);
  } else if (MODE == 5) {
    tab[h] = ((unsigned long long)key << 32) | i;
  }
  out[i] = r;
}

int main() {
  const uint32_t n = 100000, slots = 1u << 20, cap = 1u << 18;
  std::mt19937_64 rng(5);
  std::vector<uint32_t> keys(n);
  for (auto &k : keys) k = (uint32_t)(rng() % slots);
  uint32_t *dk, *dout;
  unsigned long long *tab;
  CK(hipMalloc(&dk, 4ull * n));
  CK(hipMalloc(&dout, 4ull * n));
  CK(hipMalloc(&tab, 8ull * cap));
  CK(hipMemcpy(dk, keys.data(), 4ull * n, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char *names[] = {"load+store only", "64-bit CAS (returning)", "32-bit CAS (returning)",
                         "64-bit atomicMax (no return)", "32-bit atomicExch (returning)", "plain 64-bit store"};
  for (int mode = 0; mode < 6; ++mode) {
    float total = 0, mtotal = 0;
    for (int rep = 0; rep < 60; ++rep) {
      hipEvent_t m0, m1;
      CK(hipEventCreate(&m0));
      CK(hipEventCreate(&m1));
      CK(hipEventRecord(m0));
      CK(hipMemsetAsync(tab, 0xFF, 8ull * cap));
      CK(hipEventRecord(m1));
      CK(hipEventRecord(a));
      const dim3 g((n + 255) / 256), t(256);
      switch (mode) {
        case 0: hipLaunchKernelGGL(ins<0>, g, t, 0, 0, dk, n, tab, cap - 1, dout); break;
        case 1: hipLaunchKernelGGL(ins<1>, g, t, 0, 0, dk, n, tab, cap - 1, dout); break;
        case 2: hipLaunchKernelGGL(ins<2>, g, t, 0, 0, dk, n, tab, cap - 1, dout); break;
        case 3: hipLaunchKernelGGL(ins<3>, g, t, 0, 0, dk, n, tab, cap - 1, dout); break;
        case 4: hipLaunchKernelGGL(ins<4>, g, t, 0, 0, dk, n, tab, cap - 1, dout); break;
        default: hipLaunchKernelGGL(ins<5>, g, t, 0, 0, dk, n, tab, cap - 1, dout); break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0, mms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      CK(hipEventElapsedTime(&mms, m0, m1));
      if (rep >= 10) {
        total += ms;
        mtotal += mms;
      }
      CK(hipEventDestroy(m0));
      CK(hipEventDestroy(m1));
    }
    std::printf("%-32s kernel %7.2f us   (memset 2 MiB %5.2f us)\n", names[mode], total / 50 * 1e3,
                mtotal / 50 * 1e3);
  }
  return 0;
}
