// Host->device->kernel->host coherence probe under /opt/rocm's HIP runtime: which
// allocation / staging combinations hand a kernel the bytes just copied?  The kernel only
// reads inside the buffer it was given (no pointer chasing), so a wrong answer cannot fault.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/coherence_probe scripts/coherence_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void sum_kernel(const uint8_t *p, uint32_t n, uint32_t *out) {
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s += p[i] * (i % 251 + 1);
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ uint32_t w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = w[0] + w[1] + w[2] + w[3];
}

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return -1;                                                        \
    }                                                                   \
  } while (0)

// alloc: 0 hipMallocAsync/hipFreeAsync, 1 pooled hipMalloc (reused), 2 hipMalloc/hipFree per iteration
// src:   0 pageable, 1 pinned (reused)
static int run(int alloc, int src, hipStream_t st, int iters) {
  std::mt19937 rng(alloc * 10 + src);
  std::vector<uint8_t> pageable(1 << 20);
  uint8_t *pinned = nullptr;
  uint32_t *res_pin = nullptr;
  CK(hipHostMalloc((void **)&pinned, 1 << 20, 0));
  CK(hipHostMalloc((void **)&res_pin, 64, 0));
  uint8_t *pool = nullptr;
  CK(hipMalloc((void **)&pool, 2 << 20));
  int bad = 0;
  for (int it = 0; it < iters; ++it) {
    const uint32_t n = 1 + rng() % (64 << 10);
    uint8_t *h = src ? pinned : pageable.data();
    uint32_t want = 0;
    for (uint32_t i = 0; i < n; ++i) {
      h[i] = (uint8_t)(rng() >> 7);
      want += h[i] * (i % 251 + 1);
    }
    uint8_t *d = nullptr;
    if (alloc == 0) CK(hipMallocAsync((void **)&d, n + 64, st));
    else if (alloc == 1) d = pool + (rng() % 4) * 4096;
    else CK(hipMalloc((void **)&d, n + 64));
    uint32_t *dres = (uint32_t *)(d + ((n + 15) & ~15u));
    CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, st, d, n, dres);
    CK(hipMemcpyAsync(res_pin, dres, 4, hipMemcpyDeviceToHost, st));
    if (alloc == 0) CK(hipFreeAsync(d, st));
    CK(hipStreamSynchronize(st));
    if (alloc == 2) CK(hipFree(d));
    bad += *res_pin != want;
  }
  (void)hipFree(pool);
  (void)hipHostFree(pinned);
  (void)hipHostFree(res_pin);
  return bad;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  const char *an[3] = {"hipMallocAsync", "pooled hipMalloc", "hipMalloc/hipFree"};
  const char *sn[2] = {"pageable", "pinned"};
  for (int alloc = 0; alloc < 3; ++alloc)
    for (int src = 0; src < 2; ++src)
      for (int so = 0; so < 2; ++so) {
        const int bad = run(alloc, src, so ? s : nullptr, 300);
        std::printf("%-18s %-9s %-6s stream: %3d / 300 wrong\n", an[alloc], sn[src], so ? "own" : "null", bad);
      }
  return 0;
}
