// prim_probe.hip -- timing probe for the rocPRIM primitives a device-side UpdateIO
// pipeline would use (100k items): radix sort of (chunk key, op index) pairs at several
// key widths (merge-sort path vs forced onesweep), exclusive scan, and scan_by_key over a
// 20-byte affine element.  Tuning aid only; prints one line per primitive.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

struct Pair5 {
  uint32_t m, a, b, e, f;
};
struct Pair5Op {
  __host__ __device__ Pair5 operator()(const Pair5 &x, const Pair5 &y) const {
    return Pair5{x.m ^ y.m, x.a ^ y.b, x.b ^ y.b, x.e ^ y.e, x.f ^ y.f};
  }
};

__global__ void empty_kernel() {}

using MergeCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config,
                                            1024 * 1024>;
using SweepCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config,
                                            0>;

template <class F>
float time_it(hipStream_t st, F f, int reps = 20) {
  for (int i = 0; i < 3; ++i) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? std::strtoul(argv[1], nullptr, 0) : 100000;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<uint32_t> hk(n), hv(n);
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < n; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    hk[i] = (uint32_t)x;
    hv[i] = (uint32_t)i;
  }
  uint32_t *k, *k2, *v, *v2;
  CK(hipMalloc(&k, 4 * n));
  CK(hipMalloc(&k2, 4 * n));
  CK(hipMalloc(&v, 4 * n));
  CK(hipMalloc(&v2, 4 * n));
  CK(hipMemcpy(v, hv.data(), 4 * n, hipMemcpyHostToDevice));
  void *tmp = nullptr;
  size_t tmpb = 64u << 20;
  CK(hipMalloc(&tmp, tmpb));
  for (int bits : {7, 12, 17, 20, 32}) {
    std::vector<uint32_t> kk(n);
    for (size_t i = 0; i < n; ++i) kk[i] = bits == 32 ? hk[i] : hk[i] & ((1u << bits) - 1);
    CK(hipMemcpy(k, kk.data(), 4 * n, hipMemcpyHostToDevice));
    const float tm = time_it(st, [&] {
      size_t t = tmpb;
      CK(rocprim::radix_sort_pairs<MergeCfg>(tmp, t, k, k2, v, v2, n, 0, bits, st));
    });
    const float ts = time_it(st, [&] {
      size_t t = tmpb;
      CK(rocprim::radix_sort_pairs<SweepCfg>(tmp, t, k, k2, v, v2, n, 0, bits, st));
    });
    std::printf("radix_sort_pairs n=%zu bits=%2d  merge-path %8.1f us  onesweep %8.1f us\n", n, bits, tm, ts);
  }
  {
    const float t = time_it(st, [&] {
      size_t tb = tmpb;
      CK(rocprim::exclusive_scan(tmp, tb, v, v2, 0u, n, rocprim::plus<uint32_t>(), st));
    });
    std::printf("exclusive_scan u32 n=%zu  %8.1f us\n", n, t);
  }
  {
    Pair5 *p, *p2;
    CK(hipMalloc(&p, sizeof(Pair5) * n));
    CK(hipMalloc(&p2, sizeof(Pair5) * n));
    CK(hipMemset(p, 1, sizeof(Pair5) * n));
    std::vector<uint32_t> kk(n);
    for (size_t i = 0; i < n; ++i) kk[i] = (uint32_t)(i / 1563);
    CK(hipMemcpy(k, kk.data(), 4 * n, hipMemcpyHostToDevice));
    const float t = time_it(st, [&] {
      size_t tb = tmpb;
      CK(rocprim::inclusive_scan_by_key(tmp, tb, k, p, p2, n, Pair5Op(), rocprim::equal_to<uint32_t>(), st));
    });
    std::printf("inclusive_scan_by_key 20B n=%zu  %8.1f us\n", n, t);
  }
  {
    const float t = time_it(st, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st); }, 200);
    std::printf("empty launch  %8.2f us\n", t);
  }
  return 0;
}
