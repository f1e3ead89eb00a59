// Memory-ceiling probe for the partial-update pattern (upd_delta_kernel): per 4 KiB block
// write, read the payload (sequential over the batch), read the old slot (random 4 KiB in a
// 4 GiB chunk set) and write the payload into the slot.  Variants isolate each stream.
// `ord` (optional) processes the writes in another order: "sorted" walks them in slot address
// order (payload reads become random), "sorted+seqpay" also lays the payloads out in that order
// (the ceiling of an address-ordered pass with staged payloads).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/rmwbw scripts/rmwbw.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <random>
#include <vector>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u __attribute__((address_space(1))) *gv4p;

// MODE bit0: read payload, bit1: read slot, bit2: write slot, bit3: plain (not nontemporal) stores.
// INF blocks in flight per wave.
template <int MODE, int INF>
__global__ __launch_bounds__(1024) void rmw(const char *pay, char *region, const uint32_t *slot, uint32_t n,
                                            uint32_t *out, const uint32_t *ord) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint32_t lo = (uint32_t)(gw * n / nw), hi = (uint32_t)((gw + 1) * n / nw);
  v4u acc = {0, 0, 0, 0};
  for (uint32_t i = lo; i < hi; i += INF) {
    v4u a[INF][4], b[INF][4];
#pragma unroll
    for (int f = 0; f < INF; ++f) {
      const uint32_t k0 = min(i + f, hi - 1), k = ord ? ord[k0] : k0;
      const char *p = pay + (uint64_t)k * 4096 + 16 * lane;
      const char *s = region + (uint64_t)slot[k] * 4096 + 16 * lane;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (MODE & 1) a[f][u] = __builtin_nontemporal_load((gv4p)(p + 1024 * u));
        if (MODE & 2) b[f][u] = __builtin_nontemporal_load((gv4p)(s + 1024 * u));
      }
    }
#pragma unroll
    for (int f = 0; f < INF; ++f) {
      if (i + f >= hi) break;
      char *s = region + (uint64_t)slot[ord ? ord[i + f] : i + f] * 4096 + 16 * lane;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (MODE & 2) acc ^= b[f][u];
        if (MODE & 4) {
          v4u w = (MODE & 1) ? a[f][u] : v4u{lane, i, 0, 0};
          if (MODE & 8)
            *(gv4p)(s + 1024 * u) = w;
          else
            __builtin_nontemporal_store(w, (gv4p)(s + 1024 * u));
        } else if (MODE & 1) {
          acc ^= a[f][u];
        }
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
  // address order, and the same slots pre-sorted (payload sequential in that order)
  std::vector<uint32_t> ho(n), hsorted(hs);
  for (uint32_t i = 0; i < n; ++i) ho[i] = i;
  std::stable_sort(ho.begin(), ho.end(), [&](uint32_t x, uint32_t y) { return hs[x] < hs[y]; });
  std::sort(hsorted.begin(), hsorted.end());
  uint32_t *ord, *slot_sorted;
  hipMalloc(&ord, 4ull * n);
  hipMalloc(&slot_sorted, 4ull * n);
  hipMemcpy(ord, ho.data(), 4ull * n, hipMemcpyHostToDevice);
  hipMemcpy(slot_sorted, hsorted.data(), 4ull * n, hipMemcpyHostToDevice);
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
  for (int wpc : {8, 16}) {
    char nm[96];
    snprintf(nm, sizeof nm, "[%2d waves/CU]", wpc);
    printf("%s\n", nm);
#define RO(MODE, INF, BYTES, LABEL, SLOT, ORD)                                             \
  snprintf(nm, sizeof nm, "  %-22s inf%d", LABEL, INF);                                    \
  run(nm, BYTES, [&] { rmw<MODE, INF><<<dim3(cus), dim3(64 * wpc)>>>(pay, region, SLOT, n, o, ORD); });
#define R(MODE, INF, BYTES, LABEL) RO(MODE, INF, BYTES, LABEL, slot, nullptr)
    R(7, 1, 12288, "rmw (pay+old+write)")
    R(7, 2, 12288, "rmw (pay+old+write)")
    R(15, 1, 12288, "rmw plain stores")
    R(15, 2, 12288, "rmw plain stores")
    R(12, 1, 4096, "write only, plain")
    R(3, 1, 8192, "read pay+old")
    R(3, 2, 8192, "read pay+old")
    R(6, 1, 8192, "read old+write")
    R(5, 1, 8192, "copy pay->slot")
    R(4, 1, 4096, "write slot only")
    R(2, 1, 4096, "read old only")
    R(1, 1, 4096, "read pay only")
    RO(7, 1, 12288, "rmw sorted", slot, ord)
    RO(7, 2, 12288, "rmw sorted", slot, ord)
    RO(7, 1, 12288, "rmw sorted+seqpay", slot_sorted, nullptr)
    RO(7, 2, 12288, "rmw sorted+seqpay", slot_sorted, nullptr)
    RO(4, 1, 4096, "write sorted only", slot_sorted, nullptr)
    RO(6, 1, 8192, "read old+write sorted", slot_sorted, nullptr)
  }
  return 0;
}
