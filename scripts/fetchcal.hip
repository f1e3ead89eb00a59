// FETCH_SIZE calibration for the small-chunk row shape.  Each kernel below reads
// exactly 8 GiB (a footprint 32x the 256 MiB Infinity Cache, so every line comes from HBM) with
// the load shape of one engine kernel and no CRC work:
//   rows4   4 lanes x 16 B per 4 KiB chunk (64-byte rows), the seg_uni_kernel<4, 1> shape
//   rows8   8 lanes x 16 B per chunk (128-byte rows, whole lines)
//   wide    64 lanes x 16 B (1 KiB per wave instruction), the seg_crc_kernel shape the guide's
//           x2 correction was calibrated on
// Run under rocprofv3 --pmc (FETCH_SIZE in one pass; TCC_EA0_RDREQ_{32B,64B,128B,}_sum in another):
// the memory-side request sizes say which correction each shape needs.  Each kernel runs 3 times.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/fetchcal scripts/fetchcal.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef const v4u __attribute__((address_space(1))) *gv4p;

template <bool NT>
__device__ __forceinline__ v4u ld(const char *a) {
  if (NT) return __builtin_nontemporal_load((gv4p)a);
  return *(gv4p)a;
}
// G lanes per chunk, B rows in flight per lane (as scripts/smallbw.hip); NT: nontemporal loads;
// SPAN: a lane's two consecutive loads are the two 16-byte halves of its 32 bytes of a 128-byte
// row (lanes at 32 gl, then 32 gl + 16), so every load instruction touches each chunk's whole line
template <int G, int B, bool NT = true, bool SPAN = false>
__device__ __forceinline__ void walk_body(const char *p, uint32_t nchunks, uint32_t chunk, uint32_t *out) {
  constexpr uint32_t NG = 64 / G, kQ = 16 * G;
  const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 16;
  const uint32_t lo = (uint32_t)(gw * nchunks / nw), hi = (uint32_t)((gw + 1) * nchunks / nw);
  const uint32_t K = chunk / kQ;
  v4u acc = {0, 0, 0, 0};
  for (uint32_t q0 = lo; q0 < hi; q0 += NG) {
    const uint32_t t = q0 + grp;
    if (t >= hi) break;
    const char *cb = p + (uint64_t)t * chunk;
    for (uint32_t u0 = 0; u0 < K; u0 += B) {
      v4u v[B];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const uint32_t u = u0 + b;
        const uint64_t off = SPAN ? (uint64_t)(u >> 1) * (2 * kQ) + 32 * gl + (u & 1) * 16 : (uint64_t)u * kQ + 16 * gl;
        v[b] = u < K ? ld<NT>(cb + off) : v4u{0, 0, 0, 0};
      }
#pragma unroll
      for (int b = 0; b < B; ++b) acc ^= v[b];
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}
__global__ __launch_bounds__(1024) void fetchcal_rows4(const char *p, uint32_t n, uint32_t chunk, uint32_t *o) {
  walk_body<4, 4>(p, n, chunk, o);
}
__global__ __launch_bounds__(1024) void fetchcal_rows4_plain(const char *p, uint32_t n, uint32_t chunk, uint32_t *o) {
  walk_body<4, 4, false>(p, n, chunk, o);
}
__global__ __launch_bounds__(1024) void fetchcal_rows4_span(const char *p, uint32_t n, uint32_t chunk, uint32_t *o) {
  walk_body<4, 4, true, true>(p, n, chunk, o);
}
__global__ __launch_bounds__(1024) void fetchcal_rows4_span_plain(const char *p, uint32_t n, uint32_t chunk,
                                                                  uint32_t *o) {
  walk_body<4, 4, false, true>(p, n, chunk, o);
}
__global__ __launch_bounds__(1024) void fetchcal_rows4_b8(const char *p, uint32_t n, uint32_t chunk, uint32_t *o) {
  walk_body<4, 8>(p, n, chunk, o);
}
__global__ __launch_bounds__(1024) void fetchcal_rows8(const char *p, uint32_t n, uint32_t chunk, uint32_t *o) {
  walk_body<8, 4>(p, n, chunk, o);
}
__global__ __launch_bounds__(1024) void fetchcal_wide(const char *p, uint32_t n, uint32_t chunk, uint32_t *o) {
  walk_body<64, 4>(p, n, chunk, o);
}

int main() {
  const uint64_t bytes = 8ull << 30;
  char *d;
  uint32_t *o;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  if (hipMemset(d, 1, bytes) != hipSuccess) return 1;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](const char *name, auto launch) {
    float best = 1e30f;
    for (int k = 0; k < 3; ++k) {
      (void)hipEventRecord(a);
      launch();
      (void)hipEventRecord(b);
      if (hipEventSynchronize(b) != hipSuccess) return false;
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    printf("%-18s bytes per launch %llu  best %.1f GB/s\n", name, (unsigned long long)bytes, bytes / (best / 1e3) / 1e9);
    return true;
  };
  const uint32_t chunk = 4096, n = (uint32_t)(bytes / chunk);
  bool ok = run("rows4", [&] { fetchcal_rows4<<<cus, 1024>>>(d, n, chunk, o); }) &&
            run("rows4_plain", [&] { fetchcal_rows4_plain<<<cus, 1024>>>(d, n, chunk, o); }) &&
            run("rows4_span", [&] { fetchcal_rows4_span<<<cus, 1024>>>(d, n, chunk, o); }) &&
            run("rows4_span_plain", [&] { fetchcal_rows4_span_plain<<<cus, 1024>>>(d, n, chunk, o); }) &&
            run("rows4_b8", [&] { fetchcal_rows4_b8<<<cus, 1024>>>(d, n, chunk, o); }) &&
            run("rows8", [&] { fetchcal_rows8<<<cus, 1024>>>(d, n, chunk, o); }) &&
            run("wide", [&] { fetchcal_wide<<<cus, 1024>>>(d, n, chunk, o); });
  return ok && hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
