// Read-bandwidth ceiling probe, second pass: shapes readbw.hip did not try, to see whether the
// streaming-read ceiling the headline kernel sits at (~6.9 TB/s) moves with
//  * loads in flight per lane (4 / 8 / 16 dwordx4 per row batch),
//  * workgroup shape (256 x 4, 512 x 2, 1024 x 1 per CU) and occupancy (1-2 x),
//  * XCD-aware segment placement (workgroups of one XCD read one contiguous region),
//  * buffer loads with each cache-policy combination (sc0 / nt / sc1 bits of gfx950),
//  * direct global->LDS loads (global_load_lds_dwordx4).
// Every variant XOR-reduces 8 GiB, 20 timed launches after 3 warm-ups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef const v4u __attribute__((address_space(1))) *gv4p;

// wave-segmented: each wave owns consecutive segments of `seg` bytes; rows of 1 KiB per wave
// (16 B per lane), UNR rows in flight.  XCD = 1 maps workgroup b to XCD b % 8's contiguous region.
template <int UNR, int XCD>
__global__ void rdseg(const char *p, uint64_t nseg, uint64_t seg, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
  uint64_t b = blockIdx.x;
  if (XCD) {
    const uint64_t per = gridDim.x / 8;
    b = (b % 8) * per + b / 8;
  }
  const uint64_t gw = b * wpb + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * wpb;
  v4u acc = {0, 0, 0, 0};
  for (uint64_t s = gw * nseg / nw; s < (gw + 1) * nseg / nw; ++s) {
    const char *bp = p + s * seg + 16 * lane;
    for (uint64_t r = 0; r < seg; r += 1024 * UNR) {
      v4u v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load((gv4p)(bp + r + 1024 * u));
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc ^= v[u];
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

// buffer loads with an explicit cache policy (aux bits: 1 = sc0, 2 = nt, 16 = sc1)
template <int AUX>
__global__ __launch_bounds__(1024) void rdbuf(const char *p, uint64_t nseg, uint64_t seg, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 16;
  v4u acc = {0, 0, 0, 0};
  for (uint64_t s = gw * nseg / nw; s < (gw + 1) * nseg / nw; ++s) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p + s * seg), 0, (int)seg, 0x00020000);
    for (uint32_t r = 0; r < seg; r += 4096) {
      v4u v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, r + 1024 * u + 16 * lane, 0, AUX));
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= v[u];
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

// direct global -> LDS loads: each wave streams its segment through a private 4 KiB LDS ring
// (4 rows of 1 KiB) and XORs one dword per lane back out of it.
__global__ __launch_bounds__(1024) void rdlds(const char *p, uint64_t nseg, uint64_t seg, uint32_t *out) {
  __shared__ uint32_t ring[16][4][256];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + w, nw = (uint64_t)gridDim.x * 16;
  uint32_t acc = 0;
  for (uint64_t s = gw * nseg / nw; s < (gw + 1) * nseg / nw; ++s) {
    const char *bp = p + s * seg + 16 * lane;
    for (uint64_t r = 0; r < seg; r += 4096) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(bp + r + 1024 * u),
                                         (void __attribute__((address_space(3))) *)&ring[w][u][0], 16, 0, 2);
      __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= ring[w][u][lane * 4] ^ ring[w][u][lane * 4 + 3];
    }
  }
  if (acc == 0x12345678u) out[0] = 1;
}

int main() {
  const uint64_t bytes = 8ull << 30;
  char *d;
  uint32_t *o;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  hipMemset(d, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  auto run = [&](const char *name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", name); return; }
    hipEventRecord(a);
    const int it = 20;
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-44s %8.1f GB/s\n", name, bytes * it / (ms / 1e3) / 1e9);
    fflush(stdout);
  };
  const uint64_t S = 256 << 10, n = bytes / S;
  run("seg256K u4 1024x1/CU (readbw.hip shape)", [&] { rdseg<4, 0><<<cus, 1024>>>(d, n, S, o); });
  run("seg256K u8 1024x1/CU", [&] { rdseg<8, 0><<<cus, 1024>>>(d, n, S, o); });
  run("seg256K u16 1024x1/CU", [&] { rdseg<16, 0><<<cus, 1024>>>(d, n, S, o); });
  run("seg256K u4 1024x2/CU", [&] { rdseg<4, 0><<<cus * 2, 1024>>>(d, n, S, o); });
  run("seg256K u8 1024x2/CU", [&] { rdseg<8, 0><<<cus * 2, 1024>>>(d, n, S, o); });
  run("seg256K u4 512x2/CU", [&] { rdseg<4, 0><<<cus * 2, 512>>>(d, n, S, o); });
  run("seg256K u8 512x4/CU", [&] { rdseg<8, 0><<<cus * 4, 512>>>(d, n, S, o); });
  run("seg256K u4 256x4/CU", [&] { rdseg<4, 0><<<cus * 4, 256>>>(d, n, S, o); });
  run("seg256K u8 256x8/CU", [&] { rdseg<8, 0><<<cus * 8, 256>>>(d, n, S, o); });
  run("seg256K u4 1024x1/CU xcd-contiguous", [&] { rdseg<4, 1><<<cus, 1024>>>(d, n, S, o); });
  run("seg256K u8 1024x2/CU xcd-contiguous", [&] { rdseg<8, 1><<<cus * 2, 1024>>>(d, n, S, o); });
  run("seg64K u8 1024x1/CU", [&] { rdseg<8, 0><<<cus, 1024>>>(d, bytes / (64 << 10), 64 << 10, o); });
  run("seg1M u8 1024x1/CU", [&] { rdseg<8, 0><<<cus, 1024>>>(d, bytes / (1 << 20), 1 << 20, o); });
  run("buffer aux=0 (default)", [&] { rdbuf<0><<<cus, 1024>>>(d, n, S, o); });
  run("buffer aux=1 (sc0)", [&] { rdbuf<1><<<cus, 1024>>>(d, n, S, o); });
  run("buffer aux=2 (nt)", [&] { rdbuf<2><<<cus, 1024>>>(d, n, S, o); });
  run("buffer aux=3 (sc0 nt)", [&] { rdbuf<3><<<cus, 1024>>>(d, n, S, o); });
  run("buffer aux=16 (sc1)", [&] { rdbuf<16><<<cus, 1024>>>(d, n, S, o); });
  run("buffer aux=18 (sc1 nt)", [&] { rdbuf<18><<<cus, 1024>>>(d, n, S, o); });
  run("buffer aux=19 (sc0 sc1 nt)", [&] { rdbuf<19><<<cus, 1024>>>(d, n, S, o); });
  run("global_load_lds 16B nt 1024x1/CU", [&] { rdlds<<<cus, 1024>>>(d, n, S, o); });
  return 0;
}
