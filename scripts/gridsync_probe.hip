// Probe: the cost of a grid-wide barrier in a cooperative launch of one 1024-thread workgroup per CU (160 KiB
// of LDS each, as the update kernels), by a hand-rolled sense-reversing barrier on one agent-scope counter.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/gridsync_probe scripts/gridsync_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ void grid_barrier(unsigned *count, unsigned *gen, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (atomicAdd(count, 1u) + 1 == nwg) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void k_sync(unsigned *count, unsigned *gen, int reps, unsigned long long *ts) {
  __shared__ unsigned lds[40 * 1024];  // 160 KiB: one workgroup per CU
  lds[threadIdx.x] = threadIdx.x;
  if (threadIdx.x == 0 && blockIdx.x == 0) ts[0] = wall_clock64();
  for (int r = 0; r < reps; ++r) grid_barrier(count, gen, gridDim.x);
  if (threadIdx.x == 0 && blockIdx.x == 0) ts[1] = wall_clock64() + lds[5];
}

int main() {
  int dev = 0, coop = 0, cus = 0;
  hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int per_cu = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(k_sync), 1024, 0);
  printf("cooperative launch %d, CUs %d, workgroups per CU %d\n", coop, cus, per_cu);
  unsigned *cnt, *gen;
  unsigned long long *ts;
  hipMalloc(&cnt, 8);
  hipMalloc(&gen, 8);
  hipMalloc(&ts, 16);
  hipMemset(cnt, 0, 8);
  hipMemset(gen, 0, 8);
  for (int nwg : {250, 256}) {
    for (int reps : {0, 1, 10, 100}) {
      void *args[] = {&cnt, &gen, &reps, &ts};
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipError_t e = hipSuccess;
      for (int w = 0; w < 3; ++w) e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_sync), dim3(nwg), dim3(1024), args, 0, 0);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int it = 0; it < 20; ++it) e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_sync), dim3(nwg), dim3(1024), args, 0, 0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      unsigned long long h[2];
      hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost);
      printf("nwg %d reps %3d: launch rc %d, %.2f us per launch (events), first-wg span %.2f us\n", nwg, reps, (int)e,
             ms * 1e3 / 20, (double)(h[1] - h[0]) / 100.0);
    }
  }
  return 0;
}
