// PCIe host->device probe: hipMemcpyAsync piece sizes, streams, and zero-copy kernel reads.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cstdlib>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void zc_read(const v4u *p, uint64_t n16, uint32_t *out) {
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= __builtin_nontemporal_load(p + i);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x1234567u) out[0] = 1;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t total = 4ull << 30;
  uint8_t *h = nullptr, *d = nullptr;
  uint32_t *o;
  CK(hipHostMalloc(&h, total, hipHostMallocDefault));
  memset(h, 1, total);
  CK(hipMalloc(&d, 256ull << 20));
  CK(hipMalloc(&o, 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (size_t piece : {1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20, 256ull << 20}) {
    for (int nst : {1, 2}) {
      CK(hipDeviceSynchronize());
      double t0 = now();
      size_t k = 0;
      for (size_t off = 0; off < total; off += piece, ++k) {
        hipStream_t s = (nst == 2 && (k & 1)) ? s2 : s1;
        CK(hipMemcpyAsync(d + (off % (256ull << 20)) / piece * 0 + ((k & 1) ? (128ull << 20) : 0) % (256ull << 20) * (piece <= (128ull << 20)), h + off, piece, hipMemcpyHostToDevice, s));
      }
      CK(hipDeviceSynchronize());
      printf("memcpyAsync piece %4zu MiB streams %d: %.1f GB/s\n", piece >> 20, nst, total / (now() - t0) / 1e9);
    }
  }
  // zero-copy: kernel reads host memory directly
  uint8_t *hd = nullptr;
  CK(hipHostGetDevicePointer((void **)&hd, h, 0));
  for (int blocks : {256, 1024, 4096}) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    zc_read<<<blocks, 256, 0, s1>>>((const v4u *)hd, total / 16, o);
    CK(hipDeviceSynchronize());
    printf("zero-copy kernel read blocks %d: %.1f GB/s\n", blocks, total / (now() - t0) / 1e9);
  }
  return 0;
}
