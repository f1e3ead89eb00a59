// Probe: rocPRIM inclusive_scan_by_key over a 20-byte value type (the joint (t, s) affine map of
// h3c_updio.hip) against a sequential host scan, at several sizes.  Values above 16 bytes take
// rocPRIM's non-packed look-back state.  A5 composes inline; A5N calls a non-inlined function
// returning the 20-byte struct (the form that gave wrong UpdateIO results); A5S makes only the
// scalar multiply a call (the shipped form).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan_by_key.hpp>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
constexpr uint32_t kOne = 0x80000000u, kPoly = 0x82F63B78u;
__host__ __device__ inline uint32_t gmul(uint32_t a, uint32_t b) {
  if (a == 0 || b == 0) return 0;
  if (a == kOne) return b;
  if (b == kOne) return a;
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}
struct A5 { uint32_t a, b, c, d, e; };
struct A5Op {
  __host__ __device__ A5 operator()(const A5 &x, const A5 &y) const {
    return A5{gmul(y.a, x.a), gmul(y.a, x.b) ^ y.b, gmul(y.c, x.a) ^ gmul(y.d, x.c), gmul(y.d, x.d),
              gmul(y.c, x.b) ^ gmul(y.d, x.e) ^ y.e};
  }
};
__host__ __device__ __attribute__((noinline)) A5 a5_general(A5 x, A5 y) {
  return A5{gmul(y.a, x.a), gmul(y.a, x.b) ^ y.b, gmul(y.c, x.a) ^ gmul(y.d, x.c), gmul(y.d, x.d),
            gmul(y.c, x.b) ^ gmul(y.d, x.e) ^ y.e};
}
struct A5NOp {
  __host__ __device__ A5 operator()(const A5 &x, const A5 &y) const {
    if (y.a == kOne && y.c == 0u && y.d == kOne) return A5{x.a, x.b ^ y.b, x.c, x.d, x.e ^ y.e};
    return a5_general(x, y);
  }
};
__host__ __device__ __attribute__((noinline)) uint32_t gloop(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}
__host__ __device__ inline uint32_t gsc(uint32_t a, uint32_t b) {
  return (a == 0 || b == 0) ? 0u : a == kOne ? b : b == kOne ? a : gloop(a, b);
}
struct A5SOp {
  __host__ __device__ A5 operator()(const A5 &x, const A5 &y) const {
    if (y.a == kOne && y.c == 0u && y.d == kOne) return A5{x.a, x.b ^ y.b, x.c, x.d, x.e ^ y.e};
    return A5{gsc(y.a, x.a), gsc(y.a, x.b) ^ y.b, gsc(y.c, x.a) ^ gsc(y.d, x.c), gsc(y.d, x.d),
              gsc(y.c, x.b) ^ gsc(y.d, x.e) ^ y.e};
  }
};
struct A4 { uint32_t a, b, c, e; };  // 16 bytes: the same maps with d = x^0 (packed look-back)
struct A4Op {
  __host__ __device__ A4 operator()(const A4 &x, const A4 &y) const {
    return A4{gmul(y.a, x.a), gmul(y.a, x.b) ^ y.b, gmul(y.c, x.a) ^ x.c, gmul(y.c, x.b) ^ x.e ^ y.e};
  }
};
template <class T, class Op>
int run(const char *name, size_t n, std::mt19937 &g, T (*mk)(std::mt19937 &)) {
  std::vector<uint32_t> key(n);
  std::vector<T> v(n), out(n), ref(n);
  uint32_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    if (g() % 50 == 0) ++k;
    key[i] = k;
    v[i] = mk(g);
  }
  Op op;
  for (size_t i = 0; i < n; ++i) ref[i] = (i && key[i] == key[i - 1]) ? op(ref[i - 1], v[i]) : v[i];
  uint32_t *dk; T *dv, *dout; void *tmp = nullptr; size_t tb = 0;
  if (hipMalloc(&dk, 4 * n) || hipMalloc(&dv, sizeof(T) * n) || hipMalloc(&dout, sizeof(T) * n)) return 1;
  if (hipMemcpy(dk, key.data(), 4 * n, hipMemcpyHostToDevice) || hipMemcpy(dv, v.data(), sizeof(T) * n, hipMemcpyHostToDevice)) return 1;
  if (rocprim::inclusive_scan_by_key(nullptr, tb, dk, dv, dout, n, op, rocprim::equal_to<uint32_t>(), 0)) return 1;
  if (hipMalloc(&tmp, tb)) return 1;
  if (rocprim::inclusive_scan_by_key(tmp, tb, dk, dv, dout, n, op, rocprim::equal_to<uint32_t>(), 0)) return 1;
  if (hipDeviceSynchronize() || hipMemcpy(out.data(), dout, sizeof(T) * n, hipMemcpyDeviceToHost)) return 1;
  size_t bad = 0, first = n;
  for (size_t i = 0; i < n; ++i)
    if (memcmp(&out[i], &ref[i], sizeof(T))) { ++bad; if (first == n) first = i; }
  printf("%-4s sizeof %2zu n %7zu: %zu wrong (first %zd)\n", name, sizeof(T), n, bad, first == n ? (ssize_t)-1 : (ssize_t)first);
  (void)hipFree(dk); (void)hipFree(dv); (void)hipFree(dout); (void)hipFree(tmp);
  return 0;
}
static uint32_t rm(std::mt19937 &g) { uint32_t r = g() % 3; return r == 0 ? kOne : r == 1 ? 0u : (uint32_t)g(); }
static A5 mk5(std::mt19937 &g) { return A5{rm(g), (uint32_t)g(), rm(g), rm(g), (uint32_t)g()}; }
static A4 mk4(std::mt19937 &g) { return A4{rm(g), (uint32_t)g(), rm(g), (uint32_t)g()}; }
int main() {
  std::mt19937 g(7);
  for (size_t n : {400ul, 5000ul, 100000ul}) {
    if (run<A5, A5Op>("A5", n, g, mk5)) return 1;
    if (run<A5, A5NOp>("A5N", n, g, mk5)) return 1;
    if (run<A5, A5SOp>("A5S", n, g, mk5)) return 1;
    if (run<A4, A4Op>("A4", n, g, mk4)) return 1;
  }
  return 0;
}
