// h3c_engine.hip -- MI355X (gfx950) batched CRC32C / CRC32 chunk-checksum engine.
//
// Replaces the CPU arithmetic under 3FS's ChecksumInfo (src/fbs/storage/Common.h:113-201):
// folly::crc32c / crc32c_combine (Common.h:158,191) and folly::crc32 / crc32_combine
// (Common.h:161,195), batched over chunk payloads.  See DESIGN.md for the algorithm and
// the roofline; include/h3c_crc.h for the ABI.
//
// Algorithm (all arithmetic is GF(2), reflected representation, bit 31 = x^0):
//   * A chunk is cut into segments of `seg_bytes`; one wavefront owns one segment.
//   * A segment is walked in rows of 1 KiB aligned so the LAST row ends at the
//     16-byte-rounded segment end.  Lane l loads the 16 bytes at row+16l with one
//     coalesced global_load_dwordx4 (a wave reads 1 KiB contiguous per instruction).
//   * Each lane runs 4 independent CRC "streams", one per dword j of its 16 bytes.
//     Stream (l,j) sees one dword every 1024 bytes, so its register update is
//         s <- (s ^ d) * x^(8*1024)  mod P
//     computed as 4 byte lookups into tables T_k[b] = (b << 8k) * x^(8*1024).
//     Zero bytes in front of the segment do not change an init-0 CRC, so the
//     partial first row is simply masked to zero.
//   * At the end stream (l,j) sits 16l+4j (+ pad) bytes past the segment end; one
//     GF(2) multiply by x^-(8*(16l+4j)) moves it back, lanes XOR-reduce, and the
//     wave writes the segment's init-0 CRC.
//   * A finalize kernel folds segment CRCs per chunk with x^(8*seg_bytes) shifts and
//     applies the starting checksum: raw = crc0 ^ start * x^(8*len).
//   * Tables live in LDS replicated 32x and lane l reads copy l%32, so every
//     ds_read_b32 is bank-conflict-free for random bytes; the LDS address of a lookup
//     is a single v_perm_b32 of the register byte and a per-lane offset.
//     4 tables x 256 x 32 x 4 B = 128 KiB of the CU's 160 KiB.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "h3c_crc.h"

namespace {

constexpr uint32_t kPolyCrc32c = 0x82F63B78u;
constexpr uint32_t kPolyCrc32 = 0xEDB88320u;
constexpr uint32_t kOne = 0x80000000u;  // x^0 in the reflected representation
constexpr int kRowBytes = 1024;         // 64 lanes x 16 B
constexpr int kWavesPerBlock = 16;
constexpr int kThreads = kWavesPerBlock * 64;
constexpr int kCopies = 32;
constexpr int kLdsWords = 4 * 256 * kCopies;  // 32768 dwords = 128 KiB
constexpr uint64_t kMaxSegBytes = 1u << 20;
constexpr uint64_t kMinSegBytes = 16u << 10;
constexpr int kMaxDevices = 64;

// ---------------------------------------------------------------- host GF(2)
uint32_t hgf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (kOne >> i)) p ^= b;
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

uint32_t hgf_pow(uint32_t base, uint64_t e, uint32_t poly) {
  uint32_t r = kOne;
  while (e) {
    if (e & 1u) r = hgf_mul(r, base, poly);
    base = hgf_mul(base, base, poly);
    e >>= 1;
  }
  return r;
}

uint32_t hxpow8n(uint64_t n, uint32_t poly) { return hgf_pow(0x00800000u /* x^8 */, n, poly); }

// x^-1: the y with y*x == 1.  Multiplying by x is y>>1 ^ (poly if y&1); the
// result is x^0 (bit 31) only when y&1 and (y>>1)^poly == 1<<31.
uint32_t hx_inverse(uint32_t poly) { return ((poly ^ kOne) << 1) | 1u; }

// Device-side constant block, one per polynomial per device.
struct PolyConsts {
  uint32_t tab[4][256];  // tab[k][b] = (b << 8k) * x^(8*kRowBytes)
  uint32_t fix[256];     // [4l+j] = x^-(8*(16l+4j))
  uint32_t fixz[16];     // [z]    = x^-(8z)
  uint32_t pow8[64];     // [k]    = x^(8*2^k)
  uint32_t poly;
  uint32_t pad[3];
};

void build_consts(PolyConsts &pc, uint32_t poly) {
  std::memset(&pc, 0, sizeof(pc));
  pc.poly = poly;
  const uint32_t row = hxpow8n(kRowBytes, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) pc.tab[k][b] = hgf_mul(b << (8 * k), row, poly);
  const uint32_t xinv8 = hgf_pow(hx_inverse(poly), 8, poly);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 4; ++j) pc.fix[4 * l + j] = hgf_pow(xinv8, 16u * l + 4u * j, poly);
  for (int z = 0; z < 16; ++z) pc.fixz[z] = hgf_pow(xinv8, z, poly);
  uint32_t p = 0x00800000u;
  for (int k = 0; k < 64; ++k) {
    pc.pow8[k] = p;
    p = hgf_mul(p, p, poly);
  }
}

// Device copy of a descriptor (32 B).
struct DevChunk {
  uint64_t ptr;
  uint64_t len;
  uint32_t start;
  uint32_t out_idx;
  uint32_t seg_begin;
  uint32_t flags;  // bit0: result is {NONE,0}
};
constexpr uint32_t kFlagNone = 1u;

// ---------------------------------------------------------------- device GF(2)
__device__ __forceinline__ uint32_t dgf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
#pragma unroll 4
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

__device__ uint32_t dxpow8n(uint64_t n, const PolyConsts *__restrict__ pc, uint32_t poly) {
  uint32_t r = kOne;
  int k = 0;
  while (n) {
    if (n & 1u) r = (r == kOne) ? pc->pow8[k] : dgf_mul(r, pc->pow8[k], poly);
    n >>= 1;
    ++k;
  }
  return r;
}

#ifndef H3C_PERM_LAYOUT
#define H3C_PERM_LAYOUT 1
#endif
#ifndef H3C_XOR3_ASM
#define H3C_XOR3_ASM 1
#endif

// Per-lane LDS addressing of the replicated tables (see kernel header comment).
struct LaneLut {
  uint32_t off[4];
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if H3C_XOR3_ASM
  uint32_t d;  // gfx950 has no v_xor3_b32; v_bitop3_b32 with truth table 0x96 is a^b^c
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
#else
  return a ^ b ^ c;
#endif
}

#if H3C_PERM_LAYOUT
// Layout: table t (0..3), entry b, copy c at byte address
//   (t>>1)*64 KiB + b*256 + (t&1)*128 + c*4,
// i.e. each 256-byte LDS row holds entry b of two tables x 32 copies.  ds_read_b32
// banks on (addr/4)%32 = c, so lane l reading copy l%32 never conflicts.  The
// address is one v_perm_b32: byte1 <- byte k of r, bytes 0 and 2 <- the lane's
// per-table offset (byte0 = (t&1)<<7 | c<<2, byte2 = t>>1), byte3 <- 0.
__device__ __forceinline__ LaneLut make_lut(uint32_t lane) {
  LaneLut L;
  const uint32_t c4 = (lane & 31u) * 4u;
#pragma unroll
  for (int t = 0; t < 4; ++t) L.off[t] = ((uint32_t)(t >> 1) << 16) | ((uint32_t)(t & 1) << 7) | c4;
  return L;
}
__device__ __forceinline__ uint32_t row_step(uint32_t r, const char *lb, const LaneLut &L) {
  const uint32_t a0 = __builtin_amdgcn_perm(r, L.off[0], 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(r, L.off[1], 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(r, L.off[2], 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(r, L.off[3], 0x0C020700u);
  const uint32_t t0 = *reinterpret_cast<const uint32_t *>(lb + a0);
  const uint32_t t1 = *reinterpret_cast<const uint32_t *>(lb + a1);
  const uint32_t t2 = *reinterpret_cast<const uint32_t *>(lb + a2);
  const uint32_t t3 = *reinterpret_cast<const uint32_t *>(lb + a3);
  return xor3(t0, t1, t2) ^ t3;
}
// LDS dword i holds table ((i>>14)<<1 | (i>>5)&1), entry (i>>6)&255.
__device__ __forceinline__ uint32_t fill_value(const PolyConsts *__restrict__ pc, int i) {
  return pc->tab[((i >> 14) << 1) | ((i >> 5) & 1)][(i >> 6) & 255];
}
#else
// Layout: table k, entry b, copy c at byte address k*32 KiB + b*128 + c*4.
__device__ __forceinline__ LaneLut make_lut(uint32_t lane) {
  LaneLut L;
  L.off[0] = (lane & 31u) * 4u;
  L.off[1] = L.off[0] + 65536u;
  L.off[2] = L.off[3] = 0;
  return L;
}
__device__ __forceinline__ uint32_t row_step(uint32_t r, const char *lb, const LaneLut &L) {
  const uint32_t a0 = ((r << 7) & 0x7F80u) | L.off[0];
  const uint32_t a1 = ((r >> 1) & 0x7F80u) | L.off[0];
  const uint32_t a2 = ((r >> 9) & 0x7F80u) | L.off[1];
  const uint32_t a3 = ((r >> 17) & 0x7F80u) | L.off[1];
  const uint32_t t0 = *reinterpret_cast<const uint32_t *>(lb + a0);
  const uint32_t t1 = *reinterpret_cast<const uint32_t *>(lb + a1 + 32768);
  const uint32_t t2 = *reinterpret_cast<const uint32_t *>(lb + a2);
  const uint32_t t3 = *reinterpret_cast<const uint32_t *>(lb + a3 + 32768);
  return xor3(t0, t1, t2) ^ t3;
}
__device__ __forceinline__ uint32_t fill_value(const PolyConsts *__restrict__ pc, int i) {
  return pc->tab[i >> 13][(i >> 5) & 255];
}
#endif

__device__ __forceinline__ uint32_t byte_mask(uint64_t d, uint64_t s, uint64_t e) {
  const uint32_t lo = s > d ? (uint32_t)min<uint64_t>(s - d, 4) : 0u;
  const uint32_t hi = e > d ? (uint32_t)min<uint64_t>(e - d, 4) : 0u;
  if (hi <= lo) return 0u;
  const uint32_t hm = hi == 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u);
  const uint32_t lm = (1u << (8 * lo)) - 1u;
  return hm & ~lm;
}

// Edge-row load: bytes outside [s, e) read as zero; a piece with no byte inside
// is never dereferenced (it may lie outside the allocation).
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef const v4u __attribute__((address_space(1))) *gv4p;  // global (not flat) pointer

#ifndef H3C_NT_LOADS
#define H3C_NT_LOADS 1  // streamed payload is read once: nontemporal loads (+9% measured)
#endif


__device__ __forceinline__ uint4 load_row(uint64_t a) {
#if H3C_NT_LOADS
  const v4u v = __builtin_nontemporal_load((gv4p)a);
#else
  const v4u v = *(gv4p)a;
#endif
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Edge-row load: bytes outside [s, e) read as zero; a piece with no byte inside
// is never dereferenced (it may lie outside the allocation).
__device__ __forceinline__ uint4 load_masked(uint64_t a, uint64_t s, uint64_t e) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (a + 16 > s && a < e) {
    v = load_row(a);
    v.x &= byte_mask(a, s, e);
    v.y &= byte_mask(a + 4, s, e);
    v.z &= byte_mask(a + 8, s, e);
    v.w &= byte_mask(a + 12, s, e);
  }
  return v;
}

struct Streams {
  uint32_t s0, s1, s2, s3;
};

__device__ __forceinline__ void consume(Streams &st, uint4 v, const char *lb, const LaneLut &L) {
  st.s0 = row_step(st.s0 ^ v.x, lb, L);
  st.s1 = row_step(st.s1 ^ v.y, lb, L);
  st.s2 = row_step(st.s2 ^ v.z, lb, L);
  st.s3 = row_step(st.s3 ^ v.w, lb, L);
}

#ifndef H3C_UNROLL
#define H3C_UNROLL 4
#endif
constexpr int kUnroll = H3C_UNROLL;  // rows in flight per batch (x2 with the prefetch)

// init-0 CRC of bytes [S, E) (E > S), computed by one wavefront.
__device__ uint32_t segment_crc0(uint64_t S, uint64_t E, uint32_t lane, const char *lb, const LaneLut &L,
                                 const uint32_t fix[4], const PolyConsts *__restrict__ pc,
                                 uint32_t poly, uint32_t dbg) {
  const uint64_t E16 = (E + 15) & ~uint64_t(15);
  const uint64_t S16 = S & ~uint64_t(15);
  const uint32_t K = (uint32_t)((E16 - S16 + kRowBytes - 1) / kRowBytes);
  const uint64_t base = E16 - (uint64_t)K * kRowBytes + 16u * lane;

  Streams st{0, 0, 0, 0};
  // row 0 (masked)
  consume(st, load_masked(base, S, E), lb, L);
  // Rows 1 .. K-2 lie fully inside [S, E).  They are read with saddr-form global
  // loads: wave-uniform 64-bit row base in SGPRs + per-lane 32-bit offset 16*lane,
  // so no per-row VGPR address arithmetic.  Prefetch rows are clamped to the last
  // plain row (every load stays inside the segment; the few clamped re-reads at a
  // segment's end hit in cache).  One batch of kUnroll rows is in flight while the
  // previous batch is consumed.
  uint32_t r = 1;
  const uint32_t plain_end = K >= 2 ? K - 1 : 1;
  if (!(dbg & 1u) && r + kUnroll <= plain_end) {
    // readfirstlane returns int: widen through uint32_t so the low half is not sign-extended.
    const uint64_t row0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base - 16u * lane)) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((base - 16u * lane) >> 32))
                           << 32);
    typedef const char __attribute__((address_space(1))) *gcp;
    const gcp gbase = (gcp)row0;
    const uint32_t voff = 16u * lane;
    const uint32_t last = plain_end - 1;
    auto ld = [&](uint32_t row) -> uint4 {
      row = min(row, last);
      const gcp rp = gbase + (uint64_t)row * kRowBytes;  // uniform (SGPR) part
#if H3C_NT_LOADS
      const v4u v = __builtin_nontemporal_load((gv4p)(rp + voff));
#else
      const v4u v = *(gv4p)(rp + voff);  // + per-lane 32-bit offset
#endif
      return make_uint4(v.x, v.y, v.z, v.w);
    };
    // NOTE: an explicit two-buffer ping-pong form of this loop (no copy) miscompiled
    // under ROCm 7.2 hipcc -O3 at kUnroll=4 (wrong CRCs from the first pipelined
    // row; correct at -O1 and at kUnroll=2); this copy form is correct at every
    // setting tried and the copies are register renames.
    uint4 a[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) a[u] = ld(r + u);
    for (;;) {
      uint4 b[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) b[u] = ld(r + kUnroll + u);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) consume(st, a[u], lb, L);
      r += kUnroll;
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) a[u] = b[u];
      if (r + kUnroll > plain_end) break;
    }
    // a[] holds rows r .. r+kUnroll-1; fewer than kUnroll plain rows remain.
#pragma unroll
    for (int u = 0; u < kUnroll - 1; ++u)
      if (r + u < plain_end) consume(st, a[u], lb, L);
    r = plain_end;
  }
  for (; r < plain_end; ++r) consume(st, load_row(base + (uint64_t)r * kRowBytes), lb, L);
  // row K-1 (masked)
  if (K >= 2) consume(st, load_masked(base + (uint64_t)(K - 1) * kRowBytes, S, E), lb, L);

  // Move every stream back to the 16-byte-rounded end, then to the true end.
  // The per-lane constants are made opaque here so the compiler does not hoist
  // 4 x 32 shifted copies of them out of the segment loop (that spills).
  uint32_t f0 = fix[0], f1 = fix[1], f2 = fix[2], f3 = fix[3];
  asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
  uint32_t acc = dgf_mul(f0, st.s0, poly) ^ dgf_mul(f1, st.s1, poly) ^ dgf_mul(f2, st.s2, poly) ^
                 dgf_mul(f3, st.s3, poly);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
  const uint32_t z = (uint32_t)(E16 - E);
  if (z) acc = dgf_mul(acc, pc->fixz[z], poly);
  return acc;
}

// Kernel A: one wave per segment; waves take contiguous segment ranges.
__global__ __launch_bounds__(kThreads) void seg_crc_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                           uint32_t total_segs, uint64_t seg_bytes, uint32_t dbg,
                                                           const PolyConsts *__restrict__ pc,
                                                           uint32_t *__restrict__ seg_crc) {
  __shared__ uint32_t lds[kLdsWords];
  for (int i = threadIdx.x; i < kLdsWords; i += kThreads) lds[i] = fill_value(pc, i);
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t s_lo = (uint32_t)(gw * total_segs / nw);
  const uint32_t s_hi = (uint32_t)((gw + 1) * total_segs / nw);
  if (s_lo >= s_hi) return;

  const uint32_t poly = pc->poly;
  uint32_t fix[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) fix[j] = pc->fix[4 * lane + j];
  const char *lb = reinterpret_cast<const char *>(lds);
  const LaneLut L = make_lut(lane);

  // chunk owning s_lo: last c with seg_begin <= s_lo
  uint32_t lo = 0, hi = nchunks;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (chunks[mid].seg_begin <= s_lo) lo = mid; else hi = mid;
  }
  uint32_t c = lo;
  for (uint32_t s = s_lo; s < s_hi; ++s) {
    while (c + 1 < nchunks && chunks[c + 1].seg_begin <= s) ++c;
    const uint64_t k = s - chunks[c].seg_begin;
    const uint64_t p = chunks[c].ptr;
    const uint64_t len = chunks[c].len;
    const uint64_t S = p + k * seg_bytes;
    const uint64_t E = p + min(len, (k + 1) * seg_bytes);
    const uint32_t v = segment_crc0(S, E, lane, lb, L, fix, pc, poly, dbg);
    if (lane == 0) seg_crc[s] = v;
  }
}

// Kernel B: per chunk, fold segment CRCs, apply start, optionally compare.
__global__ void finalize_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks, uint32_t total_segs,
                                uint64_t seg_bytes, uint32_t seg_mul, const PolyConsts *__restrict__ pc,
                                const uint32_t *__restrict__ seg_crc, const uint32_t *__restrict__ expected,
                                uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                uint32_t *__restrict__ mismatch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nchunks) return;
  const DevChunk ch = chunks[i];
  const uint32_t poly = pc->poly;
  uint32_t raw = 0;
  if (!(ch.flags & kFlagNone)) {
    const uint32_t b = ch.seg_begin;
    const uint32_t e = (i + 1 < nchunks) ? chunks[i + 1].seg_begin : total_segs;
    uint32_t crc0 = 0;
    if (e > b) {
      crc0 = seg_crc[b];
      for (uint32_t s = b + 1; s < e; ++s) {
        const uint64_t seg_len = min<uint64_t>(seg_bytes, ch.len - (uint64_t)(s - b) * seg_bytes);
        const uint32_t m = seg_len == seg_bytes ? seg_mul : dxpow8n(seg_len, pc, poly);
        crc0 = dgf_mul(crc0, m, poly) ^ seg_crc[s];
      }
    }
    raw = crc0 ^ (ch.len ? dgf_mul(ch.start, dxpow8n(ch.len, pc, poly), poly) : ch.start);
  }
  out_raw[ch.out_idx] = raw;
  if (expected) {
    const bool good = raw == expected[ch.out_idx];
    ok[ch.out_idx] = good ? 1 : 0;
    if (!good && mismatch) atomicAdd(mismatch, 1u);
  }
}

__global__ void combine_kernel(const uint32_t *__restrict__ c1, const uint32_t *__restrict__ c2,
                               const uint64_t *__restrict__ len2, uint64_t n, const PolyConsts *__restrict__ pc,
                               uint32_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t poly = pc->poly;
  out[i] = dgf_mul(c1[i], dxpow8n(len2[i], pc, poly), poly) ^ c2[i];
}

__device__ __forceinline__ uint64_t dsplitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void fill_kernel(uint8_t *base, uint64_t chunk_words, uint64_t nchunks, uint64_t stride, uint64_t seed,
                            uint64_t first_chunk) {
  const uint64_t total = chunk_words * nchunks;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = t / chunk_words, k = t % chunk_words;
    *reinterpret_cast<uint64_t *>(base + c * stride + 8 * k) = dsplitmix64(seed ^ ((first_chunk + c) << 40) ^ k);
  }
}

// ---------------------------------------------------------------- host runtime
thread_local std::string g_last_error;

void set_error(const char *what, hipError_t e) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  g_last_error = buf;
}

#define HIP_TRY(expr)                 \
  do {                                \
    hipError_t e_ = (expr);           \
    if (e_ != hipSuccess) {           \
      set_error(#expr, e_);           \
      return H3C_ERR_HIP;             \
    }                                 \
  } while (0)

struct DeviceCtx {
  std::once_flag once;
  int status = H3C_ERR_NO_DEVICE;
  PolyConsts *d_consts[2] = {nullptr, nullptr};  // [0] CRC32C, [1] CRC32
  int num_cu = 0;
};
DeviceCtx g_dev[kMaxDevices];

int init_device(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return H3C_ERR_INVALID_ARG;
  DeviceCtx &ctx = g_dev[dev];
  std::call_once(ctx.once, [&] {
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) { ctx.status = H3C_ERR_NO_DEVICE; return; }
    auto body = [&]() -> int {
      HIP_TRY(hipSetDevice(dev));
      HIP_TRY(hipDeviceGetAttribute(&ctx.num_cu, hipDeviceAttributeMultiprocessorCount, dev));
      const uint32_t polys[2] = {kPolyCrc32c, kPolyCrc32};
      for (int i = 0; i < 2; ++i) {
        PolyConsts h;
        build_consts(h, polys[i]);
        HIP_TRY(hipMalloc(&ctx.d_consts[i], sizeof(PolyConsts)));
        HIP_TRY(hipMemcpy(ctx.d_consts[i], &h, sizeof(PolyConsts), hipMemcpyHostToDevice));
      }
      return H3C_OK;
    };
    ctx.status = body();
    (void)hipSetDevice(prev);
  });
  return ctx.status;
}

int current_device(int *dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    g_last_error = "no HIP device";
    return H3C_ERR_NO_DEVICE;
  }
  HIP_TRY(hipGetDevice(dev));
  return init_device(*dev);
}

// ---- profiling (events around seg_crc_kernel) ----
struct ProfRec {
  hipEvent_t a, b;
  uint64_t bytes;
};
std::mutex g_prof_mu;
std::vector<ProfRec> g_prof;
std::atomic<int> g_prof_on{0};
double g_prof_ms_done = 0;
uint64_t g_prof_launch_done = 0, g_prof_bytes_done = 0;

// test hook: H3C_DEBUG_FLAGS bit0 disables the pipelined row loop (read per plan)
uint32_t read_dbg_flags() {
  const char *e = std::getenv("H3C_DEBUG_FLAGS");
  return e ? (uint32_t)std::strtoul(e, nullptr, 0) : 0u;
}

struct Group {
  uint8_t type = H3C_TYPE_CRC32C;
  uint32_t nchunks = 0;
  uint32_t total_segs = 0;
  uint64_t bytes = 0;
  DevChunk *d_chunks = nullptr;
};

uint64_t pick_seg_bytes(uint64_t total_bytes, int num_cu) {
  // Aim for >= 2 segments per wave slot on the chip, within [16 KiB, 1 MiB].
  const uint64_t slots = (uint64_t)std::max(num_cu, 1) * kWavesPerBlock * 2;
  uint64_t want = total_bytes / slots;
  uint64_t seg = kMaxSegBytes;
  while (seg > kMinSegBytes && seg > want) seg >>= 1;
  return seg;
}

}  // namespace

struct h3c_plan {
  int device = 0;
  size_t n = 0;
  uint64_t seg_bytes = kMaxSegBytes;
  uint64_t bytes = 0;
  uint32_t dbg = 0;
  std::vector<Group> groups;
  uint32_t *d_segcrc = nullptr;
};

extern "C" {

uint32_t h3c_crc32c_shift(uint32_t crc, uint64_t nbytes) {
  return hgf_mul(crc, hxpow8n(nbytes, kPolyCrc32c), kPolyCrc32c);
}

uint32_t h3c_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2) { return h3c_crc32c_shift(c1, len2) ^ c2; }

uint32_t h3c_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
  return hgf_mul(c1, hxpow8n(len2, kPolyCrc32), kPolyCrc32) ^ c2;
}

int h3c_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int h3c_init(int device) { return init_device(device); }

const char *h3c_last_error(void) { return g_last_error.c_str(); }

void h3c_profile_enable(int on) { g_prof_on.store(on ? 1 : 0); }

int h3c_profile_read(double *seg_kernel_ms, uint64_t *seg_launches, uint64_t *seg_bytes, int reset) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto &r : g_prof) {
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    g_prof_ms_done += ms;
    g_prof_launch_done += 1;
    g_prof_bytes_done += r.bytes;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.clear();
  if (seg_kernel_ms) *seg_kernel_ms = g_prof_ms_done;
  if (seg_launches) *seg_launches = g_prof_launch_done;
  if (seg_bytes) *seg_bytes = g_prof_bytes_done;
  if (reset) {
    g_prof_ms_done = 0;
    g_prof_launch_done = 0;
    g_prof_bytes_done = 0;
  }
  return H3C_OK;
}

int h3c_plan_create(const h3c_desc *d, size_t n, int device, h3c_plan **out) {
  if (!out || (n && !d) || n > 0xFFFFFFF0u) return H3C_ERR_INVALID_ARG;
  int rc = init_device(device);
  if (rc) return rc;
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(device));
  auto *p = new h3c_plan();
  p->device = device;
  p->n = n;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i)
    if ((d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) && d[i].ptr) total += d[i].len;
  p->seg_bytes = pick_seg_bytes(total, g_dev[device].num_cu);
  p->dbg = read_dbg_flags();
  if (const char *e = std::getenv("H3C_SEG_BYTES")) {  // test hook: force the segment size
    const uint64_t v = std::strtoull(e, nullptr, 0);
    if (v >= kRowBytes && v % kRowBytes == 0) p->seg_bytes = v;
  }
  p->bytes = total;

  std::vector<DevChunk> hc[2];
  uint32_t segs[2] = {0, 0};
  uint64_t bytes[2] = {0, 0};
  for (size_t i = 0; i < n; ++i) {
    const h3c_desc &x = d[i];
    DevChunk c{};
    c.out_idx = (uint32_t)i;
    c.start = x.start_raw;
    int g = x.type == H3C_TYPE_CRC32 ? 1 : 0;
    const bool none = !(x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32) || (x.ptr == nullptr && x.len > 0);
    if (!none && x.len > 0 && x.mem != H3C_MEM_DEVICE) {
      delete p;
      (void)hipSetDevice(prev);
      g_last_error = "h3c_plan_create: descriptors must be device-resident";
      return H3C_ERR_INVALID_ARG;
    }
    c.seg_begin = segs[g];
    if (none) {
      c.flags = kFlagNone;
    } else {
      c.ptr = (uint64_t)(uintptr_t)x.ptr;
      c.len = x.len;
      const uint64_t ns = (x.len + p->seg_bytes - 1) / p->seg_bytes;
      if (segs[g] + ns > 0xFFFFFFF0u) {
        delete p;
        (void)hipSetDevice(prev);
        g_last_error = "h3c_plan_create: too many segments";
        return H3C_ERR_INVALID_ARG;
      }
      segs[g] += (uint32_t)ns;
      bytes[g] += x.len;
    }
    hc[g].push_back(c);
  }
  uint32_t max_segs = 0;
  for (int g = 0; g < 2; ++g) {
    if (hc[g].empty()) continue;
    Group gr;
    gr.type = g == 0 ? H3C_TYPE_CRC32C : H3C_TYPE_CRC32;
    gr.nchunks = (uint32_t)hc[g].size();
    gr.total_segs = segs[g];
    gr.bytes = bytes[g];
    hipError_t e = hipMalloc(&gr.d_chunks, hc[g].size() * sizeof(DevChunk));
    if (e == hipSuccess)
      e = hipMemcpy(gr.d_chunks, hc[g].data(), hc[g].size() * sizeof(DevChunk), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      set_error("h3c_plan_create: descriptor upload", e);
      h3c_plan_destroy(p);
      (void)hipSetDevice(prev);
      return H3C_ERR_HIP;
    }
    max_segs = std::max(max_segs, segs[g]);
    p->groups.push_back(gr);
  }
  if (max_segs) {
    hipError_t e = hipMalloc(&p->d_segcrc, (size_t)max_segs * sizeof(uint32_t));
    if (e != hipSuccess) {
      set_error("h3c_plan_create: segment scratch", e);
      h3c_plan_destroy(p);
      (void)hipSetDevice(prev);
      return H3C_ERR_HIP;
    }
  }
  (void)hipSetDevice(prev);
  *out = p;
  return H3C_OK;
}

uint64_t h3c_plan_bytes(const h3c_plan *p) { return p ? p->bytes : 0; }

void h3c_plan_destroy(h3c_plan *p) {
  if (!p) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(p->device);
  for (auto &g : p->groups)
    if (g.d_chunks) (void)hipFree(g.d_chunks);
  if (p->d_segcrc) (void)hipFree(p->d_segcrc);
  (void)hipSetDevice(prev);
  delete p;
}

int h3c_plan_run(h3c_plan *p, const uint32_t *expected_raw_dev, uint32_t *out_raw_dev, uint8_t *ok_dev,
                 uint32_t *mismatch_dev, void *stream) {
  if (!p || (p->n && !out_raw_dev) || (expected_raw_dev && !ok_dev)) return H3C_ERR_INVALID_ARG;
  if (p->n == 0) return H3C_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  if (prev != p->device) HIP_TRY(hipSetDevice(p->device));
  const DeviceCtx &ctx = g_dev[p->device];
  int rc = H3C_OK;
  for (const Group &g : p->groups) {
    const PolyConsts *pc = ctx.d_consts[g.type == H3C_TYPE_CRC32 ? 1 : 0];
    const uint32_t poly = g.type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;
    if (g.total_segs) {
      const uint32_t blocks =
          std::min<uint32_t>(ctx.num_cu, (g.total_segs + kWavesPerBlock - 1) / kWavesPerBlock);
      const bool prof = g_prof_on.load() != 0;
      ProfRec rec{};
      if (prof) {
        HIP_TRY(hipEventCreate(&rec.a));
        HIP_TRY(hipEventCreate(&rec.b));
        HIP_TRY(hipEventRecord(rec.a, st));
      }
      hipLaunchKernelGGL(seg_crc_kernel, dim3(blocks), dim3(kThreads), 0, st, g.d_chunks, g.nchunks, g.total_segs,
                         p->seg_bytes, p->dbg, pc, p->d_segcrc);
      HIP_TRY(hipGetLastError());
      if (prof) {
        HIP_TRY(hipEventRecord(rec.b, st));
        rec.bytes = g.bytes;
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof.push_back(rec);
      }
    }
    const uint32_t seg_mul = hxpow8n(p->seg_bytes, poly);
    const uint32_t fb = (g.nchunks + 255) / 256;
    hipLaunchKernelGGL(finalize_kernel, dim3(fb), dim3(256), 0, st, g.d_chunks, g.nchunks, g.total_segs,
                       p->seg_bytes, seg_mul, pc, p->d_segcrc, expected_raw_dev, out_raw_dev, ok_dev, mismatch_dev);
    HIP_TRY(hipGetLastError());
  }
  if (prev != p->device) HIP_TRY(hipSetDevice(prev));
  return rc;
}

// Synchronous API: stage host payloads, run a temporary plan, copy results back.
static int batch_sync(const h3c_desc *d, size_t n, const uint32_t *expected, uint8_t *out_type, uint32_t *out_raw,
                      uint8_t *ok, uint64_t *n_mismatch, void *stream) {
  if (n == 0) {
    if (n_mismatch) *n_mismatch = 0;
    return H3C_OK;
  }
  if (!d || !out_raw) return H3C_ERR_INVALID_ARG;
  int dev = 0;
  int rc = current_device(&dev);
  if (rc) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);

  // Stage host payloads into one device buffer.
  std::vector<h3c_desc> dd(d, d + n);
  uint64_t host_bytes = 0;
  for (auto &x : dd)
    if (x.mem != H3C_MEM_DEVICE && x.ptr && x.len && (x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32))
      host_bytes += (x.len + 255) & ~uint64_t(255);
  uint8_t *stage = nullptr;
  uint32_t *d_out = nullptr, *d_exp = nullptr, *d_mis = nullptr;
  uint8_t *d_ok = nullptr;
  h3c_plan *plan = nullptr;
  auto cleanup = [&]() {
    if (plan) h3c_plan_destroy(plan);
    if (stage) (void)hipFree(stage);
    if (d_out) (void)hipFree(d_out);
    if (d_exp) (void)hipFree(d_exp);
    if (d_ok) (void)hipFree(d_ok);
    if (d_mis) (void)hipFree(d_mis);
  };
#define SYNC_TRY(expr)        \
  do {                        \
    hipError_t e_ = (expr);   \
    if (e_ != hipSuccess) {   \
      set_error(#expr, e_);   \
      cleanup();              \
      return H3C_ERR_HIP;     \
    }                         \
  } while (0)
  if (host_bytes) {
    SYNC_TRY(hipMalloc(&stage, host_bytes));
    uint64_t off = 0;
    for (auto &x : dd) {
      if (x.mem != H3C_MEM_DEVICE && x.ptr && x.len && (x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32)) {
        SYNC_TRY(hipMemcpyAsync(stage + off, x.ptr, x.len, hipMemcpyHostToDevice, st));
        x.ptr = stage + off;
        x.mem = H3C_MEM_DEVICE;
        off += (x.len + 255) & ~uint64_t(255);
      }
    }
  }
  rc = h3c_plan_create(dd.data(), n, dev, &plan);
  if (rc) {
    cleanup();
    return rc;
  }
  SYNC_TRY(hipMalloc(&d_out, n * sizeof(uint32_t)));
  if (expected) {
    SYNC_TRY(hipMalloc(&d_exp, n * sizeof(uint32_t)));
    SYNC_TRY(hipMalloc(&d_ok, n));
    SYNC_TRY(hipMalloc(&d_mis, sizeof(uint32_t)));
    SYNC_TRY(hipMemcpyAsync(d_exp, expected, n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    SYNC_TRY(hipMemsetAsync(d_mis, 0, sizeof(uint32_t), st));
  }
  rc = h3c_plan_run(plan, d_exp, d_out, d_ok, d_mis, stream);
  if (rc) {
    cleanup();
    return rc;
  }
  SYNC_TRY(hipMemcpyAsync(out_raw, d_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  uint32_t mis = 0;
  if (expected) {
    SYNC_TRY(hipMemcpyAsync(ok, d_ok, n, hipMemcpyDeviceToHost, st));
    SYNC_TRY(hipMemcpyAsync(&mis, d_mis, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  }
  SYNC_TRY(hipStreamSynchronize(st));
#undef SYNC_TRY
  if (out_type)
    for (size_t i = 0; i < n; ++i) {
      const bool valid = (d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) &&
                         !(d[i].ptr == nullptr && d[i].len > 0);
      out_type[i] = valid ? d[i].type : (uint8_t)H3C_TYPE_NONE;
    }
  if (n_mismatch) *n_mismatch = mis;
  cleanup();
  return H3C_OK;
}

int h3c_batch_create(const h3c_desc *d, size_t n, uint8_t *out_type, uint32_t *out_raw, void *stream) {
  return batch_sync(d, n, nullptr, out_type, out_raw, nullptr, nullptr, stream);
}

int h3c_batch_verify(const h3c_desc *d, const uint32_t *expected_raw, size_t n, uint32_t *out_raw, uint8_t *ok,
                     uint64_t *n_mismatch, void *stream) {
  if (n && (!expected_raw || !ok)) return H3C_ERR_INVALID_ARG;
  return batch_sync(d, n, expected_raw, nullptr, out_raw, ok, n_mismatch, stream);
}

int h3c_batch_combine(uint8_t type, const uint32_t *c1_dev, const uint32_t *c2_dev, const uint64_t *len2_dev,
                      size_t n, uint32_t *out_dev, void *stream) {
  if (n == 0) return H3C_OK;
  if (!c1_dev || !c2_dev || !len2_dev || !out_dev) return H3C_ERR_INVALID_ARG;
  if (type != H3C_TYPE_CRC32C && type != H3C_TYPE_CRC32) return H3C_ERR_INVALID_ARG;
  int dev = 0;
  int rc = current_device(&dev);
  if (rc) return rc;
  const PolyConsts *pc = g_dev[dev].d_consts[type == H3C_TYPE_CRC32 ? 1 : 0];
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(combine_kernel, dim3((uint32_t)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     c1_dev, c2_dev, len2_dev, (uint64_t)n, pc, out_dev);
  HIP_TRY(hipGetLastError());
  return H3C_OK;
}

int h3c_fill_splitmix(void *base_dev, uint64_t chunk_len, uint64_t nchunks, uint64_t stride, uint64_t seed,
                      uint64_t first_chunk, void *stream) {
  if (!base_dev || chunk_len % 8 || stride % 8 || ((uintptr_t)base_dev & 7) || stride < chunk_len)
    return H3C_ERR_INVALID_ARG;
  int dev = 0;
  int rc = current_device(&dev);
  if (rc) return rc;
  const uint32_t blocks = (uint32_t)std::max(1, g_dev[dev].num_cu * 8);
  hipLaunchKernelGGL(fill_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<uint8_t *>(base_dev), chunk_len / 8, nchunks, stride, seed, first_chunk);
  HIP_TRY(hipGetLastError());
  return H3C_OK;
}

}  // extern "C"
