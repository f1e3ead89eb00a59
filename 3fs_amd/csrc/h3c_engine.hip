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
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "h3c_crc.h"

#include "h3c_common.hpp"


namespace {

// Kernel A: one wave per segment; waves take contiguous segment ranges.  With `fin` (every chunk
// exactly one segment: config 2's 1 MiB chunks) the wave finishes its chunk itself -- the init's
// share, the result, the verify flag and count -- and no finalize launch follows.
__device__ __forceinline__ void seg_crc_kernel_body(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                           uint32_t total_segs, uint64_t seg_bytes, uint32_t dbg,
                                                           const PolyConsts *__restrict__ pc,
                                                           uint32_t *__restrict__ seg_crc, uint32_t fin,
                                                           const uint32_t *__restrict__ expected,
                                                           uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                           uint32_t *__restrict__ mismatch) {
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRedWords];
  fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, threadIdx.x, kThreads);
  __syncthreads();
  const uint32_t *red = lds + kLdsWords;

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
    // (fin: the chunk's result slot, init share and expected value, loaded before the segment so
    // that their round trip overlaps it)
    uint32_t idx = 0, xs = 0, ex = 0;
    if (fin) {
      idx = chunks[c].out_idx;
      xs = (chunks[c].flags & kFlagNone) ? 0u : chunks[c].xstart;
      if (expected) ex = expected[idx];
    }
    const uint32_t v = segment_crc0(S, E, lane, lb, L, fix, red, pc, poly, dbg);
    if (!fin) {
      if (lane == 0) seg_crc[s] = v;
    } else if (lane == 0) {  // (finalize_kernel's one-segment case)
      const uint32_t raw = (chunks[c].flags & kFlagNone) ? 0u : v ^ xs;
      out_raw[idx] = raw;
      if (expected) {
        const bool good = raw == ex;
        ok[idx] = good ? 1 : 0;
        if (!good && mismatch) atomicAdd(mismatch, 1u);
      }
    }
  }
}
__global__ __launch_bounds__(kThreads) void seg_crc_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                           uint32_t total_segs, uint64_t seg_bytes, uint32_t dbg,
                                                           const PolyConsts *__restrict__ pc,
                                                           uint32_t *__restrict__ seg_crc, uint32_t fin,
                                                           const uint32_t *__restrict__ expected,
                                                           uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                           uint32_t *__restrict__ mismatch,
                                                           unsigned long long *ts) {  // ts: h3c_rt::prof_stamp's slot, or nullptr
  stamp_begin(ts);
  seg_crc_kernel_body(chunks, nchunks, total_segs, seg_bytes, dbg, pc, seg_crc, fin, expected, out_raw, ok, mismatch);
  stamp_end(ts);
}

// Bytes of a row outside a chunk's [S, E) masked off (the small-chunk kernels' edge rows).
__device__ __forceinline__ uint4 mask_row(uint4 v, uint64_t a, uint64_t S, uint64_t E) {
  v.x &= byte_mask(a, S, E);
  v.y &= byte_mask(a + 4, S, E);
  v.z &= byte_mask(a + 8, S, E);
  v.w &= byte_mask(a + 12, S, E);
  return v;
}


// Kernel A'': the same batches with several chunks per wave.  A group of G lanes owns one
// chunk and walks it in rows of 16*G bytes (tables with stride x^(8*16*G)); the 64/G
// groups' Horner passes and their log2(G)-level shuffle trees run in the same
// instructions, so a chunk pays G/64 of a wave fold instead of a whole one (the fold was
// about a third of a one-chunk-per-wave kernel's instructions per chunk; that form,
// seg_small_kernel, is gone).  G = 4 for chunks up to
// ~5 KiB, 16 above.
#ifndef H3C_SMALL_LANES_LO
#define H3C_SMALL_LANES_LO 4  // lanes per chunk for chunks of at most 6 rows of 1 KiB (4 or 8)
#endif
#ifndef H3C_SMALL_PIECES_LO
#define H3C_SMALL_PIECES_LO 1  // 16-byte pieces per lane and row there (1 or 2)
#endif
#ifndef H3C_SMALL_LANES_HI
#define H3C_SMALL_LANES_HI 16  // lanes per chunk above that
#endif
#ifndef H3C_SMALL_PIECES_HI
#define H3C_SMALL_PIECES_HI 1
#endif
#ifndef H3C_QUAD_BATCH
#define H3C_QUAD_BATCH 4
#endif
constexpr int kQuadBatch = H3C_QUAD_BATCH;  // rows per load batch (two batches in flight)
#ifndef H3C_UNI_BATCH
#define H3C_UNI_BATCH 4
#endif
constexpr int kUniBatch = H3C_UNI_BATCH;  // the same for seg_uni_kernel
#ifndef H3C_UNI_LANES_LO
#define H3C_UNI_LANES_LO 4  // seg_uni_kernel's lanes per chunk up to 6 rows of 1 KiB
#endif
#ifndef H3C_UNI_COPIES
#define H3C_UNI_COPIES 32  // seg_uni_kernel's LDS table copies: 32 (1 x 1024 threads per CU) or 16 (2 x 768)
#endif
constexpr int kUniCopies = H3C_UNI_COPIES;
constexpr int kUniThreads = kUniCopies == 16 ? 768 : kThreads;
constexpr int kUniWaves = kUniThreads / 64;
constexpr int kUniLdsWords = kUniCopies == 16 ? kLdsWords16 : kLdsWords;
#ifndef H3C_UNI_LANES_HI
#define H3C_UNI_LANES_HI 16
#endif

__device__ __forceinline__ uint32_t shfl32(uint32_t v, uint32_t src) { return (uint32_t)__shfl((int)v, (int)src, 64); }

// G lanes per chunk, each reading W adjacent 16-byte pieces of a row of 16*G*W bytes
// (16 x 1: 256-byte rows, four chunks per wave; 4 x 1: 64-byte rows, sixteen chunks).
template <int G, int W>
__device__ __forceinline__ void seg_quad_kernel_body(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                           const PolyConsts *__restrict__ pc,
                                                           const uint32_t *__restrict__ expected,
                                                           uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                           uint32_t *__restrict__ mismatch) {
  static_assert(G == 4 || G == 8 || G == 16, "4, 8 or 16 lanes per chunk");
  static_assert(W == 1 || W == 2, "one or two 16-byte pieces per lane and row");
  static_assert(G * W <= 16, "rows of at most 256 bytes");
  constexpr int kLevels = G == 16 ? 4 : G == 8 ? 3 : 2;  // shuffle-tree levels inside a group
  constexpr int kLw = W == 2 ? 1 : 0;                    // log2(W)
  constexpr uint32_t NG = 64 / G;                        // chunks per wave step
  constexpr int kRed = (1 + kLw + kLevels) * 1024;       // x^-32, x^-128 (W = 2), the tree levels
  constexpr uint64_t kQ = 16u * G * W;                   // row bytes
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRed];
  fill_tables(lds, kQ == 256 ? pc->tabq : kQ == 128 ? pc->tabo : pc->tabf, &pc->red[0][0][0], kRed, threadIdx.x,
              kThreads);
  __syncthreads();
  const uint32_t *red = lds + kLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t lo = (uint32_t)(gw * nchunks / nw), hi = (uint32_t)((gw + 1) * nchunks / nw);
  if (lo >= hi) return;
  const uint32_t poly = pc->poly;
  const LaneLut L = make_lut(lane);
  // Descriptors come in groups of 64 (lane k holds chunk g0 + k's).  The next group's are
  // loaded when a group starts, so the last quad of a group can already load the first
  // rows of the next group's first quad: the row pipeline never drains between groups.
  struct Desc {
    uint32_t plo, phi, len, xs, out, cnt;
  };
  auto load_desc = [&](uint32_t g) {
    Desc d{0, 0, 0, 0, 0, g < hi ? min(64u, hi - g) : 0u};
    if (lane < d.cnt) {
      const DevChunk &ch = chunks[g + lane];
      d.plo = (uint32_t)ch.ptr;
      d.phi = (uint32_t)(ch.ptr >> 32);
      d.len = (uint32_t)ch.len;  // one short segment: below 4 GiB
      d.xs = ch.xstart;
      d.out = ch.out_idx;
    }
    return d;
  };
  // quad q's chunk for this group of lanes: start, end, row count, this lane's first address
  auto quad = [&](const Desc &d, uint32_t q, uint64_t &S, uint64_t &E, uint32_t &K, uint64_t &la, uint32_t &src) {
    const uint32_t t = q + grp;
    const bool valid = t < d.cnt;
    src = valid ? t : q;
    S = (uint64_t)shfl32(d.plo, src) | ((uint64_t)shfl32(d.phi, src) << 32);
    E = S + shfl32(d.len, src);
    const uint64_t base = S & ~(kQ - 1);
    K = valid ? (uint32_t)((E - base + kQ - 1) / kQ) : 0u;
    la = base + 16u * W * gl;
  };
  Desc m = load_desc(lo);
  uint64_t S, E, la;
  uint32_t K, src;
  quad(m, 0, S, E, K, la, src);
  uint4 cur[kQuadBatch][W], nxt[kQuadBatch][W];
#pragma unroll
  for (int b = 0; b < kQuadBatch; ++b)
#pragma unroll
    for (int w = 0; w < W; ++w)
      cur[b][w] = (uint32_t)b < K ? load_row_w<kQ>(la + (uint64_t)b * kQ + 16u * w) : make_uint4(0, 0, 0, 0);
  for (uint32_t g0 = lo; g0 < hi; g0 += 64) {
    const uint32_t cnt = m.cnt;
    const Desc n = load_desc(hi - g0 > 64 ? g0 + 64 : hi);
    const uint32_t m_exp = expected && lane < cnt ? expected[m.out] : 0u;
    for (uint32_t q0 = 0; q0 < cnt; q0 += NG) {
      const bool valid = q0 + grp < cnt;
      // the next quad's first batch (in this group or the next) is loaded during this
      // quad's last batch and fold
      uint64_t S1 = S, E1 = E, la1 = la;
      uint32_t K1 = 0, src1 = src;
      if (q0 + NG < cnt)
        quad(m, q0 + NG, S1, E1, K1, la1, src1);
      else if (n.cnt)
        quad(n, 0, S1, E1, K1, la1, src1);
      uint32_t kmax = 0;
#pragma unroll
      for (uint32_t g = 0; g < NG; ++g) kmax = max(kmax, (uint32_t)__builtin_amdgcn_readlane(K, g * G));
      Streams st[W];
#pragma unroll
      for (int w = 0; w < W; ++w) st[w] = Streams{0, 0, 0, 0};
      for (uint32_t u0 = 0; u0 < kmax; u0 += kQuadBatch) {
        const uint32_t n0 = u0 + kQuadBatch;
        if (n0 < kmax) {  // the next batch in flight while this one is consumed
#pragma unroll
          for (int b = 0; b < kQuadBatch; ++b)
#pragma unroll
            for (int w = 0; w < W; ++w)
              nxt[b][w] = n0 + b < K ? load_row_w<kQ>(la + (uint64_t)(n0 + b) * kQ + 16u * w) : make_uint4(0, 0, 0, 0);
        } else {
#pragma unroll
          for (int b = 0; b < kQuadBatch; ++b)
#pragma unroll
            for (int w = 0; w < W; ++w)
              nxt[b][w] = (uint32_t)b < K1 ? load_row_w<kQ>(la1 + (uint64_t)b * kQ + 16u * w) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int b = 0; b < kQuadBatch; ++b) {
          const uint32_t u = u0 + b;
          if (u < K) {
            const bool edge = (u == 0 && (S & (kQ - 1))) || (u + 1 == K && (E & (kQ - 1)));
#pragma unroll
            for (int w = 0; w < W; ++w) {
              uint4 x = cur[b][w];
              if (edge) x = mask_row(x, la + (uint64_t)u * kQ + 16u * w, S, E);
              consume(st[w], x, lb, L);
            }
          }
        }
#pragma unroll
        for (int b = 0; b < kQuadBatch; ++b)
#pragma unroll
          for (int w = 0; w < W; ++w) cur[b][w] = nxt[b][w];
      }
      // fold each group's stream states: Horner over a piece's 4 streams with x^-32, the
      // lane's second piece (16 bytes further) with x^-128, then log2(G) shuffle levels
      // inside the group (lane gl + 2^k is 16 * W * 2^k bytes further)
      uint32_t v = 0;
#pragma unroll
      for (int w = W - 1; w >= 0; --w) {
        if (w != W - 1) v = tab_mul(v, red + 1024);
        uint32_t p = tab_mul(st[w].s3, red) ^ st[w].s2;
        p = tab_mul(p, red) ^ st[w].s1;
        v ^= tab_mul(p, red) ^ st[w].s0;
      }
#pragma unroll
      for (int k = 0; k < kLevels; ++k) {
        const uint32_t o = (uint32_t)__shfl_down((int)v, 1u << k, G);
        if ((gl & ((2u << k) - 1u)) == 0) v ^= tab_mul(o, red + 1024 * (k + 1 + kLw));
      }
      // the bytes of the last row past E were walked as zeros: remove them
      const uint32_t pad = (uint32_t)(((E + kQ - 1) & ~(kQ - 1)) - E);
      if (gl == 0 && valid) {
        if (pad >> 4) v = dgf_mul(v, pc->fix[4 * (pad >> 4)], poly);
        if (pad & 15) v = dgf_mul(v, pc->fixz[pad & 15], poly);
      }
      const uint32_t xs = shfl32(m.xs, src), o = shfl32(m.out, src), want = shfl32(m_exp, src);
      if (gl == 0 && valid) {
        const uint32_t raw = v ^ xs;
        out_raw[o] = raw;
        if (expected) {
          const bool good = raw == want;
          ok[o] = good ? 1 : 0;
          if (!good && mismatch) atomicAdd(mismatch, 1u);
        }
      }
      S = S1;
      E = E1;
      K = K1;
      la = la1;
      src = src1;
    }
    m = n;
  }
}
template <int G, int W>
__global__ __launch_bounds__(kThreads) void seg_quad_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                           const PolyConsts *__restrict__ pc,
                                                           const uint32_t *__restrict__ expected,
                                                           uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                           uint32_t *__restrict__ mismatch,
                                                            unsigned long long *ts) {  // ts: h3c_rt::prof_stamp's slot, or nullptr
  stamp_begin(ts);
  seg_quad_kernel_body<G, W>(chunks, nchunks, pc, expected, out_raw, ok, mismatch);
  stamp_end(ts);
}

// Kernel A4: seg_quad_kernel<G, 1> for a batch whose chunks all have one length, a multiple of
// the 16*G-byte row, at row-aligned addresses, with one start value -- a plan or verify of
// uniform IO buffers / chunk pieces.  Every row is whole (no edge masks, no tail fix), the row
// count K is the same for every chunk (loop control stays scalar) and the start's share xs is
// one value.  With chunks == nullptr the batch is contiguous (chunk i at base + i * stride,
// result i): no descriptor at all.
// C chunks per group of G lanes: with C = 2 an 8-lane group walks two chunks in interleaved
// rows, so every load instruction reads whole 128-byte lines (the 8-lane access pattern alone
// reads at ~7.0 TB/s against ~6.1 TB/s for 4 lanes' 64-byte rows) while a wave step still
// covers 16 chunks and their folds overlap (profiles/r02_small_pattern_ceiling.txt).
template <int G, int C = 1>
__device__ __forceinline__ void seg_uni_kernel_body(const DevChunk *__restrict__ chunks, uint64_t base,
                                                          uint64_t stride, uint32_t nchunks, uint32_t K, uint32_t xs,
                                                          const PolyConsts *__restrict__ pc,
                                                          const uint32_t *__restrict__ expected,
                                                          uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                          uint32_t *__restrict__ mismatch) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "1, 2, 4, 8 or 16 lanes per chunk");
  static_assert(C == 1 || C == 2, "one or two chunks per group");
  constexpr int kLevels = G == 16 ? 4 : G == 8 ? 3 : G == 4 ? 2 : G == 2 ? 1 : 0;
  constexpr uint32_t NG = 64 / G;
  constexpr uint32_t kStep = NG * C;  // chunks per wave step
  constexpr int kRed = (1 + kLevels) * 1024;
  constexpr uint64_t kQ = 16u * G;
  __shared__ alignas(16) uint32_t lds[kUniLdsWords + kRed];
  __shared__ uint32_t wg_next;
  {
    const uint32_t(*tab)[256] = kQ == 256 ? pc->tabq : kQ == 128 ? pc->tabo : kQ == 64 ? pc->tabf : kQ == 32 ? pc->tab2 : pc->tab1;
    if constexpr (kUniCopies == 16) {
      for (int i = threadIdx.x; i < kUniLdsWords; i += kUniThreads) lds[i] = fill_value16_of(tab, i);
      const uint32_t *red_g = &pc->red[0][0][0];
      for (int i = threadIdx.x; i < kRed; i += kUniThreads) lds[kUniLdsWords + i] = red_g[i];
    } else {
      fill_tables(lds, tab, &pc->red[0][0][0], kRed, threadIdx.x, kUniThreads);
    }
  }
  const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
  // The workgroup owns a contiguous range; its waves take steps of kStep chunks from an LDS
  // counter, so a wave slowed by its neighbours does not leave the others idle at the end
  // (a static split per wave kept waves alive 81 % of the kernel at 8 lanes per chunk).
  const uint32_t wlo = (uint32_t)((uint64_t)blockIdx.x * nchunks / gridDim.x);
  const uint32_t hi = (uint32_t)((uint64_t)(blockIdx.x + 1) * nchunks / gridDim.x);
  if (threadIdx.x == 0) wg_next = wlo;
  __syncthreads();
  auto grab = [&]() -> uint32_t {
    uint32_t q = 0;
    if (lane == 0) q = atomicAdd(&wg_next, kStep);
    return (uint32_t)__builtin_amdgcn_readfirstlane(q);
  };
  const uint32_t lo = grab();
  if (lo >= hi) return;
  const uint32_t *red = lds + kUniLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const LaneLut L = kUniCopies == 16 ? make_lut16(lane) : make_lut(lane);
  // step q (chunks q .. q + kStep - 1; this group's j-th is q + grp + j * NG): its first row
  // address for this lane, its result index and expected value
  auto quad = [&](uint32_t q, uint32_t j, uint64_t &la, uint32_t &o, uint32_t &want, bool &valid) {
    const uint32_t t = q + grp + j * NG;
    valid = t < hi;
    uint64_t p = 0;
    o = t;
    if (valid) {
      if (chunks) {
        p = chunks[t].ptr;
        o = chunks[t].out_idx;
      } else {
        p = base + (uint64_t)t * stride;
      }
    }
    la = p + 16u * gl;
    want = valid && expected ? expected[o] : 0u;
  };
  uint64_t la[C];
  uint32_t o[C], want[C];
  bool valid[C];
#pragma unroll
  for (int j = 0; j < C; ++j) quad(lo, j, la[j], o[j], want[j], valid[j]);
  uint4 cur[C][kUniBatch], nxt[C][kUniBatch];
#pragma unroll
  for (int j = 0; j < C; ++j)
#pragma unroll
    for (int b = 0; b < kUniBatch; ++b)
      cur[j][b] = valid[j] && (uint32_t)b < K ? load_row_w<kQ * C>(la[j] + (uint64_t)b * kQ) : make_uint4(0, 0, 0, 0);
  for (uint32_t q0 = lo; q0 < hi;) {
    const uint32_t qn = grab();  // the next step, taken now so its rows load during this one's last batch
    uint64_t la1[C];
    uint32_t o1[C], want1[C];
    bool valid1[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      la1[j] = la[j];
      o1[j] = o[j];
      want1[j] = want[j];
      valid1[j] = false;
      if (qn < hi) quad(qn, j, la1[j], o1[j], want1[j], valid1[j]);  // its rows load during this step's last batch
    }
    Streams st[C];
#pragma unroll
    for (int j = 0; j < C; ++j) st[j] = Streams{0, 0, 0, 0};
    for (uint32_t u0 = 0; u0 < K; u0 += kUniBatch) {
      const uint32_t n0 = u0 + kUniBatch;
      if (n0 < K) {
#pragma unroll
        for (int b = 0; b < kUniBatch; ++b)
#pragma unroll
          for (int j = 0; j < C; ++j)
            nxt[j][b] = valid[j] && n0 + b < K ? load_row_w<kQ * C>(la[j] + (uint64_t)(n0 + b) * kQ) : make_uint4(0, 0, 0, 0);
      } else {
#pragma unroll
        for (int b = 0; b < kUniBatch; ++b)
#pragma unroll
          for (int j = 0; j < C; ++j)
            nxt[j][b] = valid1[j] && (uint32_t)b < K ? load_row_w<kQ * C>(la1[j] + (uint64_t)b * kQ) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int b = 0; b < kUniBatch; ++b)
        if (u0 + b < K) {
#pragma unroll
          for (int j = 0; j < C; ++j) {
            if constexpr (kUniCopies == 16)
              consume16(st[j], cur[j][b], lb, L);
            else
              consume(st[j], cur[j][b], lb, L);
          }
        }
#pragma unroll
      for (int j = 0; j < C; ++j)
#pragma unroll
        for (int b = 0; b < kUniBatch; ++b) cur[j][b] = nxt[j][b];
    }
    uint32_t v[C];
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = tab_mul(st[j].s3, red) ^ st[j].s2;
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = tab_mul(v[j], red) ^ st[j].s1;
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = tab_mul(v[j], red) ^ st[j].s0;
#pragma unroll
    for (int k = 0; k < kLevels; ++k) {
      uint32_t x[C];
#pragma unroll
      for (int j = 0; j < C; ++j) x[j] = (uint32_t)__shfl_down((int)v[j], 1u << k, G);
      if ((gl & ((2u << k) - 1u)) == 0) {
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] ^= tab_mul(x[j], red + 1024 * (k + 1));
      }
    }
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (gl == 0 && valid[j]) {
        const uint32_t raw = v[j] ^ xs;
        out_raw[o[j]] = raw;
        if (expected) {
          const bool good = raw == want[j];
          ok[o[j]] = good ? 1 : 0;
          if (!good && mismatch) atomicAdd(mismatch, 1u);
        }
      }
      la[j] = la1[j];
      o[j] = o1[j];
      want[j] = want1[j];
      valid[j] = valid1[j];
    }
    q0 = qn;
  }
}
template <int G, int C = 1>
__global__ __launch_bounds__(kUniThreads, kUniCopies == 16 ? 6 : 1) void seg_uni_kernel(const DevChunk *__restrict__ chunks, uint64_t base,
                                                          uint64_t stride, uint32_t nchunks, uint32_t K, uint32_t xs,
                                                          const PolyConsts *__restrict__ pc,
                                                          const uint32_t *__restrict__ expected,
                                                          uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                          uint32_t *__restrict__ mismatch,
                                                                                        unsigned long long *ts) {  // ts: h3c_rt::prof_stamp's slot, or nullptr
  stamp_begin(ts);
  seg_uni_kernel_body<G, C>(chunks, base, stride, nchunks, K, xs, pc, expected, out_raw, ok, mismatch);
  stamp_end(ts);
}

// Kernel A''': CRCs of ranges listed in device memory, without host-built descriptors (the
// device-resident h3c_update_ios pipeline: UpdateIO payloads, and chunks CRC'd before a batch).
// Piece k of item i is [4096 j, min(4096 (j+1), len)) of item i's range, where pbase[i] <= k <
// pbase[i] + pieces(i) and j = k - pbase[i]; the piece count lives in device memory (*d_total).
// A group of 4 lanes owns a piece and walks it in 64-byte rows like seg_quad_kernel<4,1>; the
// piece's init-0 CRC, moved to the end of its item (x^(8 (len - piece end))), is XORed into
// crc0_out[i], which the caller zeroes.  Src::range(i, ptr, len) names item i's bytes.
struct UioPieceSrc {  // UpdateIO payloads (items < n), then chunk contents [0, size) (item n + c)
  const h3c_update_io *ios;
  const h3c_chunk_state *chunks;
  uint32_t n;
  __device__ void range(uint32_t i, uint64_t &ptr, uint32_t &len) const {
    if (i < n) {
      ptr = ios[i].payload;
      len = ios[i].length;
    } else {
      ptr = chunks[i - n].base;
      len = chunks[i - n].size;
    }
  }
};

template <class Src>
__global__ __launch_bounds__(kThreads) void op_piece_crc_kernel(Src src, const uint32_t *__restrict__ pbase, uint32_t n,
                                                                const uint32_t *__restrict__ d_total,
                                                                const PolyConsts *__restrict__ pc,
                                                                uint32_t *__restrict__ crc0_out,
                                                                const uint32_t *__restrict__ tbase, uint32_t tshift,
                                                                uint32_t *err) {
  constexpr int G = 4, kLevels = 2, NG = 64 / G;
  constexpr uint64_t kQ = 16u * G;
  constexpr int kRed = (1 + kLevels) * 1024;
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRed];
  const uint32_t total = *d_total;
  // Each workgroup owns a contiguous range; one with none returns before filling its tables (a
  // pass with few or no pieces -- the UpdateIO late pass, usually empty -- costs a launch only).
  const uint32_t wlo = (uint32_t)((uint64_t)blockIdx.x * total / gridDim.x);
  const uint32_t whi = (uint32_t)((uint64_t)(blockIdx.x + 1) * total / gridDim.x);
  if (wlo >= whi) return;
  fill_tables(lds, pc->tabf, &pc->red[0][0][0], kRed, threadIdx.x, kThreads);
  __syncthreads();
  const uint32_t *red = lds + kLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
  const uint32_t poly = pc->poly;
  const LaneLut L = make_lut(lane);
  // Its waves take steps of NG pieces from an LDS counter (a static split per wave left a third
  // of the waves with one step more than the rest at a few steps per wave; one global counter
  // serialised thousands of atomics).
  __shared__ uint32_t wg_next;
  if (threadIdx.x == 0) wg_next = wlo;
  __syncthreads();
  for (;;) {
    uint32_t q0 = 0;
    if (lane == 0) q0 = atomicAdd(&wg_next, (uint32_t)NG);
    q0 = (uint32_t)__builtin_amdgcn_readfirstlane(q0);
    if (q0 >= whi) break;
    const uint32_t k = q0 + grp;
    bool valid = k < whi;
    uint64_t S = 0, E = 0;
    uint32_t op = 0, shift = 0;
    if (valid) {  // op i: the last with pbase[i] <= k (pieces of ops with none are skipped over)
      // first guess: one piece per op (payloads of at most 4 KiB, BASELINE config 3), two
      // independent loads; otherwise a binary search (pbase[n] is the total, > k)
      // (with `tbase`, item i's offset is pbase[i] + tbase[i >> tshift]: the prep kernel's two-level scan)
      auto at = [&](uint32_t m) -> uint32_t { return pbase[m] + (tbase ? tbase[m >> tshift] : 0u); };
      uint32_t a = min(k, n - 1);
      if (!(at(a) <= k && at(a + 1) > k)) {
        a = 0;
        uint32_t b = n;
        while (b - a > 1) {
          const uint32_t m = (a + b) >> 1;
          if (at(m) <= k) a = m; else b = m;
        }
      }
      op = a;
      const uint32_t j = k - at(a);
      uint64_t base;
      uint32_t length;
      src.range(a, base, length);
      if ((uint64_t)j * 4096u < length) {
        const uint32_t off = j * 4096u, plen = min(4096u, length - off);
        S = base + off;
        E = S + plen;
        shift = length - off - plen;
      } else {  // a piece table that disagrees with the items: read nothing, and fail the call
        valid = false;
        if (err) atomicOr(err, 1u);
      }
    }
    const uint64_t base = S & ~(kQ - 1);
    const uint64_t la = base + 16u * gl;
    const uint32_t K = valid ? (uint32_t)((E - base + kQ - 1) / kQ) : 0u;
    uint32_t kmax = 0;
#pragma unroll
    for (uint32_t g = 0; g < (uint32_t)NG; ++g) kmax = max(kmax, (uint32_t)__builtin_amdgcn_readlane(K, g * G));
    Streams st{0, 0, 0, 0};
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) cur[b] = (uint32_t)b < K ? load_row_w<kQ>(la + (uint64_t)b * kQ) : make_uint4(0, 0, 0, 0);
    for (uint32_t u0 = 0; u0 < kmax; u0 += 4) {
      const uint32_t n0 = u0 + 4;
#pragma unroll
      for (int b = 0; b < 4; ++b) nxt[b] = n0 + b < K ? load_row_w<kQ>(la + (uint64_t)(n0 + b) * kQ) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t u = u0 + b;
        if (u < K) {
          uint4 x = cur[b];
          if ((u == 0 && (S & (kQ - 1))) || (u + 1 == K && (E & (kQ - 1)))) x = mask_row(x, la + (uint64_t)u * kQ, S, E);
          consume(st, x, lb, L);
        }
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) cur[b] = nxt[b];
    }
    uint32_t v = tab_mul(st.s3, red) ^ st.s2;
    v = tab_mul(v, red) ^ st.s1;
    v = tab_mul(v, red) ^ st.s0;
#pragma unroll
    for (int lv = 0; lv < kLevels; ++lv) {
      const uint32_t o = (uint32_t)__shfl_down((int)v, 1u << lv, G);
      if ((gl & ((2u << lv) - 1u)) == 0) v ^= tab_mul(o, red + 1024 * (lv + 1));
    }
    if (gl == 0 && valid) {
      const uint32_t pad = (uint32_t)(((E + kQ - 1) & ~(kQ - 1)) - E);
      if (pad >> 4) v = dgf_mul(v, pc->fix[4 * (pad >> 4)], poly);
      if (pad & 15) v = dgf_mul(v, pc->fixz[pad & 15], poly);
      if (shift) v = dgf_mul_fast(v, dxpow8_fast(shift, pc, poly), poly);
    }
    // The step's NG pieces are consecutive, so their items never decrease: the pieces of one item form a run of
    // groups, XORed together (a suffix scan over the groups) and sent by the run's first group as one atomic.
    // (A 64 MiB chunk is 16,384 pieces: one atomic each on one address serialised the pass, ~3.4 ms for 4 GiB.)
    uint32_t x = gl == 0 && valid ? v : 0u;
    const uint32_t myop = valid ? op : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t d = 1; d < (uint32_t)NG; d <<= 1) {
      const uint32_t xo = (uint32_t)__shfl_down((int)x, G * d, 64);
      const uint32_t oo = (uint32_t)__shfl_down((int)myop, G * d, 64);
      if (grp + d < (uint32_t)NG && oo == myop) x ^= xo;
    }
    const uint32_t prev_op = (uint32_t)__shfl_up((int)myop, G, 64);
    if (gl == 0 && valid && (grp == 0 || prev_op != myop)) atomicXor(&crc0_out[op], x);
  }
}

// Kernel B: per chunk, fold segment CRCs, apply start, optionally compare.
// Chunks with more segments than this are folded by a whole wave (finalize_kernel's second mapping).
constexpr uint32_t kSmallFold = 16;

__device__ __forceinline__ void finalize_store(const DevChunk &ch, uint32_t raw, const uint32_t *__restrict__ expected,
                                               uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                               uint32_t *__restrict__ mismatch) {
  out_raw[ch.out_idx] = raw;
  if (expected) {
    const bool good = raw == expected[ch.out_idx];
    ok[ch.out_idx] = good ? 1 : 0;
    if (!good && mismatch) atomicAdd(mismatch, 1u);
  }
}

// Byte tables of the multiply by X = x^(8*seg_bytes) (the fold of full segments), built
// per workgroup in LDS: tab_mul(h, T) = h * X with 4 lookups instead of a ~200-op
// bit-serial multiply.
__device__ __forceinline__ void build_seg_table(uint32_t *T, uint32_t seg_mul, uint32_t poly) {
  for (uint32_t k = threadIdx.x; k < 1024; k += blockDim.x) T[k] = dgf_mul((k & 255u) << (8 * (k >> 8)), seg_mul, poly);
  __syncthreads();
}

// Kernel B: per chunk, fold segment CRCs, apply start, optionally compare; one launch, two
// mappings.  Blocks [0, small_blocks): one thread per chunk of <= kSmallFold segments.  The rest:
// one wave per chunk of more (a thread folding thousands of segments serially took ~1 ms for a
// 64 MiB chunk): the full segments' CRCs are the coefficients of a polynomial in X =
// x^(8*seg_bytes); lane j Horner-evaluates q consecutive coefficients (virtual zeros in front are
// harmless), multiplies its sum by its own shift X^(q*(63-j)) * x^(8r) (r the last segment's
// length; two table words and one multiply), and the lanes XOR-reduce: two multiplies on the
// critical path where a butterfly over the lanes takes twelve.  Every load a chunk's fold needs
// (its segment CRCs, the expected value, the lane's shift words) is issued before the table
// build, so the fold's latency is one round trip, not a chain of them.
constexpr uint32_t kBigBatch = 8;  // segment CRCs a lane loads per round trip

__global__ __launch_bounds__(256) void finalize_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                       uint32_t total_segs, uint64_t seg_bytes, uint32_t seg_mul,
                                                       uint32_t need_table, uint32_t small_blocks,
                                                       const PolyConsts *__restrict__ pc,
                                                       const uint32_t *__restrict__ seg_crc,
                                                       const uint32_t *__restrict__ expected,
                                                       uint32_t *__restrict__ out_raw, uint8_t *__restrict__ ok,
                                                       uint32_t *__restrict__ mismatch) {
  __shared__ uint32_t T[1024];
  const uint32_t poly = pc->poly;
  if (blockIdx.x < small_blocks) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    DevChunk ch{};
    uint32_t m = 0, sc[kSmallFold], last = 0, ex = 0;
    bool mine = false;
    if (i < nchunks) {
      ch = chunks[i];
      const uint32_t e = (i + 1 < nchunks) ? chunks[i + 1].seg_begin : total_segs;
      m = e - ch.seg_begin;
      mine = m <= kSmallFold || (ch.flags & kFlagNone);  // (else the wave mapping's)
      if (mine && !(ch.flags & kFlagNone)) {
#pragma unroll
        for (uint32_t t = 0; t < kSmallFold; ++t) sc[t] = t + 1 < m ? seg_crc[ch.seg_begin + t] : 0u;
        if (m) last = seg_crc[e - 1];
      }
      if (mine && expected) ex = expected[ch.out_idx];
    }
    if (need_table) build_seg_table(T, seg_mul, poly);  // only chunks of >= 3 segments use it
    if (!mine) return;
    uint32_t raw = 0;
    if (!(ch.flags & kFlagNone)) {
      uint32_t crc0 = 0;
      if (m == 1) crc0 = last;
      if (m >= 2) {
        crc0 = sc[0];
#pragma unroll
        for (uint32_t t = 1; t + 1 < kSmallFold; ++t)
          if (t + 1 < m) crc0 = tab_mul(crc0, T) ^ sc[t];  // full segments
        crc0 = dgf_mul(crc0, ch.xlast, poly) ^ last;       // the last one
      }
      raw = crc0 ^ ch.xstart;
    }
    out_raw[ch.out_idx] = raw;
    if (expected) {
      const bool good = raw == ex;
      ok[ch.out_idx] = good ? 1 : 0;
      if (!good && mismatch) atomicAdd(mismatch, 1u);
    }
    return;
  }
  const uint32_t i = __builtin_amdgcn_readfirstlane((blockIdx.x - small_blocks) * (blockDim.x / 64) + (threadIdx.x >> 6));
  const uint32_t j = threadIdx.x & 63;
  DevChunk ch{};
  uint32_t b = 0, m = 0, q = 0, last = 0, ex = 0, ya = kOne, yb = kOne;
  uint32_t sc[kBigBatch];
  int64_t k0 = 0;
  bool mine = false;
  if (i < nchunks) {
    ch = chunks[i];
    b = ch.seg_begin;
    const uint32_t e = (i + 1 < nchunks) ? chunks[i + 1].seg_begin : total_segs;
    m = e - b;
    mine = m > kSmallFold && !(ch.flags & kFlagNone);
  }
  if (mine) {
    q = (m - 1 + 63) / 64;
    k0 = (int64_t)(m - 1) - (int64_t)(64 - j) * q;
#pragma unroll
    for (uint32_t t = 0; t < kBigBatch; ++t) sc[t] = t < q && k0 + t >= 0 ? seg_crc[b + (uint32_t)(k0 + t)] : 0u;
    last = seg_crc[b + m - 1];
    if (expected) ex = expected[ch.out_idx];
    const uint64_t e8 = (uint64_t)(63 - j) * q * seg_bytes + (ch.len - (uint64_t)(m - 1) * seg_bytes);
    if (e8 < (1ull << 26)) {  // the lane's shift x^(8 e8): two table words, one multiply
      ya = pc->x4k[e8 >> 12];
      yb = pc->xb[e8 & 4095];
    }
  }
  build_seg_table(T, seg_mul, poly);
  if (!mine) return;
  uint32_t h = 0;
  for (uint32_t t0 = 0; t0 < q; t0 += kBigBatch) {
    if (t0) {
#pragma unroll
      for (uint32_t t = 0; t < kBigBatch; ++t) {
        const int64_t k = k0 + t0 + t;
        sc[t] = t0 + t < q && k >= 0 ? seg_crc[b + (uint32_t)k] : 0u;
      }
    }
#pragma unroll
    for (uint32_t t = 0; t < kBigBatch; ++t)
      if (t0 + t < q) h = tab_mul(h, T) ^ sc[t];
  }
  const uint64_t e8 = (uint64_t)(63 - j) * q * seg_bytes + (ch.len - (uint64_t)(m - 1) * seg_bytes);
  h = dgf_mul_fast(h, e8 < (1ull << 26) ? dgf_mul_fast(ya, yb, poly) : dxpow8n(e8, pc, poly), poly);
#pragma unroll
  for (int t = 0; t < 6; ++t) h ^= (uint32_t)__shfl_xor((int)h, 1 << t, 64);
  if (j == 0) {
    const uint32_t raw = (h ^ last) ^ ch.xstart;
    out_raw[ch.out_idx] = raw;
    if (expected) {
      const bool good = raw == ex;
      ok[ch.out_idx] = good ? 1 : 0;
      if (!good && mismatch) atomicAdd(mismatch, 1u);
    }
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
uint64_t pick_seg_bytes(uint64_t total_bytes, int num_cu);

void set_error(const char *what, hipError_t e) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  g_last_error = buf;
}

struct DeviceCtx {
  std::once_flag once;
  int status = H3C_ERR_NO_DEVICE;
  PolyConsts *d_consts[2] = {nullptr, nullptr};  // [0] CRC32C, [1] CRC32
  int num_cu = 0;
  int wall_khz = 0;  // wall_clock64() rate
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
      if (hipDeviceGetAttribute(&ctx.wall_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) {
        ctx.wall_khz = 0;  // the in-graph UpdateIO block kernel then goes untimed
        (void)hipGetLastError();
      }
      const uint32_t polys[2] = {kPolyCrc32c, kPolyCrc32};
      std::vector<PolyConsts> h(1);  // ~130 KiB: not on the caller's stack
      for (int i = 0; i < 2; ++i) {
        build_consts(h[0], polys[i]);
        HIP_TRY(hipMalloc(&ctx.d_consts[i], sizeof(PolyConsts)));
        HIP_TRY(hipMemcpy(ctx.d_consts[i], h.data(), sizeof(PolyConsts), hipMemcpyHostToDevice));
      }
      return H3C_OK;
    };
    ctx.status = body();
    (void)hipSetDevice(prev);
  });
  return ctx.status;
}

// The device count, queried once per process (the set of visible devices does not change).
int device_count() {
  static const int n = [] {
    int k = 0;
    return hipGetDeviceCount(&k) == hipSuccess ? k : 0;
  }();
  return n;
}

int current_device(int *dev) {
  if (device_count() <= 0) {
    g_last_error = "no HIP device";
    return H3C_ERR_NO_DEVICE;
  }
  HIP_TRY(hipGetDevice(dev));
  return init_device(*dev);
}

// h3c_test_hook state: read from the environment once, settable by tests.
constexpr int kHooks = 11;
std::atomic<uint64_t> g_hooks[kHooks];
const bool g_hooks_init = [] {
  const char *names[kHooks] = {nullptr, "H3C_SEG_BYTES", "H3C_DEBUG_FLAGS", "H3C_UPD_SCAN", "H3C_UPD_GRAPHS",
                                "H3C_UPD_LOOKBACK", "H3C_UPD_FRONT", "H3C_UPD_FAST", "H3C_UPD_GIVEUP",
                                "H3C_FAST_POLL_US", "H3C_UPD_ALIGNED"};
  for (int k = 1; k < kHooks; ++k) {
    uint64_t v = 0;
    if (const char *e = std::getenv(names[k])) {
      if (k == H3C_HOOK_UPD_SCAN)
        v = std::strcmp(e, "fused") == 0 ? 1 : std::strcmp(e, "tiles") == 0 ? 2 : std::strcmp(e, "sort") == 0 ? 3 : 0;
      else
        v = std::strtoull(e, nullptr, 0);
    }
    g_hooks[k].store(v);
  }
  return true;
}();

}  // namespace

namespace h3c_rt {
const void *device_consts(int dev, int type) {
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  return g_dev[dev].d_consts[type == H3C_TYPE_CRC32 ? 1 : 0];
}
int device_num_cu(int dev) { return (dev >= 0 && dev < kMaxDevices) ? g_dev[dev].num_cu : 0; }
int device_wall_clock_khz(int dev) { return (dev >= 0 && dev < kMaxDevices) ? g_dev[dev].wall_khz : 0; }
uint64_t hook(int key) { return (key > 0 && key < kHooks) ? g_hooks[key].load(std::memory_order_relaxed) : 0; }
std::shared_mutex &capture_gate() {
  static std::shared_mutex m;
  return m;
}
int current_device(int *dev) { return ::current_device(dev); }
void set_error(const char *what, hipError_t e) { ::set_error(what, e); }
void set_error_text(const char *text) { g_last_error = text; }
}  // namespace h3c_rt

namespace {

// ---- profiling: the hot kernels' own wall-clock stamps (or event pairs), per kind ----
struct ProfRec {
  hipEvent_t a, b;  // (event records)
  uint64_t bytes;
  int kind;
  int dev = -1, slot = -1;  // (stamp records: a slot of the device's stamp pool)
};
// Per device: kProfSlots stamp slots {first start, last end}, {~0, 0} when free; handed out in
// order between h3c_profile_read calls (which read them back and free them).  A launch past the
// last slot is not timed.
constexpr int kProfSlots = 8192;
struct StampPool {
  unsigned long long *d = nullptr;
  int next = 0;
};
constexpr int kProfKinds = 4;
constexpr int kProfCancelled = -3;  // a stamp record whose launch never happened (ProfToken's early return)
std::mutex g_prof_mu;
std::vector<ProfRec> g_prof;
StampPool g_stamps[kMaxDevices];
std::atomic<int> g_prof_on{0};
double g_prof_ms_done[kProfKinds] = {0, 0, 0, 0};
uint64_t g_prof_launch_done[kProfKinds] = {0, 0, 0, 0}, g_prof_bytes_done[kProfKinds] = {0, 0, 0, 0};

}  // namespace

namespace {
std::mutex g_pin_mu;
std::vector<std::pair<char *, size_t>> g_pin_free;  // pooled pinned buffers
constexpr size_t kPinPoolMax = 256u << 20;            // larger leases are freed, not pooled
}  // namespace

namespace {
std::mutex g_dev_pool_mu;
std::vector<std::pair<char *, size_t>> g_dev_pool[kMaxDevices];
constexpr size_t kDevPoolMax = 1ull << 30;  // larger leases are freed, not pooled
}  // namespace

namespace h3c_rt {
DeviceLease::DeviceLease(int dev, size_t bytes) : dev_(dev) {
  bytes = std::max<size_t>(bytes, 4096);
  if (dev < 0 || dev >= kMaxDevices) return;
  {
    std::lock_guard<std::mutex> lk(g_dev_pool_mu);
    auto &pool = g_dev_pool[dev];
    // best fit, the most recently returned first among equal sizes: a caller that repeats a
    // call gets the same buffers back when nothing else leased meanwhile
    size_t best = pool.size();
    for (size_t i = pool.size(); i-- > 0;)
      if (pool[i].second >= bytes && (best == pool.size() || pool[i].second < pool[best].second)) best = i;
    if (best != pool.size()) {
      p_ = pool[best].first;
      cap_ = pool[best].second;
      pool.erase(pool.begin() + (ptrdiff_t)best);
      return;
    }
  }
  const size_t cap = (bytes + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
  const hipError_t e = hipMalloc(reinterpret_cast<void **>(&p_), cap);
  if (e != hipSuccess) {
    set_error("hipMalloc (scratch)", e);
    p_ = nullptr;
    return;
  }
  cap_ = cap;
}
DeviceLease::~DeviceLease() {
  if (!p_) return;
  if (cap_ > kDevPoolMax) {
    (void)hipFree(p_);
    return;
  }
  std::lock_guard<std::mutex> lk(g_dev_pool_mu);
  g_dev_pool[dev_].emplace_back(p_, cap_);
}

PinnedLease::PinnedLease(size_t bytes) {
  bytes = std::max<size_t>(bytes, 4096);
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    size_t best = g_pin_free.size();  // best fit, most recently returned first (as DeviceLease)
    for (size_t i = g_pin_free.size(); i-- > 0;)
      if (g_pin_free[i].second >= bytes && (best == g_pin_free.size() || g_pin_free[i].second < g_pin_free[best].second))
        best = i;
    if (best != g_pin_free.size()) {
      p_ = g_pin_free[best].first;
      cap_ = g_pin_free[best].second;
      g_pin_free.erase(g_pin_free.begin() + (ptrdiff_t)best);
      return;
    }
  }
  const size_t cap = (bytes + (1u << 20) - 1) & ~size_t((1u << 20) - 1);
  const hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&p_), cap, 0);
  if (e != hipSuccess) {
    set_error("hipHostMalloc (staging)", e);
    p_ = nullptr;
    return;
  }
  cap_ = cap;
}
PinnedLease::~PinnedLease() {
  if (!p_) return;
  if (cap_ > kPinPoolMax) {
    (void)hipHostFree(p_);
    return;
  }
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_free.emplace_back(p_, cap_);
}

hipError_t prof_begin(hipStream_t st, ProfToken &t) {
  t.on = g_prof_on.load() != 0;
  if (!t.on) return hipSuccess;
  hipError_t e = hipEventCreate(&t.a);
  if (e == hipSuccess) e = hipEventCreate(&t.b);
  if (e == hipSuccess) e = hipEventRecord(t.a, st);
  return e;
}
hipError_t prof_stamp(int dev, ProfToken &t) {
  t.on = g_prof_on.load() != 0;
  t.ts = nullptr;
  if (!t.on || dev < 0 || dev >= kMaxDevices) return hipSuccess;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  StampPool &p = g_stamps[dev];
  if (!p.d) {
    std::vector<unsigned long long> init(2 * kProfSlots);
    for (int i = 0; i < kProfSlots; ++i) init[2 * i] = ~0ull, init[2 * i + 1] = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&p.d), init.size() * 8);
    if (e == hipSuccess) e = hipMemcpy(p.d, init.data(), init.size() * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      p.d = nullptr;
      return e;
    }
  }
  if (p.next >= kProfSlots) return hipSuccess;  // (pool used up: this launch is not timed)
  t.dev = dev;
  t.slot = p.next++;
  t.ts = p.d + 2 * t.slot;
  // the slot's record exists from now on (kind -1 until prof_end fills it in), so that an
  // h3c_profile_read in between neither frees nor re-initialises a slot still in flight
  ProfRec r{nullptr, nullptr, 0, -1};
  r.dev = dev;
  r.slot = t.slot;
  g_prof.push_back(r);
  return hipSuccess;
}
void prof_cancel(const ProfToken &t) {
  t.closed = true;
  if (t.ts) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (size_t i = g_prof.size(); i-- > 0;)
      if (g_prof[i].kind == -1 && g_prof[i].dev == t.dev && g_prof[i].slot == t.slot) {
        g_prof[i].kind = kProfCancelled;
        break;
      }
  }
  if (t.a) (void)hipEventDestroy(t.a);
  if (t.b) (void)hipEventDestroy(t.b);
}
hipError_t prof_end(hipStream_t st, const ProfToken &t, int kind, uint64_t bytes) {
  t.closed = true;
  if (!t.on) return hipSuccess;
  if (t.ts) {  // stamped by the kernel itself: its pending record gets its kind and bytes
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (size_t i = g_prof.size(); i-- > 0;)
      if (g_prof[i].kind == -1 && g_prof[i].dev == t.dev && g_prof[i].slot == t.slot) {
        g_prof[i].kind = kind;
        g_prof[i].bytes = bytes;
        break;
      }
    return hipSuccess;
  }
  if (!t.a) return hipSuccess;  // (a stamped launch with no slot left)
  hipError_t e = hipEventRecord(t.b, st);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof.push_back(ProfRec{t.a, t.b, bytes, kind});
  return e;
}

bool prof_enabled() { return g_prof_on.load() != 0; }
void prof_add(int kind, float ms, uint64_t bytes) {
  if (kind < 0 || kind >= kProfKinds) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_ms_done[kind] += ms;
  g_prof_launch_done[kind] += 1;
  g_prof_bytes_done[kind] += bytes;
}

int launch_crc(hipStream_t st, int dev, int type, const DevChunk *d_chunks, uint32_t nchunks, uint32_t total_segs,
               uint32_t max_chunk_segs, uint64_t payload_bytes, uint64_t seg_bytes, uint32_t dbg, uint32_t *d_segcrc,
               const uint32_t *expected, uint32_t *out_raw, uint8_t *ok, uint32_t *mismatch, int prof_kind,
               uint32_t small_rows, const UniformBatch *uni) {
  const DeviceCtx &ctx = g_dev[dev];
  const PolyConsts *pc = ctx.d_consts[type == H3C_TYPE_CRC32 ? 1 : 0];
  const uint32_t poly = type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;
  if (small_rows && nchunks && !(dbg & 2u)) {  // test hook: H3C_DEBUG_FLAGS bit1 disables it
    const uint32_t blocks = std::min<uint32_t>(ctx.num_cu, (nchunks + kWavesPerBlock - 1) / kWavesPerBlock);
    ProfToken tok;
    if (prof_kind >= 0) HIP_TRY(prof_stamp(dev, tok));
    if (uni && uni->lanes && !(dbg & 4u)) {  // test hook: H3C_DEBUG_FLAGS bit2 disables it
      const DevChunk *dc = uni->contiguous ? nullptr : d_chunks;
      const uint32_t ublocks = std::min<uint32_t>(ctx.num_cu * (kUniCopies == 16 ? 2 : 1),
                                                  (nchunks + kUniWaves - 1) / kUniWaves);
      if (uni->lanes == 1)
        hipLaunchKernelGGL(seg_uni_kernel<1>, dim3(ublocks), dim3(kUniThreads), 0, st, dc, uni->base, uni->stride,
                           nchunks, uni->rows, uni->xs, pc, expected, out_raw, ok, mismatch, tok.ts);
      else if (uni->lanes == 2)
        hipLaunchKernelGGL(seg_uni_kernel<2>, dim3(ublocks), dim3(kUniThreads), 0, st, dc, uni->base, uni->stride,
                           nchunks, uni->rows, uni->xs, pc, expected, out_raw, ok, mismatch, tok.ts);
      else if (uni->lanes == 4)
        hipLaunchKernelGGL(seg_uni_kernel<4>, dim3(ublocks), dim3(kUniThreads), 0, st, dc, uni->base, uni->stride,
                           nchunks, uni->rows, uni->xs, pc, expected, out_raw, ok, mismatch, tok.ts);
      else if (uni->lanes == 8)
        hipLaunchKernelGGL(seg_uni_kernel<8>, dim3(ublocks), dim3(kUniThreads), 0, st, dc, uni->base, uni->stride,
                           nchunks, uni->rows, uni->xs, pc, expected, out_raw, ok, mismatch, tok.ts);
      else
        hipLaunchKernelGGL(seg_uni_kernel<16>, dim3(ublocks), dim3(kUniThreads), 0, st, dc, uni->base, uni->stride,
                           nchunks, uni->rows, uni->xs, pc, expected, out_raw, ok, mismatch, tok.ts);
    } else if (small_rows <= 6) {
      // up to ~5 KiB chunks 4 lanes per chunk (4 KiB: +8 % over 8 lanes, +13 % over 16);
      // 16 lanes above (4 lanes lose 10 % at 8 and 16 KiB): profiles/r01d_small_lanes_ab.txt
      hipLaunchKernelGGL((seg_quad_kernel<H3C_SMALL_LANES_LO, H3C_SMALL_PIECES_LO>), dim3(blocks), dim3(kThreads), 0, st, d_chunks, nchunks,
                         pc, expected, out_raw, ok, mismatch, tok.ts);
    } else {
      hipLaunchKernelGGL((seg_quad_kernel<H3C_SMALL_LANES_HI, H3C_SMALL_PIECES_HI>), dim3(blocks), dim3(kThreads), 0, st, d_chunks, nchunks, pc, expected,
                         out_raw, ok, mismatch, tok.ts);
    }
    HIP_TRY(hipGetLastError());
    if (prof_kind >= 0) HIP_TRY(prof_end(st, tok, prof_kind, payload_bytes));
    return H3C_OK;
  }
  // every chunk exactly one segment: the segment kernel finishes the chunks (no finalize launch)
  const bool fin = total_segs && total_segs == nchunks && max_chunk_segs == 1;
  if (total_segs) {
    const uint32_t blocks = std::min<uint32_t>(ctx.num_cu, (total_segs + kWavesPerBlock - 1) / kWavesPerBlock);
    ProfToken tok;
    if (prof_kind >= 0) HIP_TRY(prof_stamp(dev, tok));
    hipLaunchKernelGGL(seg_crc_kernel, dim3(blocks), dim3(kThreads), 0, st, d_chunks, nchunks, total_segs, seg_bytes,
                       dbg, pc, d_segcrc, fin ? 1u : 0u, expected, out_raw, ok, mismatch, tok.ts);
    HIP_TRY(hipGetLastError());
    if (prof_kind >= 0) HIP_TRY(prof_end(st, tok, prof_kind, payload_bytes));
  }
  if (fin) return H3C_OK;
  const uint32_t seg_mul = hxpow8n(seg_bytes, poly);
  const uint32_t fb = (nchunks + 255) / 256;
  const uint32_t bb = max_chunk_segs > kSmallFold ? (nchunks + 3) / 4 : 0;  // 4 waves (chunks) per block
  hipLaunchKernelGGL(finalize_kernel, dim3(fb + bb), dim3(256), 0, st, d_chunks, nchunks, total_segs, seg_bytes,
                     seg_mul, max_chunk_segs >= 3 ? 1u : 0u, fb, pc, d_segcrc, expected, out_raw, ok, mismatch);
  HIP_TRY(hipGetLastError());
  return H3C_OK;
}

#ifndef H3C_PIECE_CU_PCT
#define H3C_PIECE_CU_PCT 100  // share of the CUs the UpdateIO payload-CRC kernel takes (A/B switch)
#endif
int launch_uio_piece_crc(hipStream_t st, int dev, int type, const h3c_update_io *ios, uint32_t n,
                         const h3c_chunk_state *chunks, uint32_t nchunks, const uint32_t *pbase,
                         const uint32_t *d_total, uint32_t *crc0_out, const uint32_t *tbase, uint32_t tile,
                         uint32_t *err) {
  const DeviceCtx &ctx = g_dev[dev];
  const PolyConsts *pc = ctx.d_consts[type == H3C_TYPE_CRC32 ? 1 : 0];
  hipLaunchKernelGGL(op_piece_crc_kernel<UioPieceSrc>, dim3(std::max(ctx.num_cu * H3C_PIECE_CU_PCT / 100, 1)),
                     dim3(kThreads), 0, st, UioPieceSrc{ios, chunks, n}, pbase, n + nchunks, d_total, pc, crc0_out, tbase,
                     tbase ? (uint32_t)__builtin_ctz(tile) : 0u, err);
  HIP_TRY(hipGetLastError());
  return H3C_OK;
}
template <>
struct ArgLayout<UioPieceSrc, void> {
  static void fill(ArgSpec &a) {
    struct_arg<UioPieceSrc>(a, {offsetof(UioPieceSrc, ios), offsetof(UioPieceSrc, chunks)});
  }
};
KernelSig uio_piece_kernel_sig() { return kernel_sig(op_piece_crc_kernel<UioPieceSrc>, "op_piece_crc_kernel<UioPieceSrc>"); }

// Chunks of at most this many 1 KiB rows take the small-chunk kernel when every chunk of
// the batch is one segment: seg_quad_kernel beats the segment kernel + finalize up to
// 16 KiB chunks and loses from 32 KiB (profiles/r01d_small_path_threshold.txt).
#ifndef H3C_SMALL_PATH_ROWS
#define H3C_SMALL_PATH_ROWS 16
#endif
constexpr uint32_t kSmallPathRows = H3C_SMALL_PATH_ROWS;

uint32_t small_rows_bound(uint64_t max_len, uint32_t max_segs) {
  // a range of len bytes touches at most floor(len / 1 KiB) + 2 rows of 1 KiB
  const uint64_t rows = max_len / 1024u + 2u;
  return max_segs == 1 && max_len && rows <= kSmallPathRows ? (uint32_t)rows : 0;
}

uint32_t small_rows_for(const DevChunk *c, size_t n, uint32_t max_segs) {
  if (!n || max_segs != 1) return 0;
  uint32_t rows = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t r = host_rows(c[i].ptr, c[i].len);
    if ((c[i].flags & kFlagNone) || c[i].len == 0 || r > kSmallPathRows) return 0;
    rows = std::max(rows, r);
  }
  return rows;
}

uint64_t pick_seg(uint64_t total_bytes, int dev) { return pick_seg_bytes(total_bytes, device_num_cu(dev)); }

void uniform_for(const DevChunk *c, size_t n, uint32_t small_rows, UniformBatch &u) {
  u = UniformBatch{};
  if (!n || !small_rows) return;
  uint32_t lanes = small_rows <= 6 ? H3C_UNI_LANES_LO : H3C_UNI_LANES_HI;
  if (lanes != 1 && lanes != 2 && lanes != 4 && lanes != 8 && lanes != 16) return;
  const uint64_t row = 16u * lanes, len = c[0].len;
  if (!len || len % row) return;
  const uint64_t stride = n > 1 ? c[1].ptr - c[0].ptr : len;
  bool contiguous = stride >= len && stride % row == 0;
  for (size_t i = 0; i < n; ++i) {
    if (c[i].len != len || (c[i].ptr % row) || (c[i].flags & kFlagNone) || c[i].xstart != c[0].xstart) return;
    contiguous = contiguous && c[i].out_idx == i && c[i].ptr == c[0].ptr + i * stride;
  }
  u.lanes = lanes;
  u.rows = (uint32_t)(len / row);
  u.xs = c[0].xstart;
  u.contiguous = contiguous;
  u.base = c[0].ptr;
  u.stride = stride;
}
}  // namespace h3c_rt

namespace {

// test hook H3C_HOOK_DEBUG_FLAGS: bit0 disables the pipelined row loop (read per plan)
uint32_t read_dbg_flags() { return (uint32_t)h3c_rt::hook(H3C_HOOK_DEBUG_FLAGS); }

// test hook H3C_HOOK_SEG_BYTES: force the segment size
uint64_t forced_seg(uint64_t seg) {
  const uint64_t v = h3c_rt::hook(H3C_HOOK_SEG_BYTES);
  return (v >= kRowBytes && v % kRowBytes == 0) ? v : seg;
}

struct Group {
  uint8_t type = H3C_TYPE_CRC32C;
  uint32_t nchunks = 0;
  uint32_t total_segs = 0;
  uint32_t max_chunk_segs = 0;
  uint64_t bytes = 0;
  uint32_t small = 0;  // seg_small_kernel rows (0: general kernels)
  h3c_rt::UniformBatch uni;
  DevChunk *d_chunks = nullptr;
};

uint64_t pick_seg_bytes(uint64_t total_bytes, int num_cu) {
  // Without the chunk lengths: aim for >= 8 segments per wave slot, within [16 KiB, 1 MiB].
  const uint64_t slots = (uint64_t)std::max(num_cu, 1) * kWavesPerBlock * 8;
  uint64_t want = total_bytes / slots;
  uint64_t seg = kMaxSegBytes;
  while (seg > kMinSegBytes && seg > want) seg >>= 1;
  return seg;
}

// With the chunk lengths: waves take contiguous segment ranges by count, so the
// slowest wave carries ceil(S / waves) segments.  Take the largest power of two in
// [16 KiB, 1 MiB] whose balance total / (waves * ceil(S / waves) * seg) is >= 97 %
// (larger segments mean fewer per-segment pipeline drains): 1 MiB for 8192 x 1 MiB
// chunks (exactly 2 per wave), 256 KiB for a mixed 64 KiB-64 MiB batch (with 1 MiB
// segments some waves got a third one: 6.2 vs 6.7 TB/s).
uint64_t pick_seg_for(const h3c_desc *d, size_t n, int num_cu) {
  const uint64_t waves = (uint64_t)std::max(num_cu, 1) * kWavesPerBlock;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i)
    if ((d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) && d[i].ptr) total += d[i].len;
  if (total == 0) return kMinSegBytes;
  // the segment size whose busiest wave finishes first: ceil(segs / waves) segments of `seg` bytes each,
  // plus a fixed cost per segment worth ~8 KiB of streaming (its fold and result).  Mixed 64 KiB-64 MiB
  // batches: 128 KiB (1.326 ms) against the balance-only rule's 64 KiB (1.341 ms), profiles/r06_mixed_seg.txt;
  // 1 MiB and 4 MiB chunks keep 1 MiB segments
  constexpr uint64_t kSegCost = 8u << 10;
  uint64_t best = kMinSegBytes, best_t = ~0ull;
  for (uint64_t seg = kMaxSegBytes; seg >= kMinSegBytes; seg >>= 1) {
    uint64_t segs = 0;
    for (size_t i = 0; i < n; ++i)
      if ((d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) && d[i].ptr) segs += (d[i].len + seg - 1) / seg;
    const uint64_t t = (segs + waves - 1) / waves * (seg + kSegCost);
    if (t < best_t) {
      best_t = t;
      best = seg;
    }
  }
  return best;
}

}  // namespace

namespace {
// Splits descriptors into one DevChunk list per polynomial with segment numbering;
// shared by h3c_plan_create and the synchronous batch path.
struct GroupLayout {
  std::vector<DevChunk> hc[2];
  uint32_t segs[2] = {0, 0}, max_segs[2] = {0, 0};
  uint64_t bytes[2] = {0, 0};
  // every chunk one short segment: its largest row count (seg_small_kernel), else 0
  uint32_t small[2] = {0, 0};
  h3c_rt::UniformBatch uni[2];
};

// Recomputes GroupLayout::small from the final device pointers.
void mark_small(GroupLayout &g) {
  for (int k = 0; k < 2; ++k) {
    g.small[k] = h3c_rt::small_rows_for(g.hc[k].data(), g.hc[k].size(), g.max_segs[k]);
    h3c_rt::uniform_for(g.hc[k].data(), g.hc[k].size(), g.small[k], g.uni[k]);
  }
}

// Extent check for device payloads: a descriptor whose bytes start inside a HIP allocation the
// runtime knows (hipMalloc'd memory, torch's caching-allocator segments) must end inside it, or
// the kernels would read unmapped memory and fault the device (round 2: a test plan's stride
// walked 8 MiB past its buffer).  Rejected with kInvalidArg before any launch.  Pointers the
// runtime cannot place (e.g. device addresses of registered host memory) are not checked.  The
// last allocation found is cached, so a batch inside one buffer costs one runtime query.
struct ExtentCheck {
  uint64_t lo = 1, hi = 0;  // empty
  bool ok(uint64_t p, uint64_t len) {
    if (p >= lo && p < hi) return len <= hi - p;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(p)) != hipSuccess || !base || !size) {
      (void)hipGetLastError();
      return true;  // unknown to the runtime: cannot check
    }
    lo = (uint64_t)(uintptr_t)base;
    hi = lo + size;
    return p >= lo && len <= hi - p;
  }
};

int layout_groups(const h3c_desc *d, size_t n, uint64_t seg_bytes, GroupLayout &g, bool check_extent = true) {
  ExtentCheck ext;
  for (size_t i = 0; i < n; ++i) {
    const h3c_desc &x = d[i];
    DevChunk c{};
    c.out_idx = (uint32_t)i;
    c.start = x.start_raw;
    const int k = x.type == H3C_TYPE_CRC32 ? 1 : 0;
    const bool none = !(x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32) || (x.ptr == nullptr && x.len > 0);
    if (!none && x.len > 0 && x.mem != H3C_MEM_DEVICE) {
      g_last_error = "descriptors must be device-resident";
      return H3C_ERR_INVALID_ARG;
    }
    if (!none && x.len > 0 && check_extent && !ext.ok((uint64_t)(uintptr_t)x.ptr, x.len)) {
      g_last_error = "descriptor " + std::to_string(i) + " (" + std::to_string(x.len) +
                     " bytes) runs past the end of its device allocation";
      return H3C_ERR_INVALID_ARG;
    }
    c.seg_begin = g.segs[k];
    if (none) {
      c.flags = kFlagNone;
    } else {
      c.ptr = (uint64_t)(uintptr_t)x.ptr;
      c.len = x.len;
      const uint64_t ns = (x.len + seg_bytes - 1) / seg_bytes;
      if (g.segs[k] + ns > 0xFFFFFFF0u) {
        g_last_error = "too many segments";
        return H3C_ERR_INVALID_ARG;
      }
      g.segs[k] += (uint32_t)ns;
      g.max_segs[k] = std::max(g.max_segs[k], (uint32_t)ns);
      set_fold_consts(c, seg_bytes, k ? kPolyCrc32 : kPolyCrc32c);
      g.bytes[k] += x.len;
    }
    g.hc[k].push_back(c);
  }
  mark_small(g);
  return H3C_OK;
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

int h3c_device_count(void) { return device_count(); }

int h3c_test_hook(int key, uint64_t value) {
  if (key < 1 || key >= kHooks) return H3C_ERR_INVALID_ARG;
  g_hooks[key].store(value);
  return H3C_OK;
}

int h3c_init(int device) { return init_device(device); }

const char *h3c_last_error(void) { return g_last_error.c_str(); }

void h3c_profile_enable(int on) { g_prof_on.store(on ? 1 : 0); }

int h3c_profile_read(int kind, double *kernel_ms, uint64_t *launches, uint64_t *bytes, int reset) {
  if (kind < 0 || kind >= kProfKinds) return H3C_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  // the stamp slots in use, per device: read back once every launch has ended, then freed
  for (int d = 0; d < kMaxDevices; ++d) {
    StampPool &p = g_stamps[d];
    if (!p.d || !p.next) continue;
    int prev = -1;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(d));
    std::vector<unsigned long long> v(2 * (size_t)p.next);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(v.data(), p.d, v.size() * 8, hipMemcpyDeviceToHost);
    bool pend = false;
    for (auto &r : g_prof) pend = pend || (r.dev == d && r.slot >= 0 && r.kind == -1);
    if (!pend) {  // every slot handed out is recorded: the pool rewinds (else slots are freed one by one below)
      std::vector<unsigned long long> init(v.size());
      for (size_t i = 0; i < init.size(); i += 2) init[i] = ~0ull, init[i + 1] = 0;
      if (e == hipSuccess) e = hipMemcpy(p.d, init.data(), init.size() * 8, hipMemcpyHostToDevice);
    }
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
      set_error("h3c_profile_read (stamps)", e);
      return H3C_ERR_HIP;
    }
    const int khz = h3c_rt::device_wall_clock_khz(d);
    bool pending = false;  // a slot handed out whose launch is not recorded yet (prof_stamp .. prof_end)
    for (auto &r : g_prof) pending = pending || (r.dev == d && r.slot >= 0 && r.kind == -1);
    int top_pending = -1;  // the pool rewinds to just past the highest slot still in flight
    for (auto &r : g_prof)
      if (r.dev == d && r.slot >= 0 && r.kind == -1) top_pending = std::max(top_pending, r.slot);
    for (auto &r : g_prof) {
      if (r.dev != d || r.slot < 0 || r.kind == -1) continue;
      const unsigned long long t0 = v[2 * (size_t)r.slot], t1 = v[2 * (size_t)r.slot + 1];
      if (r.kind >= 0 && t1 > t0 && t0 != ~0ull && khz > 0) {
        g_prof_ms_done[r.kind] += (double)(t1 - t0) / khz;
        g_prof_launch_done[r.kind] += 1;
        g_prof_bytes_done[r.kind] += r.bytes;
      }
      if (pending) {  // only the slots read here are freed; the pool is not rewound past a pending one
        (void)hipSetDevice(d);
        const unsigned long long fr[2] = {~0ull, 0ull};
        (void)hipMemcpy(p.d + 2 * (size_t)r.slot, fr, 16, hipMemcpyHostToDevice);
        (void)hipSetDevice(prev);
      }
      r.slot = -2;  // (done)
    }
    p.next = top_pending + 1;  // (0 when nothing is pending: the whole pool was re-initialised above)
  }
  std::vector<ProfRec> keep;  // pending stamp records stay for the next read
  for (auto &r : g_prof) {
    if (r.kind == -1) {
      keep.push_back(r);
      continue;
    }
    if (r.slot != -1) continue;  // (stamp records were read above)
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    g_prof_ms_done[r.kind] += ms;
    g_prof_launch_done[r.kind] += 1;
    g_prof_bytes_done[r.kind] += r.bytes;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.swap(keep);
  if (kernel_ms) *kernel_ms = g_prof_ms_done[kind];
  if (launches) *launches = g_prof_launch_done[kind];
  if (bytes) *bytes = g_prof_bytes_done[kind];
  if (reset) {
    g_prof_ms_done[kind] = 0;
    g_prof_launch_done[kind] = 0;
    g_prof_bytes_done[kind] = 0;
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
  p->seg_bytes = pick_seg_for(d, n, g_dev[device].num_cu);
  p->dbg = read_dbg_flags();
  p->seg_bytes = forced_seg(p->seg_bytes);
  p->bytes = total;

  GroupLayout gl;
  rc = layout_groups(d, n, p->seg_bytes, gl);
  if (rc) {
    delete p;
    (void)hipSetDevice(prev);
    return rc;
  }
  std::vector<DevChunk> *hc = gl.hc;
  uint32_t *segs = gl.segs, *max_segs_chunk = gl.max_segs;
  uint64_t *bytes = gl.bytes;
  uint32_t max_segs = 0;
  for (int g = 0; g < 2; ++g) {
    if (hc[g].empty()) continue;
    Group gr;
    gr.type = g == 0 ? H3C_TYPE_CRC32C : H3C_TYPE_CRC32;
    gr.nchunks = (uint32_t)hc[g].size();
    gr.total_segs = segs[g];
    gr.max_chunk_segs = max_segs_chunk[g];
    gr.bytes = bytes[g];
    gr.small = gl.small[g];
    gr.uni = gl.uni[g];
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
  (void)ctx;
  for (const Group &g : p->groups) {
    rc = h3c_rt::launch_crc(st, p->device, g.type, g.d_chunks, g.nchunks, g.total_segs, g.max_chunk_segs, g.bytes,
                            p->seg_bytes, p->dbg, p->d_segcrc, expected_raw_dev, out_raw_dev, ok_dev, mismatch_dev,
                            H3C_PROF_SEG, g.small, &g.uni);
    if (rc) break;
  }
  if (prev != p->device) HIP_TRY(hipSetDevice(prev));
  return rc;
}

// Synchronous API: stage host payloads through a pinned lease into a pooled device lease
// and run the kernels on the caller's stream.  Neither lease allocates in steady state,
// so concurrent callers on their own streams never force a device-wide synchronisation
// (hipMalloc / hipFree would; hipMallocAsync pools are not used, see DeviceLease).
constexpr uint64_t kZeroCopyMin = 64u << 10;  // pinned payloads above this are read in place
#ifndef H3C_SYNC_IN_PLACE
#define H3C_SYNC_IN_PLACE 1  // 0: results copied back from the device arena (the same-box A/B)
#endif

static int batch_sync(const h3c_desc *d, size_t n, const uint32_t *expected, uint8_t *out_type, uint32_t *out_raw,
                      uint8_t *ok, uint64_t *n_mismatch, void *stream) {
  if (n == 0) {
    if (n_mismatch) *n_mismatch = 0;
    return H3C_OK;
  }
  if (!d || !out_raw || n > 0xFFFFFFF0u) return H3C_ERR_INVALID_ARG;
  int dev = 0;
  int rc = current_device(&dev);
  if (rc) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);

  std::vector<h3c_desc> dd(d, d + n);
  uint64_t host_bytes = 0;
  for (auto &x : dd) {
    const bool crc = x.ptr && x.len && (x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32);
    if (crc && x.mem == H3C_MEM_HOST_PINNED && x.len > kZeroCopyMin) {
      // page-locked host memory the device can address (hipHostMalloc / hipHostRegister, e.g.
      // RDMA buffers): the kernels read it in place over PCIe, no staging copy.  Small buffers
      // are staged anyway (a few 1 KiB rows per chunk over PCIe are latency-bound: 34 us for
      // 32 x 4 KiB read in place against ~5 us copied, profiles/r02_sync_*); memory the runtime
      // does not know as pinned is staged like pageable memory.
      void *dp = nullptr;
      if (hipHostGetDevicePointer(&dp, const_cast<void *>(x.ptr), 0) == hipSuccess && dp) {
        x.ptr = dp;
        x.mem = H3C_MEM_DEVICE;
      } else {
        (void)hipGetLastError();
      }
    }
    if (crc && x.mem != H3C_MEM_DEVICE) host_bytes += (x.len + 255) & ~uint64_t(255);
  }
  const uint64_t seg_bytes = forced_seg(pick_seg_for(d, n, g_dev[dev].num_cu));
  // staging offsets first (descriptor pointers are rewritten to the arena below)
  auto align = [](uint64_t v) { return (v + 255) & ~uint64_t(255); };
  const uint64_t off_stage = 0;
  GroupLayout gl;
  {
    ExtentCheck ext;  // the caller's device payloads only (staged copies are ours)
    for (size_t i = 0; i < n; ++i)
      if (d[i].mem == H3C_MEM_DEVICE && d[i].ptr && d[i].len &&
          (d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) &&
          !ext.ok((uint64_t)(uintptr_t)d[i].ptr, d[i].len)) {
        g_last_error = "descriptor " + std::to_string(i) + " runs past the end of its device allocation";
        return H3C_ERR_INVALID_ARG;
      }
    // layout with placeholder pointers for staged payloads (device-ness is all that matters)
    std::vector<h3c_desc> probe(dd);
    for (auto &x : probe)
      if (x.mem != H3C_MEM_DEVICE) x.mem = H3C_MEM_DEVICE;
    rc = layout_groups(probe.data(), n, seg_bytes, gl, /*check_extent=*/false);
    if (rc) return rc;
  }
  // one layout for the device arena and the pinned staging buffer, so that everything going
  // up is one copy; the results come back by the kernels' own stores into the pinned buffer
  // (H3C_SYNC_IN_PLACE 0: one D2H copy):
  //   [staged payloads | DevChunk lists | expected | mismatch | results out | ok] [segment partials]
  //   |<--------------------- H2D ----------------------------->|<- in place -->|
  const uint64_t off_chunks0 = align(off_stage + host_bytes);
  const uint64_t off_chunks1 = align(off_chunks0 + gl.hc[0].size() * sizeof(DevChunk));
  const uint64_t off_exp = align(off_chunks1 + gl.hc[1].size() * sizeof(DevChunk));
  const uint64_t off_mis = align(off_exp + (expected ? 4ull * n : 0));
  const uint64_t off_out = off_mis + 256;
  const uint64_t off_ok = align(off_out + 4ull * n);
  const uint64_t off_seg = align(off_ok + (expected ? n : 0));
  const uint64_t arena_bytes = off_seg + 4ull * std::max(gl.segs[0], gl.segs[1]) + 256;
  h3c_rt::PinnedLease pin(off_seg);
  if (!pin.ok()) return H3C_ERR_HIP;
  char *const pb = pin.data();
  h3c_rt::DeviceLease scratch(dev, arena_bytes);
  if (!scratch.ok()) return H3C_ERR_HIP;
  char *const arena = scratch.data();
  uint32_t mis = 0;
  // launches onto the legacy stream wait out an engine graph capture (h3c_rt::capture_gate)
  std::shared_lock<std::shared_mutex> gate;
  if (!st) gate = std::shared_lock<std::shared_mutex>(h3c_rt::capture_gate());
  auto body = [&]() -> int {
    // stage host payloads and point their DevChunks at the staged copies
    uint64_t off = off_stage;
    std::vector<uint64_t> staged(n, 0);
    for (size_t i = 0; i < n; ++i) {
      const h3c_desc &x = dd[i];
      if (x.mem != H3C_MEM_DEVICE && x.ptr && x.len && (x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32)) {
        std::memcpy(pb + off, x.ptr, x.len);  // staging and arena share offsets
        staged[i] = (uint64_t)(uintptr_t)(arena + off);
        off += (x.len + 255) & ~uint64_t(255);
      }
    }
    for (int k = 0; k < 2; ++k)
      for (DevChunk &c : gl.hc[k])
        if (staged[c.out_idx]) c.ptr = staged[c.out_idx];
    mark_small(gl);  // staged copies have their own alignment
    std::memcpy(pb + off_chunks0, gl.hc[0].data(), gl.hc[0].size() * sizeof(DevChunk));
    std::memcpy(pb + off_chunks1, gl.hc[1].data(), gl.hc[1].size() * sizeof(DevChunk));
    if (expected) {
      std::memcpy(pb + off_exp, expected, 4ull * n);
      std::memset(pb + off_mis, 0, 4);
    }
    HIP_TRY(hipMemcpyAsync(arena, pb, off_out, hipMemcpyHostToDevice, st));
    DevChunk *d_chunks[2] = {reinterpret_cast<DevChunk *>(arena + off_chunks0),
                             reinterpret_cast<DevChunk *>(arena + off_chunks1)};
    uint32_t *d_seg = reinterpret_cast<uint32_t *>(arena + off_seg);
    uint32_t *d_exp = expected ? reinterpret_cast<uint32_t *>(arena + off_exp) : nullptr;
#if H3C_SYNC_IN_PLACE
    // the results and flags go straight into the pinned lease (no copy back on the call's path); the
    // mismatch count is taken from the flags below
    uint32_t *d_out = reinterpret_cast<uint32_t *>(pb + off_out);
    uint8_t *d_ok = expected ? reinterpret_cast<uint8_t *>(pb + off_ok) : nullptr;
    uint32_t *d_mis = nullptr;
#else
    uint32_t *d_out = reinterpret_cast<uint32_t *>(arena + off_out);
    uint8_t *d_ok = expected ? reinterpret_cast<uint8_t *>(arena + off_ok) : nullptr;
    uint32_t *d_mis = expected ? reinterpret_cast<uint32_t *>(arena + off_mis) : nullptr;
#endif
    for (int k = 0; k < 2; ++k) {
      if (gl.hc[k].empty()) continue;
      const int r = h3c_rt::launch_crc(st, dev, k == 0 ? H3C_TYPE_CRC32C : H3C_TYPE_CRC32, d_chunks[k],
                                       (uint32_t)gl.hc[k].size(), gl.segs[k], gl.max_segs[k], gl.bytes[k], seg_bytes,
                                       read_dbg_flags(), d_seg, d_exp, d_out, d_ok, d_mis, H3C_PROF_SEG,
                                       gl.small[k], &gl.uni[k]);
      if (r) return r;
    }
#if !H3C_SYNC_IN_PLACE
    HIP_TRY(hipMemcpyAsync(pb + off_mis, arena + off_mis, off_seg - off_mis, hipMemcpyDeviceToHost, st));
#endif
    return H3C_OK;
  };
  rc = body();
  const hipError_t se = hipStreamSynchronize(st);  // the leases are reused only after this
  if (rc) return rc;
  if (se != hipSuccess) {
    set_error("batch_sync: hipStreamSynchronize", se);
    return H3C_ERR_HIP;
  }
  std::memcpy(out_raw, pb + off_out, 4ull * n);
  if (expected) {
    std::memcpy(ok, pb + off_ok, n);
    if (H3C_SYNC_IN_PLACE)
      for (size_t i = 0; i < n; ++i) mis += ok[i] == 0;
    else
      std::memcpy(&mis, pb + off_mis, 4);
  }
  if (out_type)
    for (size_t i = 0; i < n; ++i) {
      const bool valid = (d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) &&
                         !(d[i].ptr == nullptr && d[i].len > 0);
      out_type[i] = valid ? d[i].type : (uint8_t)H3C_TYPE_NONE;
    }
  if (n_mismatch) *n_mismatch = mis;
  return H3C_OK;
}

}  // extern "C"

namespace {

// ---- coalescing submission queue (h3c_set_coalescing) ----
// The reference checksums one IO per call from 32 AIO and 32 update threads
// (BatchReadJob.cc:34, ChunkReplica.cc:194).  With coalescing on, synchronous calls on the
// default stream queue per device; a caller that finds no batch in flight becomes the
// leader, takes every queued request (its own included), runs them as ONE batch (one
// staging copy, one launch, one synchronisation) and wakes the others; callers that arrive
// meanwhile form the next batch.
std::atomic<int> g_coalesce{0};

struct SyncReq {
  const h3c_desc *d;
  size_t n;
  const uint32_t *expected;
  uint8_t *out_type;
  uint32_t *out_raw;
  uint8_t *ok;
  uint64_t *n_mismatch;
  int rc = H3C_OK;
  bool done = false;
};

struct Coalescer {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<SyncReq *> pending;
  bool busy = false;
};
Coalescer g_coal[kMaxDevices];

constexpr size_t kMergeMax = 1u << 20;  // descriptors per merged batch

void run_merged(std::vector<SyncReq *> &b) {
  if (b.size() == 1) {
    SyncReq &r = *b[0];
    r.rc = batch_sync(r.d, r.n, r.expected, r.out_type, r.out_raw, r.ok, r.n_mismatch, nullptr);
    return;
  }
  size_t total = 0;
  bool verify = false;
  for (const SyncReq *r : b) {
    total += r->n;
    verify |= r->expected != nullptr;
  }
  std::vector<h3c_desc> dd;
  std::vector<uint32_t> exp(verify ? total : 0), raw(total);
  std::vector<uint8_t> ok(verify ? total : 0);
  dd.reserve(total);
  for (const SyncReq *r : b) {
    if (r->expected) std::copy_n(r->expected, r->n, exp.begin() + dd.size());  // creates verify against 0
    dd.insert(dd.end(), r->d, r->d + r->n);
  }
  const int rc = batch_sync(dd.data(), total, verify ? exp.data() : nullptr, nullptr, raw.data(),
                            verify ? ok.data() : nullptr, nullptr, nullptr);
  if (rc != H3C_OK) {  // one caller's bad descriptor (or a HIP error) must not fail the others:
    for (SyncReq *r : b)  // each request again on its own, with its own status
      r->rc = batch_sync(r->d, r->n, r->expected, r->out_type, r->out_raw, r->ok, r->n_mismatch, nullptr);
    return;
  }
  size_t at = 0;
  for (SyncReq *r : b) {
    r->rc = rc;
    if (rc == H3C_OK) {
      std::copy_n(raw.begin() + at, r->n, r->out_raw);
      if (r->expected) {
        std::copy_n(ok.begin() + at, r->n, r->ok);
        if (r->n_mismatch) *r->n_mismatch = (uint64_t)std::count(ok.begin() + at, ok.begin() + at + r->n, (uint8_t)0);
      }
      if (r->out_type)
        for (size_t i = 0; i < r->n; ++i) {
          const h3c_desc &x = r->d[i];
          const bool valid = (x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32) && !(x.ptr == nullptr && x.len > 0);
          r->out_type[i] = valid ? x.type : (uint8_t)H3C_TYPE_NONE;
        }
    }
    at += r->n;
  }
}

int submit_sync(const h3c_desc *d, size_t n, const uint32_t *expected, uint8_t *out_type, uint32_t *out_raw, uint8_t *ok,
                uint64_t *n_mismatch, void *stream) {
  if (stream != nullptr || n == 0 || !g_coalesce.load(std::memory_order_relaxed))
    return batch_sync(d, n, expected, out_type, out_raw, ok, n_mismatch, stream);
  if (!d || !out_raw || n > 0xFFFFFFF0u) return H3C_ERR_INVALID_ARG;
  int dev = 0;
  const int rc = current_device(&dev);
  if (rc) return rc;
  SyncReq r{d, n, expected, out_type, out_raw, ok, n_mismatch};
  Coalescer &q = g_coal[dev];
  std::unique_lock<std::mutex> lk(q.mu);
  q.pending.push_back(&r);
  while (!r.done) {
    if (!q.busy) {  // lead: everything queued so far is one batch
      q.busy = true;
      // the leader also runs the batch that queued behind its own (once), so the device is
      // not idle while a woken waiter gets scheduled
      for (int round = 0; round < 2 && !q.pending.empty(); ++round) {
        // at most kMergeMax descriptors per merged batch (the rest waits for the next one), so a
        // merged batch stays within the per-call limits every request met on its own
        std::vector<SyncReq *> batch;
        size_t taken = 0, total = 0;
        while (taken < q.pending.size() && (taken == 0 || total + q.pending[taken]->n <= kMergeMax))
          total += q.pending[taken++]->n;
        batch.assign(q.pending.begin(), q.pending.begin() + (long)taken);
        q.pending.erase(q.pending.begin(), q.pending.begin() + (long)taken);
        lk.unlock();
        run_merged(batch);
        lk.lock();
        for (SyncReq *x : batch) x->done = true;
        q.cv.notify_all();
      }
      q.busy = false;
      q.cv.notify_all();
    } else {
      q.cv.wait(lk);
    }
  }
  return r.rc;
}
}  // namespace

extern "C" {

int h3c_set_coalescing(int on) {
  g_coalesce.store(on ? 1 : 0);
  return H3C_OK;
}

int h3c_batch_create(const h3c_desc *d, size_t n, uint8_t *out_type, uint32_t *out_raw, void *stream) {
  return submit_sync(d, n, nullptr, out_type, out_raw, nullptr, nullptr, stream);
}

int h3c_batch_verify(const h3c_desc *d, const uint32_t *expected_raw, size_t n, uint32_t *out_raw, uint8_t *ok,
                     uint64_t *n_mismatch, void *stream) {
  if (n && (!expected_raw || !ok)) return H3C_ERR_INVALID_ARG;
  return submit_sync(d, n, expected_raw, nullptr, out_raw, ok, n_mismatch, stream);
}

// Benchmark driver for the synchronous surface (bench.py --workload sync): `threads` host
// threads each call h3c_batch_verify (api 0) or h3c_crc32c (api 1) `calls` times on their
// own `bytes`-byte pinned host buffer; lat_us[t * calls + k] receives each call's latency.
int h3c_diag_sync_bench(int threads, uint64_t bytes, int calls, int api, double *lat_us, double *wall_s) {
  if (threads < 1 || threads > 1024 || calls < 1 || !lat_us || !wall_s || !bytes) return H3C_ERR_INVALID_ARG;
  int dev = 0;
  int rc = current_device(&dev);
  if (rc) return rc;
  std::vector<uint8_t *> bufs(threads, nullptr);
  for (int t = 0; t < threads; ++t) {
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&bufs[t]), bytes, hipHostMallocDefault));
    uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
    for (uint64_t i = 0; i < bytes; ++i) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      bufs[t][i] = (uint8_t)x;
    }
  }
  std::atomic<int> ready{0}, status{H3C_OK};
  std::atomic<bool> go{false};
  std::vector<double> t0(threads), t1(threads);
  auto body = [&](int t) {
    (void)hipSetDevice(dev);
    const h3c_desc d{bufs[t], bytes, 0xFFFFFFFFu, H3C_TYPE_CRC32C, H3C_MEM_HOST_PINNED, 0};
    uint32_t want = 0, raw = 0;
    uint8_t ok = 0, ty = 0;
    int r = h3c_batch_create(&d, 1, &ty, &want, nullptr);
    for (int w = 0; w < 3 && r == H3C_OK; ++w) r = h3c_batch_verify(&d, &want, 1, &raw, &ok, nullptr, nullptr);
    ready.fetch_add(1);
    while (!go.load()) std::this_thread::yield();
    using clk = std::chrono::steady_clock;
    const auto start = clk::now();
    for (int k = 0; k < calls && r == H3C_OK; ++k) {
      const auto a = clk::now();
      r = api == 0 ? h3c_batch_verify(&d, &want, 1, &raw, &ok, nullptr, nullptr)
                   : h3c_batch_create(&d, 1, &ty, &raw, nullptr);
      if (r == H3C_OK && raw != want) r = H3C_ERR_CHECKSUM_MISMATCH;
      lat_us[(size_t)t * calls + k] = std::chrono::duration<double, std::micro>(clk::now() - a).count();
    }
    t0[t] = std::chrono::duration<double>(start.time_since_epoch()).count();
    t1[t] = std::chrono::duration<double>(clk::now().time_since_epoch()).count();
    if (r != H3C_OK) status.store(r);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) th.emplace_back(body, t);
  while (ready.load() < threads) std::this_thread::yield();
  go.store(true);
  for (auto &x : th) x.join();
  for (uint8_t *b : bufs) (void)hipHostFree(b);
  *wall_s = *std::max_element(t1.begin(), t1.end()) - *std::min_element(t0.begin(), t0.end());
  return status.load();
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
