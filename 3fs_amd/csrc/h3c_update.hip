// h3c_update.hip -- batched partial-update checksums on MI355X (BASELINE config 3).
//
// Replaces, for a batch of block-aligned overwrites, the per-write work of
// ChunkReplica::update + ChunkReplica::updateChecksum (src/storage/store/ChunkReplica.cc:
// 132-300, 319-394).  For an overwrite inside the chunk the reference re-reads the
// prefix [0,off) and the suffix [off+len,size) from disk, CRCs them and does two
// crc32c_combine()s (case iv, :356-390): O(chunk) bytes per write.
//
// Here the chunk checksum is updated by linearity instead (CRC is affine over GF(2)):
//     raw(M') = raw(M) ^ crc0(old ^ new) * x^(8*(L - off - len))
// so a write costs its own bytes: read new + read old + write back = 12 KiB per 4 KiB
// block.  Writes are applied in sequence order.  The batch is split into block writes
// (chunk c, block b, payload i); for each slot (c,b) the "old" data of write i is the
// payload of the previous write to that slot, or the chunk's original bytes for the
// first one.  Kernels:
//   1. tlink     per tile of 256 consecutive writes: an LDS match gives each write its
//                previous writer of the same slot (c,b) inside the tile; the tile's last
//                writer of a slot joins that slot's list in a hash table
//   2. resolve   a write with no predecessor in its tile takes the largest listed index
//                below its own (prev[i]); a slot's first writer also gets final[i] = the
//                slot's last writer (whose bytes must end up there).  No sort.
//   3. shifts    sh[b] = x^(8*(L-(b+1)*G)) per block index, cached per chunk geometry
//   4. delta     one wave per block write: crc0(new^old) over G bytes with the same
//                replicated-LDS stride tables as the create kernel, folded across the
//                wave with table multiplies by uniform constants (wave_fold_tab);
//                the first writer of a slot also writes the slot's final bytes back
//                (it is the only wave that reads the slot's original bytes: no race)
//   5. per-chunk prefix XOR in sequence order:
//        out_raw[i] = raw_in[c] ^ XOR of delta_j * sh[b_j] over writes j<=i to chunk c
//      i.e. the chunk checksum right after write i, which is what updateChecksum stores.
//      Dense tiles (tile / column / apply kernels) when tiles x chunks is small, else a
//      rocPRIM stable sort by chunk + inclusive_scan_by_key(XOR) + scatter.
// Fused path (4 KiB blocks, <= 128 chunks: BASELINE config 3): steps 2, 4 and 5 are one
// launch.  Each wave resolves its writes' links itself, keeps per-chunk running XORs in
// its lanes (lane c holds chunk c, c+64), and workgroups chain their per-chunk aggregates
// in ticket order by decoupled look-back over 8-byte {state, value} granules (one aligned
// agent-scope store each: the data is the flag, no fences); the last workgroup writes the
// final checksums and the counters.  One memset (hash heads, ticket, granules) + tlink +
// the fused kernel: 3 launches instead of 8.
// H3C_UPD_EXACT: the chunks' checksums are first recomputed from their bytes (one create
// launch over the chunk set), so results do not depend on the stored values -- what
// updateChecksum case (iv) computes by re-reading the chunk (ChunkReplica.cc:356-390).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#include "h3c_common.hpp"

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// Write-back store policy per kernel.  upd_fused_kernel: plain stores (round 5: 265 -> 234 us with
// load_row_rmw, profiles/r05s_rmw_policy_ab).  The separate-kernel delta path (upd_delta_kernel, the tiles and
// sort paths) keeps nontemporal stores, the policy it was measured and tested with (r02: +2 %); the round-5
// A/B covered the fused kernels only.
#ifndef H3C_FUSED_NT_STORES
#define H3C_FUSED_NT_STORES 0
#endif
#ifndef H3C_DELTA_NT_STORES
#define H3C_DELTA_NT_STORES 1
#endif
template <bool NT>
__device__ __forceinline__ void store_row(uint64_t a, uint4 v) {
  if (NT) {
    v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (v4u __attribute__((address_space(1))) *)a);
  } else {
    *reinterpret_cast<uint4 *>(a) = v;
  }
}


// rocPRIM picks merge sort below this many items.  Forcing its onesweep radix passes
// (limit 0) measured slower at 100k items: 4 x 23 us lookback-bound iterations.
#ifndef H3C_SORT_MERGE_LIMIT
#define H3C_SORT_MERGE_LIMIT (1024 * 1024)
#endif
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, H3C_SORT_MERGE_LIMIT>;

struct XorOp {
  __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a ^ b; }
};

uint32_t bits_for(uint64_t v) {  // number of bits to represent values < v
  uint32_t b = 0;
  while (b < 64 && (1ull << b) < v) ++b;
  return b;
}

// Sort path only: chunk keys and sequence indices for the per-chunk scan.
__global__ void upd_keys_kernel(const uint32_t *__restrict__ blk_chunk, const uint32_t *__restrict__ blk_index,
                                uint32_t n, uint32_t nchunks, uint32_t bpc, uint32_t *__restrict__ kchunk,
                                uint32_t *__restrict__ iota) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t c = blk_chunk[i], b = blk_index[i];
  iota[i] = i;
  const bool bad = c >= nchunks || b >= bpc;  // invalid entry: parked on the sentinel chunk, no effect
  kchunk[i] = bad ? nchunks : c;
}

// ---- previous-writer links without a sort (tile match + hash of per-tile last writers) ----
// Writes are cut into tiles of kLinkTile consecutive sequence positions.  Within a tile
// each write finds its previous writer of the same slot by an LDS match.  Each tile's last
// writer of a slot is pushed (one atomicExch) on the list of its hash bucket (key = chunk *
// bpc + block); a bucket's list may also hold other slots' writers, told apart by their
// stored key (list entries are index + 1, so an all-zero table is empty: one memset per call
// clears it with the other per-call words).  A write with no predecessor in its tile then takes the largest listed index
// of its slot below its own: a list holds at most one entry per tile and slot, so the walk
// stays short even when every write hammers one slot.  (A returning atomicCAS costs about
// twice an atomicExch here: scripts/atomic_probe.hip.)
#ifndef H3C_LINK_TILE
#define H3C_LINK_TILE 256
#endif
constexpr uint32_t kLinkTile = H3C_LINK_TILE;
// control words (the workspace's, zeroed per call; or the stream's UpdScratch, left reset by each batch's last
// workgroup): [kCtlEpoch] the scratch's batch epoch (8 bits; 0 in a zeroed workspace)
// [kCtlAcc, +1] one u64: the fused kernel's tickets taken << 40 | the range weights summed; [kCtlW, +8) each
// workgroup class's range weight (blockIdx % 8, one XCD each; 16.16 fixed point, 0 = 1.0), learnt by
// upd_tlink_kernel from the previous batch's per-ticket throughput records (UpdScratch only)
enum { kCtlErr = 1, kCtlTimeout = 2, kCtlDone = 3, kCtlEpoch = 4, kCtlAcc = 8, kCtlW = 16, kCtlWords = 64 };
constexpr uint32_t kClasses = 8;
constexpr uint32_t kWOne = 1u << 16;  // weight 1.0
__device__ uint32_t g_uw_seed[kClasses];  // the device's last learnt weights (0: none yet), seeding new scratches
// Hash list entries: op index + 1 (0 ends a list) in a zeroed workspace; in an UpdScratch (`tagged`: never
// cleared between batches) epoch << 24 | (op index + 1), so an entry of an earlier batch ends the list.
constexpr uint32_t kTaggedMaxOps = (1u << 24) - 2;
__device__ __forceinline__ uint32_t hentry(uint32_t i, uint32_t E, uint32_t tagged) {
  return tagged ? (E << 24) | (i + 1) : i + 1;
}
__device__ __forceinline__ bool hvalid(uint32_t e, uint32_t E, uint32_t tagged) {
  return tagged ? (e >> 24) == E && (e & 0xFFFFFFu) != 0 : e != 0;
}
__device__ __forceinline__ uint32_t hindex(uint32_t e, uint32_t tagged) { return (tagged ? e & 0xFFFFFFu : e) - 1; }
// a chunk some write of batch E reaches (a zeroed word never matches)
__device__ __forceinline__ uint32_t touch_mark(uint32_t E) { return 0x100u | E; }

__device__ __forceinline__ uint32_t slot_hash(uint32_t key, uint32_t mask) { return (key * 0x9E3779B1u >> 7) & mask; }

// In-tile grouping by key: an LDS open-addressing table (2 x tile entries) whose entries
// head unordered lists of the tile positions holding that key.  Returns the list head of
// `key` (kNone keys are not inserted).  Collisions inside a tile are rare, so the lists
// are short; one hammered key gives one list of the whole tile.
template <uint32_t kT>
struct TileGroups {
  uint32_t key[2 * kT], head[2 * kT], next[kT];
};

template <uint32_t kT>
__device__ __forceinline__ uint32_t tile_group(TileGroups<kT> &g, uint32_t t, uint32_t key) {
  for (uint32_t e = t; e < 2 * kT; e += kT) {
    g.key[e] = kNone;
    g.head[e] = kNone;
  }
  __syncthreads();
  uint32_t h = kNone;
  if (key != kNone) {
    h = (key * 0x9E3779B1u >> 16) & (2 * kT - 1);
    for (;;) {
      const uint32_t k = atomicCAS(&g.key[h], kNone, key);
      if (k == kNone || k == key) break;
      h = (h + 1) & (2 * kT - 1);
    }
    g.next[t] = atomicExch(&g.head[h], t);
  }
  __syncthreads();
  return h == kNone ? kNone : g.head[h];
}

__global__ __launch_bounds__(kLinkTile) void upd_tlink_kernel(const uint32_t *__restrict__ blk_chunk,
                                                              const uint32_t *__restrict__ blk_index, uint32_t n,
                                                              uint32_t nchunks, uint32_t bpc, uint32_t *hhead,
                                                              uint32_t hmask, uint32_t *__restrict__ nkey,
                                                              uint32_t *__restrict__ next, uint32_t *__restrict__ prev,
                                                              uint32_t *ctl, uint32_t *__restrict__ touched,
                                                              uint32_t tagged, const uint32_t *__restrict__ stat,
                                                              uint32_t nstat) {
  __shared__ TileGroups<kLinkTile> g;
  const uint32_t t = threadIdx.x, i0 = blockIdx.x * kLinkTile, i = i0 + t;
  const uint32_t E = ctl[kCtlEpoch] & 0xFFu;  // (0 in a zeroed workspace)
  if (stat && blockIdx.x == gridDim.x - 1) {  // (a block of its own, no writes) the fused kernel's range weights
                                              // from the previous batch's throughput
    __shared__ unsigned long long w_ops[kClasses], w_ticks[kClasses];
    if (t < kClasses) w_ops[t] = w_ticks[t] = 0;
    __syncthreads();
    const uint32_t Ep = (E + 0xFFu) & 0xFFu;  // (the previous batch's epoch)
    for (uint32_t r = t; r < nstat; r += kLinkTile) {
      const uint32_t a = stat[3 * r];
      if ((a >> 8) != Ep || (a & 0xFFu) >= kClasses) continue;
      atomicAdd(&w_ops[a & 0xFFu], (unsigned long long)stat[3 * r + 1]);
      atomicAdd(&w_ticks[a & 0xFFu], (unsigned long long)stat[3 * r + 2]);
    }
    __syncthreads();
    if (t == 0) {
      double rate[kClasses], mean = 0;
      uint32_t have = 0;
      for (uint32_t c = 0; c < kClasses; ++c) {
        rate[c] = w_ticks[c] ? (double)w_ops[c] / (double)w_ticks[c] : 0.0;
        if (rate[c] > 0) {
          mean += rate[c];
          ++have;
        }
      }
      if (have == kClasses) {  // every class measured: w <- (w + rate / mean rate) / 2, within [0.5, 2]
        mean /= kClasses;
        for (uint32_t c = 0; c < kClasses; ++c) {
          const uint32_t w0 = ctl[kCtlW + c] ? ctl[kCtlW + c] : kWOne;
          double w = (double)w0 / kWOne + H3C_W_GAIN * (-(double)w0 / kWOne + rate[c] / mean);
          w = w < 0.5 ? 0.5 : w > 2.0 ? 2.0 : w;
          ctl[kCtlW + c] = (uint32_t)(w * kWOne);
          __hip_atomic_store(&g_uw_seed[c], (uint32_t)(w * kWOne), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {  // a new scratch (no weights yet): the device's last learnt ones, from any stream's scratch
        bool none = true;
        for (uint32_t c = 0; c < kClasses; ++c) none = none && ctl[kCtlW + c] == 0;
        if (none)
          for (uint32_t c = 0; c < kClasses; ++c)
            ctl[kCtlW + c] = __hip_atomic_load(&g_uw_seed[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  uint32_t key = kNone;
  if (i < n) {
    const uint32_t c = blk_chunk[i], b = blk_index[i];
    if (c < nchunks && b < bpc) {
      key = c * bpc + b;
      touched[c] = touch_mark(E);  // chunks no write reaches keep their stored checksum
    }
  }
  const int ninv = __syncthreads_count(i < n && key == kNone);  // out-of-range entries
  if (t == 0 && ninv) atomicAdd(&ctl[kCtlErr], (uint32_t)ninv);
  const uint32_t head = tile_group(g, t, key);
  uint32_t pin = kNone;
  bool last = true;
  for (uint32_t u = head; u != kNone; u = g.next[u]) {
    if (u < t && (pin == kNone || u > pin)) pin = u;
    if (u > t) last = false;
  }
  if (i < n) prev[i] = pin == kNone ? kNone : i0 + pin;
  if (key != kNone && last) {  // push i on its bucket's list (entries are index + 1; 0 ends a list)
    nkey[i] = key;
    next[i] = atomicExch(&hhead[slot_hash(key, hmask)], hentry(i, E, tagged));
  }
}

// prev[i] for writes with no predecessor in their tile, and final_of[i] (the slot's last
// writer) for each slot's first writer.
__global__ void upd_resolve_kernel(const uint32_t *__restrict__ blk_chunk, const uint32_t *__restrict__ blk_index,
                                   uint32_t n, uint32_t nchunks, uint32_t bpc, const uint32_t *__restrict__ hhead,
                                   uint32_t hmask, const uint32_t *__restrict__ nkey,
                                   const uint32_t *__restrict__ next, uint32_t *__restrict__ prev,
                                   uint32_t *__restrict__ final_of) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || prev[i] != kNone) return;
  const uint32_t c = blk_chunk[i], b = blk_index[i];
  if (c >= nchunks || b >= bpc) return;
  const uint32_t key = c * bpc + b;
  uint32_t p = kNone, fmax = i;  // i's tile's last writer of the slot is on the list
  for (uint32_t e = hhead[slot_hash(key, hmask)]; e != 0; e = next[e - 1]) {
    const uint32_t j = e - 1;
    if (nkey[j] != key) continue;
    if (j < i && (p == kNone || j > p)) p = j;
    fmax = max(fmax, j);
  }
  prev[i] = p;
  if (p == kNone) final_of[i] = fmax;
}

__global__ void upd_shift_kernel(uint32_t bpc, uint64_t chunk_len, uint32_t block_bytes,
                                 const PolyConsts *__restrict__ pc, uint32_t *__restrict__ sh) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= bpc) return;
  sh[b] = dxpow8n(chunk_len - (uint64_t)(b + 1) * block_bytes, pc, pc->poly);
}

// crc0(new ^ old) over `rows` full 1 KiB rows (both 16-byte aligned), by one wave
// (valid in lane 0).
// When `dst` is non-zero the wave also stores the slot's final bytes (from `fin`,
// which may equal `pnew`) after it has read the old bytes of each batch.
__device__ uint32_t delta_crc0(uint64_t pnew, uint64_t pold, uint64_t dst, uint64_t fin, uint32_t rows,
                               uint32_t lane, const char *lb, const LaneLut &L, const uint32_t *red) {
  Streams st{0, 0, 0, 0};
  const uint64_t lo = 16u * lane;
  for (uint32_t r0 = 0; r0 < rows; r0 += 4) {
    const uint32_t nb = min(4u, rows - r0);
    uint4 vn[4], vo[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < (int)nb) {
        vn[u] = load_row_rmw(pnew + (uint64_t)(r0 + u) * kRowBytes + lo);
        vo[u] = load_row_rmw(pold + (uint64_t)(r0 + u) * kRowBytes + lo);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < (int)nb) {
        const uint4 d = make_uint4(vn[u].x ^ vo[u].x, vn[u].y ^ vo[u].y, vn[u].z ^ vo[u].z, vn[u].w ^ vo[u].w);
        consume(st, d, lb, L);
      }
    if (dst) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < (int)nb) {
          const uint4 v = fin == pnew ? vn[u] : load_row_rmw(fin + (uint64_t)(r0 + u) * kRowBytes + lo);
          *reinterpret_cast<uint4 *>(dst + (uint64_t)(r0 + u) * kRowBytes + lo) = v;
        }
    }
  }
  return wave_fold_tab(st, lane, red);
}

__device__ __forceinline__ void upd_delta_kernel_body(
    const uint64_t *__restrict__ chunk_base, uint32_t nchunks, uint32_t bpc, uint32_t block_bytes,
    const uint32_t *__restrict__ blk_chunk, const uint32_t *__restrict__ blk_index, const uint8_t *payload,
    uint32_t n, const uint32_t *__restrict__ prev, const uint32_t *__restrict__ final_of,
    const PolyConsts *__restrict__ pc, uint32_t *__restrict__ delta) {
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRedWords];
  fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, threadIdx.x, kThreads);
  __syncthreads();
  const uint32_t *red = lds + kLdsWords;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wave;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t lo = (uint32_t)(gw * n / nw), hi = (uint32_t)((gw + 1) * n / nw);
  if (lo >= hi) return;
  const char *lb = reinterpret_cast<const char *>(lds);
  const LaneLut L = make_lut(lane);
  const uint32_t rows = block_bytes / kRowBytes;
  auto job_of = [&](uint32_t i, uint64_t &pnew, uint64_t &pold, uint64_t &dst, uint64_t &fin, uint32_t &b) -> bool {
    const uint32_t c = blk_chunk[i];
    b = blk_index[i];
    if (c >= nchunks || b >= bpc) return false;
    const uint32_t p = prev[i];
    const uint64_t slot_addr = chunk_base[c] + (uint64_t)b * block_bytes;
    pnew = (uint64_t)(uintptr_t)payload + (uint64_t)i * block_bytes;
    pold = p == kNone ? slot_addr : (uint64_t)(uintptr_t)payload + (uint64_t)p * block_bytes;
    dst = 0;
    fin = 0;
    if (p == kNone) {
      dst = slot_addr;
      fin = (uint64_t)(uintptr_t)payload + (uint64_t)final_of[i] * block_bytes;
    }
    return true;
  };
  if (rows != 4) {  // generic block size: one block at a time
    for (uint32_t i = lo; i < hi; ++i) {
      uint64_t pnew, pold, dst, fin;
      uint32_t b;
      uint32_t d = 0;
      if (job_of(i, pnew, pold, dst, fin, b))
        d = delta_crc0(pnew, pold, dst, fin, rows, lane, lb, L, red);
      if (lane == 0) delta[i] = d;
    }
    return;
  }
  // 4 KiB blocks (3FS's write granularity).  Per group of 64 block writes, lane k
  // loads block (g0+k)'s metadata with vector loads (one round trip instead of a
  // chain of dependent scalar loads per block); the wave then walks the group with
  // readlane, keeping the next block's 8 payload loads in flight while the current
  // block is folded, written back and fixed up.
  const uint64_t lo16 = 16u * lane;
  const uint64_t pay = (uint64_t)(uintptr_t)payload;
  for (uint32_t g0 = lo; g0 < hi; g0 += 64) {
    const uint32_t cnt = min(64u, hi - g0);
    const uint32_t k = g0 + lane;
    uint32_t m_ok = 0;
    uint64_t m_new = 0, m_old = 0, m_dst = 0, m_fin = 0;
    if (lane < cnt) {
      const uint32_t c = blk_chunk[k], bb = blk_index[k];
      if (c < nchunks && bb < bpc) {
        const uint32_t p = prev[k];
        const uint64_t slot = chunk_base[c] + (uint64_t)bb * block_bytes;
        m_ok = 1;
        m_new = pay + (uint64_t)k * block_bytes;
        m_old = p == kNone ? slot : pay + (uint64_t)p * block_bytes;
        if (p == kNone) {
          m_dst = slot;
          m_fin = pay + (uint64_t)final_of[k] * block_bytes;
        }
      }
    }
    auto rl64 = [](uint64_t v, uint32_t t) -> uint64_t {
      return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, t) |
             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), t) << 32);
    };
    uint4 vn[4], vo[4];
    bool valid = __builtin_amdgcn_readlane(m_ok, 0) != 0;
    uint64_t pnew = rl64(m_new, 0), pold = rl64(m_old, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vn[u] = valid ? load_row_rmw(pnew + u * kRowBytes + lo16) : make_uint4(0, 0, 0, 0);
      vo[u] = valid ? load_row_rmw(pold + u * kRowBytes + lo16) : make_uint4(0, 0, 0, 0);
    }
    for (uint32_t t = 0; t < cnt; ++t) {
      const bool nvalid = t + 1 < cnt && __builtin_amdgcn_readlane(m_ok, t + 1) != 0;
      uint4 wn[4], wo[4];
      uint64_t npnew = 0, npold = 0;
      if (nvalid) {
        npnew = rl64(m_new, t + 1);
        npold = rl64(m_old, t + 1);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        wn[u] = nvalid ? load_row_rmw(npnew + u * kRowBytes + lo16) : make_uint4(0, 0, 0, 0);
        wo[u] = nvalid ? load_row_rmw(npold + u * kRowBytes + lo16) : make_uint4(0, 0, 0, 0);
      }
      uint32_t d = 0;
      if (valid) {
        Streams st{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u)
          consume(st, make_uint4(vn[u].x ^ vo[u].x, vn[u].y ^ vo[u].y, vn[u].z ^ vo[u].z, vn[u].w ^ vo[u].w), lb, L);
        const uint64_t dst = rl64(m_dst, t);
        if (dst) {  // first writer of the slot: leave the slot's final bytes in the chunk
          const uint64_t fin = rl64(m_fin, t);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint4 v = fin == pnew ? vn[u] : load_row_rmw(fin + u * kRowBytes + lo16);
            store_row<H3C_DELTA_NT_STORES>(dst + u * kRowBytes + lo16, v);
          }
        }
        d = wave_fold_tab(st, lane, red);  // lane 0; the block's x^(8*bytes after it) is applied in gather
      }
      if (lane == 0) delta[g0 + t] = d;
      valid = nvalid;
      pnew = npnew;
      pold = npold;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        vn[u] = wn[u];
        vo[u] = wo[u];
      }
    }
  }
}
__global__ __launch_bounds__(kThreads) void upd_delta_kernel(
    const uint64_t *__restrict__ chunk_base, uint32_t nchunks, uint32_t bpc, uint32_t block_bytes,
    const uint32_t *__restrict__ blk_chunk, const uint32_t *__restrict__ blk_index, const uint8_t *payload,
    uint32_t n, const uint32_t *__restrict__ prev, const uint32_t *__restrict__ final_of,
    const PolyConsts *__restrict__ pc, uint32_t *__restrict__ delta,
                                                             unsigned long long *ts) {  // ts: h3c_rt::prof_stamp's slot, or nullptr
  stamp_begin(ts);
  upd_delta_kernel_body(chunk_base, nchunks, bpc, block_bytes, blk_chunk, blk_index, payload, n, prev, final_of, pc, delta);
  stamp_end(ts);
}

// ---- fused path: links, deltas, write-back and per-chunk prefix in one launch ----
constexpr uint32_t kFusedCols = 128;    // chunk columns of the look-back: lane c holds chunks c and c + 64
constexpr uint32_t kFusedMaxWG = 1024;  // granule rows reserved in the workspace
constexpr uint32_t kGranAgg = 1, kGranIncl = 2;
#ifndef H3C_UPD_LOOK_WIN
#define H3C_UPD_LOOK_WIN 4
#endif
constexpr uint32_t kLookWin = H3C_UPD_LOOK_WIN;  // look-back rows read per column per round trip
constexpr uint32_t kSpinLimit = 1u << 22;  // bounded look-back spins (about a quarter second)
#ifndef H3C_UPD_WAVES
#define H3C_UPD_WAVES 16  // upd_fused_kernel's waves per workgroup (one workgroup per CU)
#endif
#ifndef H3C_UPD_DEPTH
#define H3C_UPD_DEPTH 1  // upd_fused_kernel: writes whose rows load while one is consumed
#endif
constexpr uint32_t kFW = H3C_UPD_WAVES, kFThreads = 64 * kFW;
constexpr int kFD = H3C_UPD_DEPTH;
static_assert(kFW >= 2 && kFW <= 16 && kFD >= 1 && kFD <= 4, "fused kernel shape");
typedef unsigned long long __attribute__((address_space(1))) gu64;

// granules: {epoch << 8 | state, value} (state 0: not published in batch E; a zeroed row never matches)
__device__ __forceinline__ void gran_store(uint64_t *p, uint32_t E, uint32_t state, uint32_t v) {
  __hip_atomic_store((gu64 *)p, ((unsigned long long)((E << 8) | state) << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t gran_state(uint64_t g, uint32_t E) {
  const uint32_t hi = (uint32_t)(g >> 32);
  return (hi >> 8) == E ? (hi & 3u) : 0u;
}
__device__ __forceinline__ uint64_t gran_load(const uint64_t *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave w of workgroup L takes writes [lo, hi) of (16 L + w); workgroup L's look-back waits only
// on workgroups below it.  L is a ticket taken when the workgroup starts (not blockIdx.x), so a
// workgroup only ever waits on workgroups that are already running, whatever order the hardware
// dispatches them in or however many CUs other work holds.  Every spin is still bounded: a
// workgroup that gives up publishes what it has and flags the batch, and the last workgroup
// reports the flag as *n_invalid = counters.invalid = all ones (the chunk bytes are right; the
// checksums of that call are void -- a create pass over the chunks recovers them).
// Per group of 64 writes lane k loads write k's metadata -- resolving its previous writer
// from the tile link or the hash of per-tile last writers -- then the wave walks the group as
// upd_delta_kernel does.  Afterwards each write's v = delta * sh[b] is folded into the running
// XOR of its chunk (lane c mod 64), whose value right after the write is kept in inpre[i].
__device__ __forceinline__ void upd_fused_kernel_body(
    const uint64_t *__restrict__ chunk_base, uint32_t nchunks, uint32_t bpc, const uint32_t *__restrict__ blk_chunk,
    const uint32_t *__restrict__ blk_index, const uint8_t *payload, uint32_t n, const uint32_t *__restrict__ prev,
    const uint32_t *__restrict__ hhead, uint32_t hmask, const uint32_t *__restrict__ nkey,
    const uint32_t *__restrict__ next, const uint32_t *__restrict__ sh, const PolyConsts *__restrict__ pc,
    const uint32_t *__restrict__ raw_base, const uint32_t *__restrict__ raw_in, uint32_t exact, uint32_t reuse_case,
    const uint32_t *__restrict__ touched, uint32_t *ctl, uint64_t *gran, uint32_t *__restrict__ inpre,
    uint32_t *__restrict__ out_raw, uint32_t *__restrict__ raw_out, uint32_t *__restrict__ n_invalid,
    unsigned long long *__restrict__ counters, uint32_t force_timeout, uint32_t tagged, uint32_t *stat) {
  constexpr uint32_t G4 = 4096;
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRedWords];
  __shared__ uint32_t s_ticket, s_E, s_wlo, s_whi;
  __shared__ uint64_t s_wt, s_t0;
  const uint32_t cls = blockIdx.x % kClasses;  // (workgroups are dealt round-robin over the 8 XCDs)
  if (threadIdx.x == 0) {
    // the ticket and the range: workgroups take tickets in order, and ticket L's range is the next slice
    // of the batch, sized by its class's weight (a slower XCD gets fewer writes)
    uint64_t wt = 0, wmine = 0;
    for (uint32_t c = 0; c < kClasses; ++c) {
      const uint32_t w = ctl[kCtlW + c] ? ctl[kCtlW + c] : kWOne;
      const uint32_t cnt = gridDim.x > c ? (gridDim.x - 1 - c) / kClasses + 1 : 0u;
      wt += (uint64_t)cnt * w;
      if (c == cls) wmine = w;
    }
    const unsigned long long old =
        atomicAdd(reinterpret_cast<unsigned long long *>(ctl + kCtlAcc), (1ull << 40) | wmine);
    const uint64_t cum = old & ((1ull << 40) - 1);
    s_ticket = (uint32_t)(old >> 40);
    s_wt = wt;
    s_wlo = (uint32_t)(cum * n / wt);
    s_whi = s_ticket + 1 == gridDim.x ? n : (uint32_t)((cum + wmine) * n / wt);
    s_E = __hip_atomic_load(&ctl[kCtlEpoch], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xFFu;
  }
  // the CRC tables fill while thread 0 takes the ticket (waves 1-15; they do not depend on the range)
  if (threadIdx.x >= 64)
    fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, threadIdx.x - 64, kFThreads - 64);
  __syncthreads();
  const uint32_t L = s_ticket, nwg = gridDim.x, E = s_E;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wlo = s_wlo, wn = s_whi - s_wlo;  // the workgroup's writes; each wave a contiguous share
  const uint32_t lo = wlo + (uint32_t)((uint64_t)wave * wn / kFW);
  const uint32_t hi = wlo + (uint32_t)((uint64_t)(wave + 1) * wn / kFW);
  const uint64_t lo16 = 16u * lane;
  const uint64_t pay = (uint64_t)(uintptr_t)payload;
  auto rl64 = [](uint64_t v, uint32_t t) -> uint64_t {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, t) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), t) << 32);
  };
  // per group of 64 writes: lane k's write (chunk, shift, new / old / destination / final bytes)
  uint32_t m_c = kNone, m_sh = 0;
  uint64_t m_new = 0, m_old = 0, m_dst = 0, m_fin = 0;
  // the rows of the write being consumed ([0]) and of the next kFD ones, their validity and payload addresses
  uint4 bn[kFD + 1][4], bo[kFD + 1][4];
  bool bv[kFD + 1];
  uint64_t bp[kFD + 1];
  // write t of the group into a buffer slot (invalid past the group)
  auto load_op = [&](uint4(&n4)[4], uint4(&o4)[4], bool &v, uint64_t &p, uint32_t t, uint32_t cnt) {
    v = t < cnt && __builtin_amdgcn_readlane(m_c, t) != kNone;
    p = 0;
    uint64_t po = 0;
    bool blk = false;
    if (v) {
      p = rl64(m_new, t);
      po = rl64(m_old, t);
      blk = rl64(m_dst, t) != 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      n4[u] = v ? load_row_rmw(p + u * kRowBytes + lo16) : make_uint4(0, 0, 0, 0);
      o4[u] = v ? load_row_old(po + u * kRowBytes + lo16, blk) : make_uint4(0, 0, 0, 0);
    }
  };
  auto start_group = [&](uint32_t g0) {
    const uint32_t cnt = min(64u, hi - g0);
    const uint32_t k = g0 + lane;
    m_c = kNone;
    m_sh = 0;
    m_new = m_old = m_dst = m_fin = 0;
    uint32_t key = kNone;
    if (lane < cnt) {
      const uint32_t c = blk_chunk[k], bb = blk_index[k];
      if (c < nchunks && bb < bpc) {
        const uint32_t p = prev[k];
        const uint64_t slot = chunk_base[c] + (uint64_t)bb * G4;
        m_c = c;
        m_sh = sh[bb];
        m_new = pay + (uint64_t)k * G4;
        // speculate the common case: no earlier writer of the slot anywhere, and no later one
        m_old = p == kNone ? slot : pay + (uint64_t)p * G4;
        m_dst = p == kNone ? slot : 0;
        m_fin = p == kNone ? m_new : 0;
        if (p == kNone) key = c * bpc + bb;
      }
    }
    const bool valid = __builtin_amdgcn_readlane(m_c, 0) != kNone;
    bv[0] = valid;
    bp[0] = rl64(m_new, 0);
    uint64_t pold = rl64(m_old, 0);
    const bool oblk = rl64(m_dst, 0) != 0;  // (the speculated old rows are the slot's own)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      bn[0][u] = valid ? load_row_rmw(bp[0] + u * kRowBytes + lo16) : make_uint4(0, 0, 0, 0);
      bo[0][u] = valid ? load_row_old(pold + u * kRowBytes + lo16, oblk) : make_uint4(0, 0, 0, 0);
    }
    // the walk over the slot's listed tile-last writers, while those rows load
    if (key != kNone) {
      uint32_t p = kNone, fmax = k;
      for (uint32_t e = hhead[slot_hash(key, hmask)]; hvalid(e, E, tagged); e = next[hindex(e, tagged)]) {
        const uint32_t j = hindex(e, tagged);
        if (nkey[j] != key) continue;
        if (j < k && (p == kNone || j > p)) p = j;
        fmax = max(fmax, j);
      }
      if (p != kNone) {  // an earlier tile wrote the slot: its bytes are the old ones, it writes back
        m_old = pay + (uint64_t)p * G4;
        m_dst = 0;
        m_fin = 0;
      } else {  // the slot's first writer leaves the slot's last writer's bytes
        m_fin = pay + (uint64_t)fmax * G4;
      }
    }
    const uint64_t pold2 = rl64(m_old, 0);
    if (valid && pold2 != pold) {  // write 0 was mis-speculated: reload its old rows
      pold = pold2;
#pragma unroll
      for (int u = 0; u < 4; ++u) bo[0][u] = load_row_rmw(pold + u * kRowBytes + lo16);
    }
    // the next writes' rows (their links are resolved now)
#pragma unroll
    for (int i = 1; i < kFD; ++i) load_op(bn[i], bo[i], bv[i], bp[i], (uint32_t)i, cnt);
  };
  if (lo < hi) start_group(lo);  // the first group's links and rows load while the tables fill
  __syncthreads();
  if (threadIdx.x == 0) s_t0 = wall_clock64();
  const uint32_t *red = lds + kLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const LaneLut Lt = make_lut(lane);
  const uint32_t poly = pc->poly;
  uint32_t acc0 = 0, acc1 = 0;  // running XOR of chunks lane, lane + 64
  uint32_t my_ip = 0;           // lane t: the chunk XOR right after write t of the group
  for (uint32_t g0 = lo; g0 < hi; g0 += 64) {
    const uint32_t cnt = min(64u, hi - g0);
    const uint32_t k = g0 + lane;
    uint32_t my_d = 0;
    for (uint32_t t = 0; t < cnt; ++t) {
      load_op(bn[kFD], bo[kFD], bv[kFD], bp[kFD], t + kFD, cnt);
      if (bv[0]) {
        Streams st{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u)
          consume(st,
                  make_uint4(bn[0][u].x ^ bo[0][u].x, bn[0][u].y ^ bo[0][u].y, bn[0][u].z ^ bo[0][u].z,
                             bn[0][u].w ^ bo[0][u].w),
                  lb, Lt);
        const uint64_t dst = rl64(m_dst, t);
        if (dst) {  // first writer of the slot: leave the slot's final bytes in the chunk
          const uint64_t fin = rl64(m_fin, t);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint4 v = fin == bp[0] ? bn[0][u] : load_row_rmw(fin + u * kRowBytes + lo16);
            store_row<H3C_FUSED_NT_STORES>(dst + u * kRowBytes + lo16, v);
          }
        }
        const uint32_t d = __builtin_amdgcn_readlane(wave_fold_tab(st, lane, red), 0);
        if (lane == t) my_d = d;
      }
#pragma unroll
      for (int i = 0; i < kFD; ++i) {
        bv[i] = bv[i + 1];
        bp[i] = bp[i + 1];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          bn[i][u] = bn[i + 1][u];
          bo[i][u] = bo[i + 1][u];
        }
      }
    }
    // the group's v, all lanes at once; each write's chunk XOR right after it (inclusive, with
    // the earlier groups' running value), and the running values moved past the group
    const uint32_t v = m_c != kNone ? dgf_mul(my_d, m_sh, poly) : 0u;
    const uint32_t src = m_c & 63;
    const uint32_t r0 = __shfl(acc0, src, 64), r1 = __shfl(acc1, src, 64);
    my_ip = m_c < 64 ? r0 : r1;
    for (uint32_t t = 0; t < cnt; ++t) {
      const uint32_t ct = __builtin_amdgcn_readlane(m_c, t), vt = __builtin_amdgcn_readlane(v, t);
      if (lane >= t && m_c == ct) my_ip ^= vt;
      if (ct == lane) acc0 ^= vt;
      if (ct == lane + 64) acc1 ^= vt;
    }
    if (lane < cnt) inpre[k] = my_ip;
    if (g0 + 64 < hi) start_group(g0 + 64);
  }
  // the chunks' base checksums, one per lane (chunks lane, lane + 64)
  const uint32_t rb0 = lane < nchunks ? raw_base[lane] : 0u, rb1 = lane + 64 < nchunks ? raw_base[64 + lane] : 0u;

  // ---- chunk aggregates: waves of the workgroup (LDS), then workgroups (look-back) ----
  __syncthreads();  // the CRC tables are done with: their LDS holds the aggregates now
  if (stat && threadIdx.x == 0 && L < kFusedMaxWG) {  // this workgroup's throughput, for the next batch's weights
    stat[3 * L] = (E << 8) | cls;
    stat[3 * L + 1] = wn;
    stat[3 * L + 2] = (uint32_t)(wall_clock64() - s_t0);
  }
  uint32_t *wagg = lds;                               // [16][128]
  uint32_t *wexcl = lds + kFW * kFusedCols;  // [128]: the workgroup's exclusive prefix
  wagg[wave * kFusedCols + lane] = acc0;
  wagg[wave * kFusedCols + 64 + lane] = acc1;
  __syncthreads();
  if (wave == 0) {
    uint32_t a0 = 0, a1 = 0;
    for (uint32_t w = 0; w < kFW; ++w) {
      a0 ^= wagg[w * kFusedCols + lane];
      a1 ^= wagg[w * kFusedCols + 64 + lane];
    }
    const bool two = nchunks > 64;
    uint64_t *row = gran + (uint64_t)L * kFusedCols;
    uint32_t x0 = 0, x1 = 0;
    if (L > 0) {
      if (lane < nchunks) gran_store(row + lane, E, kGranAgg, a0);
      if (two && lane + 64 < nchunks) gran_store(row + 64 + lane, E, kGranAgg, a1);
      int j0 = lane < nchunks ? (int)L - 1 : -1, j1 = two && lane + 64 < nchunks ? (int)L - 1 : -1;
      // test hook (H3C_HOOK_UPD_LOOKBACK): ticket 1 gives up at once, as a starved wait would
      const uint32_t limit = force_timeout && L == 1 ? 0u : kSpinLimit;
      for (uint32_t spins = 0; __builtin_amdgcn_ballot_w64(j0 >= 0 || j1 >= 0) != 0;) {
        bool moved = false;
        // a window of kLookWin rows per column in one round trip: a predecessor that has just posted
        // its aggregate is passed together with the inclusive row below it
        auto look = [&](int &j, uint32_t &x, uint32_t col) {
          if (j < 0) return;
          const int top = j;
          uint64_t g[kLookWin];
#pragma unroll
          for (int w = 0; w < (int)kLookWin; ++w)
            g[w] = top - w >= 0 ? gran_load(gran + (uint64_t)(top - w) * kFusedCols + col) : 0ull;
#pragma unroll
          for (int w = 0; w < (int)kLookWin; ++w) {
            const uint32_t state = gran_state(g[w], E);
            if (top - w >= 0 && j == top - w && state) {
              x ^= (uint32_t)g[w];
              j = state == kGranIncl ? -1 : j - 1;
              moved = true;
            }
          }
        };
        look(j0, x0, lane);
        look(j1, x1, 64 + lane);
        if (__builtin_amdgcn_ballot_w64(moved) == 0 || limit == 0) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > limit) {  // a predecessor never published: give up, flag the batch
            if (lane == 0) atomicExch(&ctl[kCtlTimeout], 1u);
            __threadfence();  // the flag before this workgroup's inclusive granules
            break;
          }
        }
      }
    }
    if (lane < nchunks) gran_store(row + lane, E, kGranIncl, x0 ^ a0);
    if (two && lane + 64 < nchunks) gran_store(row + 64 + lane, E, kGranIncl, x1 ^ a1);
    wexcl[lane] = x0;
    wexcl[64 + lane] = x1;
    // every workgroup but the last counts itself done once its flag (if it gave up) is out: the last
    // one reads the flag only after all the others' counts (look-back may have passed a workgroup's
    // aggregate before that workgroup gave up and raised the flag).  The give-up branch fences its
    // flag; the count itself needs no fence: an agent-scope release here wrote back the XCD's L2
    // (buffer_wbl2) once per workgroup, ~3 us of the kernel (profiles/r04_update_tail_ab.txt).
    if (L != nwg - 1 && lane == 0) atomicAdd(&ctl[kCtlDone], 1u);
    if (L == nwg - 1) {  // the last workgroup: final checksums, counts
      const uint32_t t0 = x0 ^ a0, t1 = x1 ^ a1;
      uint32_t stale = 0;
      if (lane < nchunks) {
        raw_out[lane] = touched[lane] == touch_mark(E) ? raw_base[lane] ^ t0 : raw_in[lane];
        stale += exact && raw_base[lane] != raw_in[lane];
      }
      if (lane + 64 < nchunks) {
        raw_out[64 + lane] = touched[64 + lane] == touch_mark(E) ? raw_base[64 + lane] ^ t1 : raw_in[64 + lane];
        stale += exact && raw_base[64 + lane] != raw_in[64 + lane];
      }
      for (int o = 32; o >= 1; o >>= 1) stale += __shfl_xor(stale, o, 64);
      if (lane == 0) {
        // wait (bounded) for every other workgroup's done count; a count that never comes voids the batch
        // (the counts and flags are agent-scope atomics at the coherence point: no L2 write-back needed)
        bool late = false;
        for (uint32_t spins = 0;
             __hip_atomic_load(&ctl[kCtlDone], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nwg - 1;) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > kSpinLimit) {
            late = true;
            break;
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last count read before the flags
        if (late) atomicExch(&ctl[kCtlTimeout], 1u);
        const uint32_t inv = __hip_atomic_load(&ctl[kCtlErr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // every workgroup's inclusive granule was read (directly or through a later one's) before
        // this: a workgroup that gave up had raised the flag first
        const bool void_batch = __hip_atomic_load(&ctl[kCtlTimeout], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n_invalid) *n_invalid = void_batch ? 0xFFFFFFFFu : inv;
        if (counters) {  // h3c_update_counters: none, reuse, combine, read_chunk, recalculate, mismatch, invalid, stale
          const unsigned long long ok = n - inv;
          counters[0] = 0;
          counters[1] = reuse_case ? ok : 0;
          counters[2] = 0;
          counters[3] = reuse_case ? 0 : ok;
          counters[4] = 0;
          counters[5] = 0;
          counters[6] = void_batch ? ~0ull : inv;
          counters[7] = stale;
        }
        // the control words back to their batch-start values for the next batch on this scratch (the
        // subtractions are exact even when a late workgroup counts itself done after this), the epoch on
        atomicAdd(reinterpret_cast<unsigned long long *>(ctl + kCtlAcc), 0ull - (((unsigned long long)nwg << 40) + s_wt));
        atomicSub(&ctl[kCtlDone], nwg - 1);
        atomicSub(&ctl[kCtlErr], inv);
        atomicExch(&ctl[kCtlTimeout], 0u);
        __hip_atomic_store(&ctl[kCtlEpoch], (E + 1) & 0xFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  __syncthreads();
  uint32_t e0 = wexcl[lane], e1 = wexcl[64 + lane];
  for (uint32_t w = 0; w < wave; ++w) {
    e0 ^= wagg[w * kFusedCols + lane];
    e1 ^= wagg[w * kFusedCols + 64 + lane];
  }
  const uint32_t be0 = rb0 ^ e0, be1 = rb1 ^ e1;
  if (hi - lo <= 64) {  // one group (the common case): its chunks and XORs are still in registers
    const uint32_t x0 = __shfl(be0, m_c & 63, 64), x1 = __shfl(be1, m_c & 63, 64);
    if (lo + lane < hi) out_raw[lo + lane] = m_c != kNone ? (m_c < 64 ? x0 : x1) ^ my_ip : 0u;
    return;
  }
  for (uint32_t i0 = lo; i0 < hi; i0 += 64) {
    const uint32_t i = i0 + lane;
    uint32_t c = kNone, b = 0;
    if (i < hi) {
      c = blk_chunk[i];
      b = blk_index[i];
    }
    const bool ok = i < hi && c < nchunks && b < bpc;
    const uint32_t x0 = __shfl(be0, c & 63, 64), x1 = __shfl(be1, c & 63, 64);
    if (i < hi) out_raw[i] = ok ? (c < 64 ? x0 : x1) ^ inpre[i] : 0u;
  }
}
__global__ __launch_bounds__(kFThreads) void upd_fused_kernel(
    const uint64_t *__restrict__ chunk_base, uint32_t nchunks, uint32_t bpc, const uint32_t *__restrict__ blk_chunk,
    const uint32_t *__restrict__ blk_index, const uint8_t *payload, uint32_t n, const uint32_t *__restrict__ prev,
    const uint32_t *__restrict__ hhead, uint32_t hmask, const uint32_t *__restrict__ nkey,
    const uint32_t *__restrict__ next, const uint32_t *__restrict__ sh, const PolyConsts *__restrict__ pc,
    const uint32_t *__restrict__ raw_base, const uint32_t *__restrict__ raw_in, uint32_t exact, uint32_t reuse_case,
    const uint32_t *__restrict__ touched, uint32_t *ctl, uint64_t *gran, uint32_t *__restrict__ inpre,
    uint32_t *__restrict__ out_raw, uint32_t *__restrict__ raw_out, uint32_t *__restrict__ n_invalid,
    unsigned long long *__restrict__ counters, uint32_t force_timeout, uint32_t tagged, uint32_t *stat,
                                                             unsigned long long *ts) {  // ts: h3c_rt::prof_stamp's slot, or nullptr
  stamp_begin(ts);
  upd_fused_kernel_body(chunk_base, nchunks, bpc, blk_chunk, blk_index, payload, n, prev, hhead, hmask, nkey, next, sh, pc, raw_base, raw_in, exact, reuse_case, touched, ctl, gran, inpre, out_raw, raw_out, n_invalid, counters, force_timeout, tagged, stat);
  stamp_end(ts);
}

// H3C_UPD_EXACT: create descriptors for the chunk set (uniform length, start 0).
__global__ void upd_exact_desc_kernel(const uint64_t *__restrict__ chunk_base, uint32_t nchunks, uint32_t spc,
                                      DevChunk tmpl, DevChunk *__restrict__ out) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  DevChunk d = tmpl;
  d.ptr = chunk_base[c];
  d.out_idx = c;
  d.seg_begin = c * spc;
  out[c] = d;
}

// Counts for the tile / sort paths (the fused kernel writes them itself).
__global__ void upd_finish_kernel(const uint32_t *__restrict__ ctl, uint32_t n, uint32_t nchunks,
                                  const uint32_t *__restrict__ raw_base, const uint32_t *__restrict__ raw_in,
                                  uint32_t exact, uint32_t reuse_case, uint32_t *__restrict__ n_invalid,
                                  unsigned long long *__restrict__ counters) {
  __shared__ unsigned int s_stale;
  if (threadIdx.x == 0) s_stale = 0;
  __syncthreads();
  uint32_t stale = 0;
  if (exact)
    for (uint32_t c = threadIdx.x; c < nchunks; c += blockDim.x) stale += raw_base[c] != raw_in[c];
  if (stale) atomicAdd(&s_stale, stale);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t inv = ctl[kCtlErr];
    if (n_invalid) *n_invalid = inv;
    if (counters) {
      const unsigned long long ok = n - inv;
      counters[0] = 0;
      counters[1] = reuse_case ? ok : 0;
      counters[2] = 0;
      counters[3] = reuse_case ? 0 : ok;
      counters[4] = 0;
      counters[5] = 0;
      counters[6] = inv;
      counters[7] = s_stale;
    }
  }
}

// vals[p] = delta of the p-th write in (chunk, sequence) order, moved to its place in
// the chunk: crc0(new ^ old) * x^(8*(L - (b+1)*G)).  One thread per write.
__global__ void upd_gather_kernel(const uint32_t *__restrict__ chunk_s, const uint32_t *__restrict__ idx2, uint32_t n,
                                  uint32_t nchunks, const uint32_t *__restrict__ blk_index,
                                  const uint32_t *__restrict__ delta, const uint32_t *__restrict__ sh, uint32_t poly,
                                  uint32_t *__restrict__ vals) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t i = idx2[p];
  vals[p] = chunk_s[p] < nchunks ? dgf_mul(delta[i], sh[blk_index[i]], poly) : 0u;  // sentinel: invalid entry
}

__global__ void upd_scatter_kernel(const uint32_t *__restrict__ chunk_s, const uint32_t *__restrict__ idx2, uint32_t n,
                                   uint32_t nchunks, const uint32_t *__restrict__ scan,
                                   const uint32_t *__restrict__ raw_in, uint32_t *__restrict__ out_raw,
                                   uint32_t *__restrict__ raw_out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t c = chunk_s[p], i = idx2[p];
  if (c >= nchunks) {  // invalid entry (sentinel chunk)
    out_raw[i] = 0;
    return;
  }
  const uint32_t v = raw_in[c] ^ scan[p];
  out_raw[i] = v;
  if (p + 1 == n || chunk_s[p + 1] != c) raw_out[c] = v;
}

// ---- per-chunk prefix XOR in sequence order without a second sort (dense tiles) ----
// Writes are cut into tiles of kTile consecutive sequence positions.  Used when
// ntiles * nchunks is small (the dense per-tile aggregate matrix stays a few MB).
constexpr uint32_t kTile = 256;

// One workgroup per tile.  v_i = delta_i * sh[b_i] (0 for an invalid entry);
// inpre[i] = XOR of v_j over tile writes j <= i to the same chunk; agg row `tile`
// [c] = XOR of v_j over all tile writes to chunk c (0 when none).
__global__ __launch_bounds__(kTile) void upd_tile_kernel(const uint32_t *__restrict__ blk_chunk,
                                                         const uint32_t *__restrict__ blk_index, uint32_t n,
                                                         uint32_t nchunks, uint32_t bpc,
                                                         const uint32_t *__restrict__ delta,
                                                         const uint32_t *__restrict__ sh, uint32_t poly,
                                                         uint32_t *__restrict__ inpre, uint32_t *__restrict__ agg) {
  __shared__ TileGroups<kTile> g;
  __shared__ uint32_t val[kTile];
  const uint32_t t = threadIdx.x, i = blockIdx.x * kTile + t;
  uint32_t c = kNone, v = 0;
  if (i < n) {
    const uint32_t cc = blk_chunk[i], b = blk_index[i];
    if (cc < nchunks && b < bpc) {
      c = cc;
      v = dgf_mul(delta[i], sh[b], poly);
    }
  }
  val[t] = v;
  uint32_t *row = agg + (uint64_t)blockIdx.x * nchunks;
  for (uint32_t k = t; k < nchunks; k += kTile) row[k] = 0;
  __syncthreads();  // orders val[] and the row zeroing
  const uint32_t head = tile_group(g, t, c);
  uint32_t acc = 0;
  bool last = true;
  for (uint32_t u = head; u != kNone; u = g.next[u]) {  // the tile's writes to chunk c
    if (u <= t) acc ^= val[u];
    else last = false;
  }
  if (i < n) inpre[i] = acc;
  if (c != kNone && last) row[c] = acc;  // the tile's last write to c carries the aggregate
}

// One workgroup per chunk: exclusive XOR scan of its agg column over tiles into
// colpre, and the chunk's final checksum.
__global__ __launch_bounds__(kTile) void upd_column_kernel(const uint32_t *__restrict__ agg, uint32_t ntiles,
                                                           uint32_t nchunks, const uint32_t *__restrict__ raw_base,
                                                           const uint32_t *__restrict__ raw_in,
                                                           const uint32_t *__restrict__ touched,
                                                           uint32_t *__restrict__ colpre,
                                                           uint32_t *__restrict__ raw_out) {
  __shared__ uint32_t part[kTile / 64];
  const uint32_t c = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < ntiles; base += kTile) {
    const uint32_t r = base + t;
    const uint32_t x = r < ntiles ? agg[(uint64_t)r * nchunks + c] : 0u;
    uint32_t inc = x;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc ^= y;
    }
    if (lane == 63) part[wave] = inc;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before ^= part[w];
    uint32_t total = carry;
    for (uint32_t w = 0; w < kTile / 64; ++w) total ^= part[w];
    if (r < ntiles) colpre[(uint64_t)r * nchunks + c] = before ^ inc ^ x;  // exclusive
    carry = total;
    __syncthreads();
  }
  if (t == 0) raw_out[c] = touched[c] ? raw_base[c] ^ carry : raw_in[c];
}

// One thread per write: the chunk checksum right after it.
__global__ void upd_apply_kernel(const uint32_t *__restrict__ blk_chunk, const uint32_t *__restrict__ blk_index,
                                 uint32_t n, uint32_t nchunks, uint32_t bpc, const uint32_t *__restrict__ raw_in,
                                 const uint32_t *__restrict__ colpre, const uint32_t *__restrict__ inpre,
                                 uint32_t *__restrict__ out_raw) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t c = blk_chunk[i], b = blk_index[i];
  out_raw[i] = (c < nchunks && b < bpc) ? raw_in[c] ^ colpre[(uint64_t)(i / kTile) * nchunks + c] ^ inpre[i] : 0u;
}

// Which per-chunk scan: the fused launch for 4 KiB blocks and <= 128 chunks, else dense tiles
// unless their aggregate matrix would be large, else sort + scan_by_key (test hook
// H3C_HOOK_UPD_SCAN forces one).
enum Path { kPathFused = 1, kPathTiles = 2, kPathSort = 3 };
bool tiles_fit(uint32_t n, uint32_t nchunks) {
  const uint64_t ntiles = (n + kTile - 1) / kTile;
  return ntiles * nchunks <= (1ull << 22);
}
int pick_path(uint32_t n, uint32_t nchunks, uint32_t block_bytes) {
  const bool fused_ok = block_bytes == 4096 && nchunks <= kFusedCols;
  const uint64_t forced = h3c_rt::hook(H3C_HOOK_UPD_SCAN);
  if (forced == kPathFused && fused_ok) return kPathFused;
  if (forced == kPathTiles && tiles_fit(n, nchunks)) return kPathTiles;
  if (forced == kPathSort) return kPathSort;
  if (fused_ok) return kPathFused;
  return tiles_fit(n, nchunks) ? kPathTiles : kPathSort;
}

struct Workspace {
  // zeroed by one memset per call, in this order from the workspace start
  uint32_t *hhead;    // link hash: hcap bucket list heads
  uint32_t *ctl;      // ticket, invalid-entry count, look-back timeout
  uint32_t *touched;  // per chunk: some write reaches it
  uint64_t *gran;     // fused look-back granules, kFusedCols per workgroup
  size_t zero_bytes;  // hhead .. gran (all rows; the call zeroes the rows its grid uses)
  uint32_t hcap;
  uint32_t *kchunk, *kchunk_s, *iota, *idx2;
  uint32_t *prev, *final_of, *next, *delta, *vals, *scan, *sh, *nkey;
  uint32_t *agg, *colpre;  // dense tile path: ntiles x nchunks each
  uint32_t *raw_exact;     // H3C_UPD_EXACT: the chunks' checksums from their bytes
  DevChunk *xdesc;         // ... their create descriptors
  uint32_t *xseg;          // ... and segment partials
  void *tmp;
  size_t tmp_bytes;
};

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

// Lays out (or, with base == nullptr, sizes) the workspace; the same layout serves every path.
int layout(void *base, uint32_t n, uint32_t nchunks, uint64_t chunk_len, uint32_t block_bytes, Workspace &w,
           size_t &total) {
  size_t off = 0;
  auto take = [&](size_t bytes) -> void * {
    void *p = base ? static_cast<char *>(base) + off : nullptr;
    off += align_up(bytes);
    return p;
  };
  const uint32_t bpc = (uint32_t)(chunk_len / block_bytes);
  w.hcap = 256;
  while (w.hcap < n) w.hcap <<= 1;
  w.hhead = (uint32_t *)take(4ull * w.hcap);
  w.ctl = (uint32_t *)take(4ull * kCtlWords);
  w.touched = (uint32_t *)take(4ull * nchunks);
  w.gran = (uint64_t *)take(8ull * kFusedCols * kFusedMaxWG);
  w.zero_bytes = off;
  uint32_t **arrays[] = {&w.kchunk, &w.kchunk_s, &w.iota, &w.idx2, &w.prev, &w.final_of,
                         &w.next,   &w.delta,    &w.vals, &w.scan, &w.nkey};
  for (uint32_t **a : arrays) *a = (uint32_t *)take(4ull * n);
  w.sh = (uint32_t *)take(4ull * bpc);
  const uint64_t tiles_cells = tiles_fit(n, nchunks) ? (uint64_t)((n + kTile - 1) / kTile) * nchunks : 0;
  w.agg = (uint32_t *)take(4ull * tiles_cells);
  w.colpre = (uint32_t *)take(4ull * tiles_cells);
  w.raw_exact = (uint32_t *)take(4ull * nchunks);
  w.xdesc = (DevChunk *)take(sizeof(DevChunk) * nchunks);
  w.xseg = (uint32_t *)take(4ull * nchunks * ((chunk_len + kMinSegBytes - 1) / kMinSegBytes));
  size_t s1 = 0, s2 = 0;
  if (rocprim::radix_sort_pairs<SortConfig>(nullptr, s1, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                (uint32_t *)nullptr, n, 0, 32) != hipSuccess)
    return H3C_ERR_HIP;
  if (rocprim::inclusive_scan_by_key(nullptr, s2, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                     (size_t)n, XorOp()) != hipSuccess)
    return H3C_ERR_HIP;
  w.tmp_bytes = std::max(s1, s2);
  w.tmp = take(w.tmp_bytes);
  total = off;
  return H3C_OK;
}

// Per-(device, polynomial, chunk_len, block_bytes) block-shift tables sh[b] =
// x^(8*(L-(b+1)*G)), built once and kept for the process ("precomputed per chunk size").
// Entries are never freed, so a table handed out stays valid; the cache is bounded.  A miss
// builds the table on a private stream with no lock held (other threads' calls are not held
// up), then publishes it; a miss past the bound, or while `st` is being captured into a graph
// (no allocation or synchronisation allowed then), computes into the caller's workspace on
// `st` instead.
struct ShiftEntry {
  int dev;
  int type;
  uint64_t chunk_len;
  uint32_t block_bytes;
  uint32_t *table;
};
std::mutex g_shift_mu;
std::vector<ShiftEntry> g_shift_cache;
constexpr size_t kShiftCacheMax = 16;

int shift_table(int dev, uint8_t type, uint64_t chunk_len, uint32_t block_bytes, const PolyConsts *pc,
                uint32_t *scratch, hipStream_t st, const uint32_t **out) {
  const uint32_t bpc = (uint32_t)(chunk_len / block_bytes);
  const uint32_t tb = 256;
  auto find = [&]() -> const uint32_t * {
    for (const ShiftEntry &e : g_shift_cache)
      if (e.dev == dev && e.type == type && e.chunk_len == chunk_len && e.block_bytes == block_bytes) return e.table;
    return nullptr;
  };
  bool room = false;
  {
    std::lock_guard<std::mutex> lk(g_shift_mu);
    if (const uint32_t *t = find()) {
      *out = t;
      return H3C_OK;
    }
    room = g_shift_cache.size() < kShiftCacheMax;
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess) cap = hipStreamCaptureStatusNone;
  if (room && cap == hipStreamCaptureStatusNone) {
    uint32_t *table = nullptr;
    hipStream_t priv = nullptr;
    bool built = hipMalloc(&table, 4ull * bpc) == hipSuccess &&
                 hipStreamCreateWithFlags(&priv, hipStreamNonBlocking) == hipSuccess;
    if (built) {
      hipLaunchKernelGGL(upd_shift_kernel, dim3((bpc + tb - 1) / tb), dim3(tb), 0, priv, bpc, chunk_len, block_bytes,
                         pc, table);
      built = hipGetLastError() == hipSuccess && hipStreamSynchronize(priv) == hipSuccess;
    }
    if (priv) (void)hipStreamDestroy(priv);
    if (built) {
      std::lock_guard<std::mutex> lk(g_shift_mu);
      if (const uint32_t *t = find()) {  // another thread published the same geometry meanwhile
        (void)hipFree(table);
        *out = t;
      } else {
        g_shift_cache.push_back({dev, type, chunk_len, block_bytes, table});
        *out = table;
      }
      return H3C_OK;
    }
    if (table) (void)hipFree(table);
    (void)hipGetLastError();
  }
  hipLaunchKernelGGL(upd_shift_kernel, dim3((bpc + tb - 1) / tb), dim3(tb), 0, st, bpc, chunk_len, block_bytes, pc,
                     scratch);
  HIP_TRY(hipGetLastError());
  *out = scratch;
  return H3C_OK;
}

// ---- the fused path's per-stream scratch (no per-call memset) ----
// The control words, touched marks, look-back granules and hash heads of the fused path, owned by the
// library per (device, stream) instead of zeroed in the caller's workspace by a memset per call: hash
// entries, touched marks and granules carry the batch's 8-bit epoch (an entry of an earlier batch reads
// as absent), and the batch's last workgroup puts the control words back and advances the epoch.  The
// scratch is zeroed when it is new, re-laid out (another hash size), suspect (a call failed between its
// launches) or 240 batches on (before the epoch wraps onto live rows).  One call at a time enqueues on a
// scratch (its mutex), so calls from several threads on one stream stay whole; calls on different
// streams use different scratches.  A call being captured into a graph, or one with more than
// kTaggedMaxOps writes, uses its workspace and the memset as before.
#ifndef H3C_UPD_SCRATCH
#define H3C_UPD_SCRATCH 1
#endif
constexpr uint32_t kUsCtl = 0, kUsTouched = kCtlWords, kUsGran = kUsTouched + kFusedCols;
constexpr uint32_t kUsStat = kUsGran + 2 * kFusedCols * kFusedMaxWG;  // per ticket: {epoch << 8 | class, writes, ticks}
constexpr uint32_t kUsHeads = kUsStat + 3 * kFusedMaxWG;
constexpr uint32_t kUsBatches = 240;
constexpr size_t kUsMaxScratches = 64;
struct UpdScratch {
  int dev = -1;
  hipStream_t st = nullptr;
  std::thread::id tid{};  // (hipStreamPerThread: one stream per thread behind one handle)
  uint64_t used = 0;      // LRU tick
  uint32_t *p = nullptr;
  size_t words = 0;
  uint32_t hcap = 0, batches = 0;
  bool dirty = true;
  bool fresh = true;  // newly allocated: its range weights are not learnt yet (zeroed with the rest)
  std::mutex mu;
};
std::mutex g_us_mu;
std::vector<std::unique_ptr<UpdScratch>> g_us;
uint64_t g_us_tick = 0;

// The scratch for (dev, st), locked by `lk`, laid out for `hcap` hash heads and zeroed on `st` if it must be;
// nullptr: none (every scratch busy, or the allocation failed): the caller uses its workspace.  At
// kUsMaxScratches the least recently used idle scratch is freed (after a device synchronisation, so no batch of
// its -- possibly destroyed -- stream is still in flight) and reused.  A stream that ran batches releases its
// scratch with h3c_stream_release before it is destroyed (a new stream may get the same handle value).
UpdScratch *upd_scratch(int dev, hipStream_t st, uint32_t hcap, std::unique_lock<std::mutex> &lk) {
  const std::thread::id tid = st == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id{};
  UpdScratch *s = nullptr;
  {
    std::lock_guard<std::mutex> g(g_us_mu);
    for (auto &x : g_us)
      if (x->dev == dev && x->st == st && x->tid == tid) s = x.get();
    if (!s) {
      if (g_us.size() < kUsMaxScratches) {
        g_us.emplace_back(new UpdScratch);
        s = g_us.back().get();
      } else {  // evict the least recently used scratch no call holds
        for (auto &x : g_us) {
          if (!x->mu.try_lock()) continue;
          if (s == nullptr || x->used < s->used) {
            if (s) s->mu.unlock();
            s = x.get();
          } else {
            x->mu.unlock();
          }
        }
        if (!s) return nullptr;
        if (s->p) {
          int prev = -1;
          (void)hipGetDevice(&prev);
          (void)hipSetDevice(s->dev);
          const bool freed = hipDeviceSynchronize() == hipSuccess && hipFree(s->p) == hipSuccess;
          (void)hipSetDevice(prev);
          if (!freed) {
            (void)hipGetLastError();
            s->mu.unlock();
            return nullptr;
          }
        }
        s->p = nullptr;
        s->words = 0;
        s->mu.unlock();
      }
      s->dev = dev;
      s->st = st;
      s->tid = tid;
      s->dirty = true;
      s->fresh = true;
      s->hcap = 0;
      s->batches = 0;
    }
    s->used = ++g_us_tick;
  }
  lk = std::unique_lock<std::mutex>(s->mu);
  bool same;
  {
    std::lock_guard<std::mutex> g(g_us_mu);  // (the key fields change only under g_us_mu)
    same = s->st == st && s->dev == dev && s->tid == tid;
  }
  if (!same) {  // evicted for another stream between the two locks
    lk.unlock();
    return nullptr;
  }
  const size_t words = kUsHeads + (size_t)hcap;
  if (s->words < words) {
    if (s->p) {  // (this stream's earlier batches may still use it)
      if (hipStreamSynchronize(st) != hipSuccess || hipFree(s->p) != hipSuccess) {
        (void)hipGetLastError();
        s->p = nullptr;
        s->words = 0;
        return nullptr;
      }
    }
    s->p = nullptr;
    s->words = 0;
    if (hipMalloc(reinterpret_cast<void **>(&s->p), 4 * words) != hipSuccess) {
      (void)hipGetLastError();
      s->p = nullptr;
      return nullptr;
    }
    s->words = words;
    s->dirty = true;
    s->fresh = true;
  }
  if (s->dirty || s->hcap != hcap || s->batches >= kUsBatches) {
    // (the range weights are kept across a re-zeroing: they describe the device, not the batches)
    const size_t w0 = s->fresh ? kUsHeads + (size_t)hcap : kUsCtl + kCtlW, w1 = s->fresh ? w0 : kUsCtl + kCtlW + kClasses;
    if (hipMemsetAsync(s->p, 0, 4 * w0, st) != hipSuccess ||
        (w1 < kUsHeads + (size_t)hcap &&
         hipMemsetAsync(s->p + w1, 0, 4 * (kUsHeads + (size_t)hcap - w1), st) != hipSuccess)) {
      (void)hipGetLastError();
      return nullptr;
    }
    s->dirty = false;
    s->fresh = false;
    s->hcap = hcap;
    s->batches = 0;
  }
  ++s->batches;
  return s;
}

// H3C_UPD_EXACT: raw_exact[c] = the raw CRC of chunk c's bytes (one create launch).
int exact_checksums(hipStream_t st, int dev, uint8_t type, const uint64_t *chunk_base, uint32_t nchunks,
                    uint64_t chunk_len, const Workspace &w) {
  const uint32_t poly = type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;
  const uint64_t seg = std::max<uint64_t>(h3c_rt::pick_seg(chunk_len * nchunks, dev), kMinSegBytes);
  const uint32_t spc = (uint32_t)((chunk_len + seg - 1) / seg);
  DevChunk tmpl{};
  tmpl.len = chunk_len;
  tmpl.start = 0xFFFFFFFFu;  // ChecksumInfo::create's default starting checksum (raw register)
  set_fold_consts(tmpl, seg, poly);
  hipLaunchKernelGGL(upd_exact_desc_kernel, dim3((nchunks + 255) / 256), dim3(256), 0, st, chunk_base, nchunks, spc,
                     tmpl, w.xdesc);
  HIP_TRY(hipGetLastError());
  return h3c_rt::launch_crc(st, dev, type, w.xdesc, nchunks, nchunks * spc, spc, chunk_len * nchunks, seg, 0, w.xseg,
                            nullptr, w.raw_exact, nullptr, nullptr, -1, 0);
}

int update_blocks_impl(uint8_t type, const uint64_t *chunk_base_dev, uint32_t nchunks, uint64_t chunk_len,
                       uint32_t block_bytes, const uint32_t *chunk_raw_in_dev, const uint32_t *blk_chunk_dev,
                       const uint32_t *blk_index_dev, const void *payload_dev, uint32_t n_blocks, uint32_t *out_raw_dev,
                       uint32_t *chunk_raw_out_dev, void *workspace_dev, size_t workspace_bytes,
                       uint32_t *n_invalid_dev, uint32_t flags, unsigned long long *counters_dev, void *stream) {
  if (type != H3C_TYPE_CRC32C && type != H3C_TYPE_CRC32) return H3C_ERR_INVALID_ARG;
  if (flags & ~(uint32_t)H3C_UPD_EXACT) return H3C_ERR_INVALID_ARG;  // raw domain only
  if (!block_bytes || block_bytes % kRowBytes || chunk_len % block_bytes || !nchunks) return H3C_ERR_INVALID_ARG;
  if ((uint64_t)nchunks * (chunk_len / block_bytes) >= 0xFFFFFFFFull || n_blocks == 0xFFFFFFFFu)
    return H3C_ERR_INVALID_ARG;
  if (!chunk_base_dev || !chunk_raw_in_dev || !chunk_raw_out_dev || !workspace_dev) return H3C_ERR_INVALID_ARG;
  if (n_blocks && (!blk_chunk_dev || !blk_index_dev || !payload_dev || !out_raw_dev)) return H3C_ERR_INVALID_ARG;
  if (((uintptr_t)payload_dev & 15) != 0) return H3C_ERR_INVALID_ARG;
  const bool exact = (flags & H3C_UPD_EXACT) != 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int dev = 0;
  int rc = h3c_rt::current_device(&dev);
  if (rc) return rc;
  const uint32_t bpc = (uint32_t)(chunk_len / block_bytes);
  Workspace w{};
  size_t need = 0;
  rc = layout(workspace_dev, std::max(n_blocks, 1u), nchunks, chunk_len, block_bytes, w, need);
  if (rc) return rc;
  if (workspace_bytes < need) {
    h3c_rt::set_error_text("h3c_update_blocks: workspace too small (see h3c_update_workspace_bytes)");
    return H3C_ERR_INVALID_ARG;
  }
  const PolyConsts *pc = static_cast<const PolyConsts *>(h3c_rt::device_consts(dev, type));
  const uint32_t num_cu = (uint32_t)std::max(1, h3c_rt::device_num_cu(dev));
  const uint32_t tb = 256, gb = (n_blocks + tb - 1) / tb;
  const uint32_t poly = type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;
  const uint32_t reuse_case = (uint64_t)block_bytes == chunk_len ? 1u : 0u;  // a block write replaces the chunk
  const int path = pick_path(n_blocks, nchunks, block_bytes);
  uint32_t fused_wg = std::min<uint32_t>(std::min(num_cu, kFusedMaxWG), (n_blocks + kFW - 1) / kFW);
                    // instead of 256 with 24-25: -1 us, profiles/r04_update_tail_ab.txt)
  {
    const uint64_t per = ((uint64_t)n_blocks + (uint64_t)fused_wg * kFW - 1) / ((uint64_t)fused_wg * kFW);
    fused_wg = (uint32_t)std::max<uint64_t>(1, ((uint64_t)n_blocks + per * kFW - 1) / (per * kFW));
  }
  // the fused path's hash heads, control words, touched marks and granules: the stream's UpdScratch, or
  // one memset of the workspace's (and the granule rows in use)
  std::unique_lock<std::mutex> us_lock;
  UpdScratch *us = nullptr;
  if (H3C_UPD_SCRATCH && path == kPathFused && n_blocks > 0 && n_blocks <= kTaggedMaxOps) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess) {
      (void)hipGetLastError();
      cap = hipStreamCaptureStatusActive;
    }
    if (cap == hipStreamCaptureStatusNone) us = upd_scratch(dev, st, w.hcap, us_lock);
  }
  const uint32_t tagged = us ? 1u : 0u;
  if (us) {
    w.ctl = us->p + kUsCtl;
    w.touched = us->p + kUsTouched;
    w.gran = reinterpret_cast<uint64_t *>(us->p + kUsGran);
    w.hhead = us->p + kUsHeads;
  } else {
    const size_t zero = path == kPathFused ? (size_t)((char *)(w.gran + (size_t)fused_wg * kFusedCols) - (char *)w.hhead)
                                           : (size_t)((char *)w.gran - (char *)w.hhead);
    HIP_TRY(hipMemsetAsync(w.hhead, 0, zero, st));
  }
  // (a failure after the first launch on the scratch leaves it suspect: the next call zeroes it)
  struct Suspect {
    UpdScratch *s;
    ~Suspect() {
      if (s) s->dirty = true;
    }
  } suspect{us};
  const uint32_t *raw_base = chunk_raw_in_dev;
  if (exact) {
    rc = exact_checksums(st, dev, type, chunk_base_dev, nchunks, chunk_len, w);
    if (rc) return rc;
    raw_base = w.raw_exact;
  }
  if (n_blocks == 0) {
    HIP_TRY(hipMemcpyAsync(chunk_raw_out_dev, chunk_raw_in_dev, 4ull * nchunks, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(upd_finish_kernel, dim3(1), dim3(256), 0, st, w.ctl, 0u, nchunks, raw_base, chunk_raw_in_dev,
                       exact ? 1u : 0u, reuse_case, n_invalid_dev, counters_dev);
    HIP_TRY(hipGetLastError());
    return H3C_OK;
  }
  // previous-writer links: tile match + hash of per-tile last writers (no sort)
  const uint32_t nlt = (n_blocks + kLinkTile - 1) / kLinkTile;
  hipLaunchKernelGGL(upd_tlink_kernel, dim3(nlt + (us ? 1 : 0)), dim3(kLinkTile), 0, st, blk_chunk_dev, blk_index_dev, n_blocks,
                     nchunks, bpc, w.hhead, w.hcap - 1, w.nkey, w.next, w.prev, w.ctl, w.touched, tagged,
                     us ? us->p + kUsStat : nullptr, kFusedMaxWG);
  HIP_TRY(hipGetLastError());
  const uint32_t *sh = nullptr;
  rc = shift_table(dev, type, chunk_len, block_bytes, pc, w.sh, st, &sh);
  if (rc) return rc;
  if (path == kPathFused) {
    h3c_rt::ProfToken tok;
    HIP_TRY(h3c_rt::prof_stamp(dev, tok));
    hipLaunchKernelGGL(upd_fused_kernel, dim3(fused_wg), dim3(kFThreads), 0, st, chunk_base_dev, nchunks, bpc,
                       blk_chunk_dev, blk_index_dev, static_cast<const uint8_t *>(payload_dev), n_blocks, w.prev,
                       w.hhead, w.hcap - 1, w.nkey, w.next, sh, pc, raw_base, chunk_raw_in_dev, exact ? 1u : 0u,
                       reuse_case, w.touched, w.ctl, w.gran, w.scan, out_raw_dev, chunk_raw_out_dev, n_invalid_dev,
                       counters_dev, (uint32_t)(h3c_rt::hook(H3C_HOOK_UPD_LOOKBACK) == 1), tagged,
                       us ? us->p + kUsStat : nullptr, tok.ts);
    HIP_TRY(hipGetLastError());
    suspect.s = nullptr;  // (the batch is enqueued whole: its last workgroup leaves the scratch reset)
    // algorithmic bytes: read new + read old + write back, per block write
    HIP_TRY(h3c_rt::prof_end(st, tok, H3C_PROF_UPDATE, 3ull * block_bytes * n_blocks));
    return H3C_OK;
  }
  hipLaunchKernelGGL(upd_resolve_kernel, dim3(gb), dim3(tb), 0, st, blk_chunk_dev, blk_index_dev, n_blocks, nchunks,
                     bpc, w.hhead, w.hcap - 1, w.nkey, w.next, w.prev, w.final_of);
  HIP_TRY(hipGetLastError());
  const uint32_t blocks = std::min<uint32_t>(num_cu, (n_blocks + kWavesPerBlock - 1) / kWavesPerBlock);
  h3c_rt::ProfToken tok;
  HIP_TRY(h3c_rt::prof_stamp(dev, tok));
  hipLaunchKernelGGL(upd_delta_kernel, dim3(blocks), dim3(kThreads), 0, st, chunk_base_dev, nchunks, bpc, block_bytes,
                     blk_chunk_dev, blk_index_dev, static_cast<const uint8_t *>(payload_dev), n_blocks, w.prev,
                     w.final_of, pc, w.delta, tok.ts);
  HIP_TRY(hipGetLastError());
  HIP_TRY(h3c_rt::prof_end(st, tok, H3C_PROF_UPDATE, 3ull * block_bytes * n_blocks));
  if (path == kPathTiles) {
    const uint32_t ntiles = (n_blocks + kTile - 1) / kTile;
    hipLaunchKernelGGL(upd_tile_kernel, dim3(ntiles), dim3(kTile), 0, st, blk_chunk_dev, blk_index_dev, n_blocks,
                       nchunks, bpc, w.delta, sh, poly, w.scan, w.agg);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(upd_column_kernel, dim3(nchunks), dim3(kTile), 0, st, w.agg, ntiles, nchunks, raw_base,
                       chunk_raw_in_dev, w.touched, w.colpre, chunk_raw_out_dev);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(upd_apply_kernel, dim3(gb), dim3(tb), 0, st, blk_chunk_dev, blk_index_dev, n_blocks, nchunks,
                       bpc, raw_base, w.colpre, w.scan, out_raw_dev);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemcpyAsync(chunk_raw_out_dev, chunk_raw_in_dev, 4ull * nchunks, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(upd_keys_kernel, dim3(gb), dim3(tb), 0, st, blk_chunk_dev, blk_index_dev, n_blocks, nchunks,
                       bpc, w.kchunk, w.iota);
    HIP_TRY(hipGetLastError());
    // stable radix sort of (chunk, sequence index) for the per-chunk scan
    size_t tmp = w.tmp_bytes;
    HIP_TRY(rocprim::radix_sort_pairs<SortConfig>(w.tmp, tmp, w.kchunk, w.kchunk_s, w.iota, w.idx2, n_blocks, 0,
                                                  bits_for((uint64_t)nchunks + 1), st));
    hipLaunchKernelGGL(upd_gather_kernel, dim3(gb), dim3(tb), 0, st, w.kchunk_s, w.idx2, n_blocks, nchunks,
                       blk_index_dev, w.delta, sh, poly, w.vals);
    HIP_TRY(hipGetLastError());
    tmp = w.tmp_bytes;
    HIP_TRY(rocprim::inclusive_scan_by_key(w.tmp, tmp, w.kchunk_s, w.vals, w.scan, (size_t)n_blocks, XorOp(),
                                           rocprim::equal_to<uint32_t>(), st));
    hipLaunchKernelGGL(upd_scatter_kernel, dim3(gb), dim3(tb), 0, st, w.kchunk_s, w.idx2, n_blocks, nchunks, w.scan,
                       raw_base, out_raw_dev, chunk_raw_out_dev);
    HIP_TRY(hipGetLastError());
  }
  if (n_invalid_dev || counters_dev) {
    hipLaunchKernelGGL(upd_finish_kernel, dim3(1), dim3(256), 0, st, w.ctl, n_blocks, nchunks, raw_base,
                       chunk_raw_in_dev, exact ? 1u : 0u, reuse_case, n_invalid_dev, counters_dev);
    HIP_TRY(hipGetLastError());
  }
  return H3C_OK;
}

}  // namespace

extern "C" {

int h3c_stream_release(void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const std::thread::id tid = st == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id{};
  std::vector<std::unique_ptr<UpdScratch>> gone;
  {
    std::lock_guard<std::mutex> g(g_us_mu);
    for (size_t i = 0; i < g_us.size();) {
      if (g_us[i]->st == st && g_us[i]->tid == tid) {
        std::lock_guard<std::mutex> one(g_us[i]->mu);  // (waits out a call enqueueing on it)
        gone.push_back(std::move(g_us[i]));
        g_us.erase(g_us.begin() + (ptrdiff_t)i);
      } else {
        ++i;
      }
    }
  }
  if (gone.empty()) return H3C_OK;
  HIP_TRY(hipStreamSynchronize(st));  // its batches end before their scratch goes
  for (auto &x : gone)
    if (x->p) {
      int prev = -1;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(x->dev);
      const hipError_t e = hipFree(x->p);
      (void)hipSetDevice(prev);
      HIP_TRY(e);
    }
  return H3C_OK;
}

size_t h3c_update_workspace_bytes(uint32_t n_blocks, uint32_t nchunks, uint64_t chunk_len, uint32_t block_bytes) {
  if (!block_bytes) return 0;
  Workspace w{};
  size_t total = 0;
  if (layout(nullptr, std::max(n_blocks, 1u), nchunks, chunk_len, block_bytes, w, total)) return 0;
  return total;
}

int h3c_update_blocks(uint8_t type, const uint64_t *chunk_base_dev, uint32_t nchunks, uint64_t chunk_len,
                      uint32_t block_bytes, const uint32_t *chunk_raw_in_dev, const uint32_t *blk_chunk_dev,
                      const uint32_t *blk_index_dev, const void *payload_dev, uint32_t n_blocks,
                      uint32_t *out_raw_dev, uint32_t *chunk_raw_out_dev, void *workspace_dev,
                      size_t workspace_bytes, uint32_t *n_invalid_dev, void *stream) {
  return update_blocks_impl(type, chunk_base_dev, nchunks, chunk_len, block_bytes, chunk_raw_in_dev, blk_chunk_dev,
                            blk_index_dev, payload_dev, n_blocks, out_raw_dev, chunk_raw_out_dev, workspace_dev,
                            workspace_bytes, n_invalid_dev, 0, nullptr, stream);
}

int h3c_update_blocks_ex(uint8_t type, const uint64_t *chunk_base_dev, uint32_t nchunks, uint64_t chunk_len,
                         uint32_t block_bytes, const uint32_t *chunk_raw_in_dev, const uint32_t *blk_chunk_dev,
                         const uint32_t *blk_index_dev, const void *payload_dev, uint32_t n_blocks,
                         uint32_t *out_raw_dev, uint32_t *chunk_raw_out_dev, void *workspace_dev,
                         size_t workspace_bytes, uint32_t *n_invalid_dev, uint32_t flags,
                         h3c_update_counters *counters_dev, void *stream) {
  return update_blocks_impl(type, chunk_base_dev, nchunks, chunk_len, block_bytes, chunk_raw_in_dev, blk_chunk_dev,
                            blk_index_dev, payload_dev, n_blocks, out_raw_dev, chunk_raw_out_dev, workspace_dev,
                            workspace_bytes, n_invalid_dev, flags,
                            reinterpret_cast<unsigned long long *>(counters_dev), stream);
}

}  // extern "C"
