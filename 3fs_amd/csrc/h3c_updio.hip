// h3c_updio.hip -- general batched chunk updates on MI355X, every per-op step on the device:
// ChunkReplica::update (src/storage/store/ChunkReplica.cc:131-317) with updateChecksum
// (:319-394), or the Rust chunk engine's Engine::update_chunk / Chunk::copy_on_write /
// safe_write (src/storage/chunk_engine/src/core/engine.rs:288-429, alloc/chunk.rs:89-281).
//
// Algebra.  With t the raw CRC of a chunk's bytes (init ~0, no final XOR) every op maps t
// affinely, t' = t*M ^ E (GF(2)[x] mod P, x invertible):
//   WRITE [o, o+len) (n -> n'):  M = x^(8(n'-n)),  E = crc0(new ^ old over the written range,
//                                positioned in an n'-byte string; old bytes past n are 0)
//   full write (o = 0, len >= n, or a syncing write):  M = 0, E = raw(payload)
//   TRUNCATE to l < n:  M = x^(-8(n-l)), E = crc0(old[l, n)) positioned likewise
//   grow to l > n (zero fill):  M = x^(8(l-n)), E = 0
// The stored checksum s follows one of four rules per op, exactly as updateChecksum picks
// them: case (i) s' = 0; reuse (ii) / prefix+suffix re-read (iv): s' = t'; append (iii):
// s' = s*M ^ E (the same M, E: combine(~s, w, len) = s*x^(8len) ^ crc0(w)); a combine of
// length 0 (TRUNCATE / EXTEND at offset == size): s' = s.  So each op is an element
//   (t, s) -> (t*M ^ E, t*A ^ s*B ^ F)
// of a monoid, and a segmented scan per chunk in sequence order gives every op's stored
// checksum from the chunk's (t0, s0).  t0 is s0 when stored checksums are trusted (default),
// or the CRC of the chunk's bytes (H3C_UPD_EXACT, or a stored type of another polynomial).
//
// E needs the old bytes an op overwrites or cuts, and those depend on earlier ops.  Every op
// is cut into fragments, one per 4 KiB block (absolute addresses) it touches.  The fragments
// of one block form a chain in sequence order, and one wavefront walks a chain: it loads the
// block once into registers, applies each fragment in order (CRC of new ^ old, then the new
// bytes), XORs each fragment's CRC, moved to its op's end, into that op's E, and stores the
// block once.  A block's traffic is one read, one write and its payload bytes.
//
// Pipeline (two streams, one graph per repeated batch; one device->host read at the end):
//   prep       per op: validation, payload piece count, sort key (chunk); per chunk: the piece
//              count of its bytes when t0 comes from them
//   pieces     op_piece_crc_kernel: payload and chunk CRCs in 4 KiB pieces (second stream), one
//              launch -> A6 verify (:193-207) and t0 per chunk, one launch
//   sort       (chunk, op) pairs, stable (counting sort; rocPRIM merge sort past 16 key bits)
//   sizes      segmented scan of the size / type maps {n -> max(n, b)} u {n -> c}
//   classify   per op: size before / after, the reference's case, fragment range
//   fragments  expansion, chain links (LDS tile grouping + hash of per-tile last links),
//              chain heads
//   blocks     one wave per chain: bytes in place, E per op
//   scan       segmented scan of the (t, s) elements; results, final chunk states, counters
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#include "h3c_common.hpp"

namespace {

constexpr uint32_t kNil = 0xFFFFFFFFu;
constexpr uint32_t kBlk = 4096;      // fragment granularity: 3FS's IO alignment (kAIOAlignSize)
constexpr uint32_t kPieceBytes = 4096;

using h3c_rt::StreamDrain;

// t-map kinds and s-map kinds (see the header comment)
enum : uint8_t { kT_IDENT = 0, kT_DELTA = 1, kT_FULL = 2 };
enum : uint8_t { kS_IDENT = 0, kS_ZERO = 1, kS_SET_T = 2, kS_APPEND = 3, kS_KEEP = 4 };
// counter codes of an applied op
enum : uint8_t { kC_NONE_ = 0, kC_NONE = 1, kC_REUSE = 2, kC_COMBINE = 3, kC_READ = 4, kC_RECALC = 5 };
// device counter slots (h3c_update_counters order)
enum { kCtrNone, kCtrReuse, kCtrCombine, kCtrRead, kCtrRecalc, kCtrMismatch, kCtrInvalid, kCtrStale, kCtrN };
// device scalars: the payload kernel's work counter, the chain-head counter
// misc words: [kMiscA6] some client checksum failed A6 (the speculative pass is void);
// [kMiscOutF], [kMiscOutA6]: the fragment count and that flag, copied for the one read-back;
// [kMiscT0], [kMiscT1]: the block kernel's first start and last end (wall clock, u64 each), its
// timing when it runs inside a replayed graph (read back with the two words before them)
// [kMiscTicket]: uio_front_kernel's tile ticket; [kMiscPBVoid]: a uio_phaseb_kernel tile gave up waiting;
// [kMiscPBDone]: uio_phaseb_kernel's finished tiles (the last one copies [kMiscOutF, kMiscN) to the host);
// [kMiscFast]: the fast branch's outcome (kFast*; 0 on the general pipeline); [kMiscErr]: a kernel met an
// inconsistent table (a piece table that disagrees with its items) -- the call fails.
// Past kMiscN (not copied back): [kMiscFDone] the fast tail's finished workgroups, [kMiscFVoid] one of
// its workgroups reported the pass void; [kMiscSlow] is unused (the slow word lives in the thread's
// FastScratch); [12] is unused.
enum {
  kMiscTicket = 0, kMiscA6 = 1, kMiscOutF = 2, kMiscOutA6 = 3, kMiscT0 = 4, kMiscT1 = 6, kMiscPBVoid = 8,
  kMiscPBDone = 9, kMiscFast = 10, kMiscErr = 11, kMiscN = 12,
  kMiscFDone = 13, kMiscFVoid = 14, kMiscSlow = 15, kMiscWords = 16
};
enum : uint32_t { kFastDone = 1, kFastAbort = 2, kFastVoid = 3 };

// ---------------------------------------------------------------- scan elements

// Size and type maps: n -> cst ? v : max(n, v); type -> tset ? t : type.
struct SzTy {
  uint32_t v;
  uint8_t cst, tset, t, pad;
};
struct SzTyOp {
  __host__ __device__ SzTy operator()(const SzTy &a, const SzTy &b) const {  // a, then b
    SzTy r;
    if (b.cst) {
      r.v = b.v;
      r.cst = 1;
    } else {
      r.v = a.v > b.v ? a.v : b.v;
      r.cst = a.cst;
    }
    r.tset = b.tset ? 1 : a.tset;
    r.t = b.tset ? b.t : a.t;
    r.pad = 0;
    return r;
  }
};

__host__ __device__ inline uint32_t hd_gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  if (a == 0 || b == 0) return 0;
  if (a == kOne) return b;
  if (b == kOne) return a;
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

// An affine map r -> r*m ^ e (GF(2)[x] mod P).  The (t, s) map of an op is two of them:
// t' = t*M ^ E, and -- once every op's t' is known from the first scan -- s' = s*B ^ c with
// c = t' (reuse / re-read), E (append, B = M), or 0 (case (i), keep).
struct Aff {
  uint32_t m, e;
};
// The general composition is a real call, so a scan whose elements take the two short cuts
// below never executes the bit-serial multiplies (inlined, they were if-converted and ran for
// every element: 28 us per 100k-op scan on config 3, where every element is x^0 or 0).
__host__ __device__ __attribute__((noinline)) Aff aff_general(Aff x, Aff y, uint32_t poly) {
  return Aff{hd_gf_mul(x.m, y.m, poly), hd_gf_mul(x.e, y.m, poly) ^ y.e};
}
struct AffOp {
  uint32_t poly;
  __host__ __device__ Aff operator()(const Aff &x, const Aff &y) const {  // x, then y
    // most ops keep the chunk length (m = x^0): composing them is a XOR
    if (y.m == kOne) return Aff{x.m, x.e ^ y.e};
    if (y.m == 0u) return y;  // y forgets its input (case iv / full rewrite: s' = t')
    return aff_general(x, y, poly);
  }
};

// Per op, in (chunk, sequence) order.
struct OpPos {
  uint32_t op;      // original index
  uint32_t nb, na;  // chunk size before / after
  uint32_t r0, r1;  // chunk-relative byte range its fragments cover
  uint32_t status;
  uint8_t tk, sk;   // t-map / s-map kinds
  uint8_t tb, ta;   // stored type before / after
  uint8_t ccode;    // counter of an applied op (kC_*)
  uint8_t ncomb;    // Rust engine: checksum_combine increments (0-2)
  uint8_t pf;       // kPos* flags
  uint8_t pad;
};
// A "fold" op's client checksum (A6) is checked by the block kernel as it reads the payload --
// the payload is read once -- instead of by the piece pass before it.  That is sound only for
// an op whose failure changes nothing but its own bytes and checksum: a typed WRITE whose bytes
// lie in one 4 KiB block and which keeps the chunk's size and stored type (its failure then
// leaves every later op's case, size and fragments as speculated; the block kernel skips its
// bytes and phase B treats it as the identity).  Other candidates are checked by a late piece
// pass before the block kernel, beside the fragment stage.
constexpr uint8_t kPosFold = 1;

// One block of one op (64 B).  Ranges are block-relative byte offsets in [0, 4096].
struct FragDesc {
  uint64_t blk;     // absolute address of the 4 KiB block
  uint64_t src;     // payload address of block offset 0 (meaningful on [w0, w1) only)
  uint32_t p;       // the op's position (E accumulator index)
  uint32_t rsv;     // (the next fragment of the same block is in its own array, fnext[])
  uint16_t w0, w1;  // new bytes
  uint16_t q0, q1;  // old bytes entering the CRC delta
  uint16_t z0, z1;  // zero fill
  uint16_t k0, k1;  // the chunk's own bytes in this block (loads / stores)
  uint32_t mult;    // CRC contribution shift x^(8e), e = the op's size after - block end (chunk-relative)
  uint32_t flags;
  uint32_t op;      // kFragA6: the op, its client checksum and payload length
  uint32_t expect;
  uint32_t len;
  uint32_t pad;
};
static_assert(sizeof(FragDesc) == 64, "FragDesc is one 64-byte record");
constexpr uint32_t kFragCrc = 1u, kFragWrite = 2u, kFragHead = 4u, kFragA6 = 8u;
// kFragSolo: the op's only fragment.  The block kernel stores its delta CRC unshifted with the
// shift beside it (eacc[2p], eacc[2p+1]) and phase B multiplies, one op per thread, instead of a
// bit-serial GF(2) multiply issued by the whole wave for lane 0.  Other fragments XOR their
// shifted contributions into eacc[2p] (eacc[2p+1] stays 0: nothing left to multiply).
constexpr uint32_t kFragSolo = 16u;

// counters: a workgroup-aggregated add -- wave sums into LDS, one global atomic per counter
// and workgroup (call from workgroup-uniform control flow; `sh` holds kCtrN slots)
__device__ __forceinline__ void ctr_add_block(unsigned int *sh, unsigned long long *ctr, const uint32_t (&v)[8]) {
  if (threadIdx.x < 8) sh[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t x = v[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, 64);
    if ((threadIdx.x & 63) == 0 && x) atomicAdd(&sh[k], x);
  }
  __syncthreads();
  if (threadIdx.x < 8 && sh[threadIdx.x]) atomicAdd(&ctr[threadIdx.x], (unsigned long long)sh[threadIdx.x]);
}

// ---------------------------------------------------------------- kernels

// Chunks whose starting CRC t0 comes from their bytes (H3C_UPD_EXACT, or a stored checksum not
// of this polynomial).
__device__ __forceinline__ bool needs_init(const h3c_chunk_state &cs, uint8_t poly_type, uint32_t exact) {
  return cs.size && cs.size <= cs.chunk_size && (exact || cs.type != poly_type);
}

// A typed, non-empty, non-syncing WRITE whose payload lands in one 4 KiB block of its chunk
// (absolute addresses): its A6 check may move into the block kernel (kPosFold, decided by
// classify).  `st` is the op's status so far.
#ifndef H3C_UIO_FOLD
#define H3C_UIO_FOLD 1  // A6 checks of local one-block writes in the block kernel (0: all in the piece pass)
#endif
__device__ __forceinline__ bool fold_candidate(const h3c_update_io &io, const h3c_chunk_state &cs, uint32_t st) {
  if (!H3C_UIO_FOLD) return false;
  if (st != H3C_OK || io.kind != H3C_UPD_WRITE || io.checksum_type == H3C_TYPE_NONE || !io.length ||
      (io.flags & H3C_IO_SYNCING))
    return false;
  const uint64_t a = cs.base + io.offset;
  return (a >> 12) == ((a + io.length - 1) >> 12);
}

// Cross-workgroup traffic inside a kernel (the prep kernel's scan, uio_front_kernel, uio_phaseb_kernel) uses relaxed agent-scope atomics only (sc1 loads and
// stores, coherent across the XCDs' L2s) and a vmcnt wait before a flag store: a release / acquire
// at agent scope would write back / invalidate the whole L2 (buffer_wbl2 / buffer_inv sc1) every
// time -- with one per published hash entry, the first version of this kernel took 117-170 us.
template <class T>
__device__ __forceinline__ T ld_agent(T *p) {  // a relaxed load at the coherence point
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_agent(T *p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void pub_flag(uint32_t *f, uint32_t v) {
  stores_done();  // this thread's payload stores are at the coherence point before the flag
  st_agent(f, v);
}
// Validation (ChunkReplica.cc:140-145 range check; the ABI's preconditions), sort keys, and
// the piece counts of the early piece-CRC pass: op i's payload is item i (fold candidates have
// none: the block kernel or the late pass checks them), chunk c's bytes (when t0 comes from
// them) item n + c; thread j handles item j (n + max(nchunks, 1) + 1 threads at least).
// With `pbase`, the kernel also scans the piece counts, in two levels and with no waiting: each
// tile of kPrepTile items writes its items' exclusive offsets within the tile to pbase[] and its
// total to tbase[k]; the last tile to finish turns tbase[] into the tiles' exclusive bases (item
// i's offset is pbase[i] + tbase[i / kPrepTile]; op_piece_crc_kernel adds them).  `sstate`
// (zeroed by the caller): [0] unused, [1] finished tiles, [2] the total, [3 + k] tbase[k].
// Zeroes up to four word ranges, grid-strided (the prep kernel's scan words; a new or suspect
// FastScratch before the fast branch uses it).
__global__ void uio_zero_kernel(uint32_t *__restrict__ a, uint32_t na, uint32_t *__restrict__ b, uint32_t nb,
                                uint32_t *__restrict__ c, uint32_t nc, uint32_t *__restrict__ d, uint32_t nd) {
  const uint32_t s = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < na + nb + nc + nd; i += s) {
    if (i < na) a[i] = 0;
    else if (i < na + nb) b[i - na] = 0;
    else if (i < na + nb + nc) c[i - na - nb] = 0;
    else d[i - na - nb - nc] = 0;
  }
}
// ---- the fast branch's per-op tables (see uio_fast_kernel) ----
// A batch whose every op is a typed, one-block, in-size WRITE (the block-aligned overwrites of
// BASELINE config 3, or any write inside one 4 KiB block of a chunk stored under the batch's
// polynomial that keeps its size) needs none of the general pipeline's sizes, cases or fragment
// numbering: op i is its own one fragment, in sequence order.  The prep kernel builds op i's
// fragment record and links the ops of one block inside its 1,024-op tile; each tile's last op of
// a block is pushed on a hash bucket list.  uio_fast_kernel does the rest in one launch.
struct FastArgs {
  FragDesc *frag;           // op i's fragment (its 4 KiB block)
  unsigned long long *key;  // (chunk << 36) | block address >> 12
  // per op {tprev, tnext, tfirst, bnext}: the previous / next op of the same block in op i's prep tile
  // (kNil: none); for a tile's last op of a block, the tile's first op of it and the next entry of its
  // bucket list (the tiles' last ops, entries index + 1; 0 ends a list)
  uint4 *link;
  uint32_t *head;           // bucket heads, hmask + 1 of them (zeroed by uio_zero_kernel)
  uint32_t hmask;
  unsigned long long *dv;   // per op: {state << 32 | delta CRC} (state 1: applied, 2: failed A6)
  uint32_t *slow;           // set when some op is not one this branch takes (FastScratch word 0)
  const PolyConsts *pc;
  uint4 *chain;             // per op (uio_fast_link_kernel): {bit 31: starts its block's chain, bits 0-25: the
                            //  next op's new bytes w0 | w1 << 13; the block's next op; the next op's payload
                            //  address at block offset 0 (lo, hi)}
};
__device__ void fast_prep_tile(const FastArgs &fa, uint32_t i, uint32_t n, const h3c_update_io &io,
                               const h3c_chunk_state &cs, uint32_t st, uint8_t poly_type, uint32_t std_domain);
// An op's validation status before any case analysis (ChunkReplica::update's argument checks, :141-180,
// and the documented limits of this engine); cs is the op's chunk state (ignored for a COMMIT or a chunk
// index out of range).
__device__ __forceinline__ uint32_t op_status(const h3c_update_io &io, const h3c_chunk_state &cs, uint32_t nchunks,
                                              uint8_t poly_type, uint32_t std_domain) {
  uint32_t st = H3C_OK;
  const uint32_t c = io.chunk;
  const bool kind_ok = io.kind == H3C_UPD_WRITE || io.kind == H3C_UPD_TRUNCATE || io.kind == H3C_UPD_EXTEND ||
                       io.kind == H3C_UPD_REMOVE || io.kind == H3C_UPD_COMMIT;
  if (c >= nchunks || !kind_ok) return H3C_ERR_INVALID_ARG;
  if (io.kind == H3C_UPD_COMMIT) return H3C_OK;
  const bool syncing = (io.flags & H3C_IO_SYNCING) != 0;
  if (!cs.base || (io.checksum_type != H3C_TYPE_NONE && io.checksum_type != poly_type)) st = H3C_ERR_INVALID_ARG;
  if (cs.size > cs.chunk_size) st = H3C_ERR_INVALID_ARG;  // a corrupt chunk state
  // documented limit: a TRUNCATE / EXTEND of a chunk stored (at the start of the batch) under the
  // other polynomial -- its stored type would be kept (:328-332), and this batch CRCs in its own
  if (!std_domain && (io.kind == H3C_UPD_TRUNCATE || io.kind == H3C_UPD_EXTEND) && cs.type != H3C_TYPE_NONE &&
      cs.type != poly_type)
    st = H3C_ERR_INVALID_ARG;
  if (io.kind == H3C_UPD_REMOVE) {  // doRemove's form (StorageOperator.cc:808-815); no range check (:141)
    if (io.offset || io.length || io.checksum_type != H3C_TYPE_NONE || syncing) st = H3C_ERR_INVALID_ARG;
  } else {
    // :141-145 against writeIO.chunkSize (H3C_IO_CHUNK_SIZE; else the chunk's own), then :171-180
    const bool own = !std_domain && (io.flags & H3C_IO_CHUNK_SIZE);
    const uint32_t wcs = own ? io.chunk_size : cs.chunk_size;
    if (io.offset >= wcs || (uint64_t)io.offset + io.length > wcs) st = H3C_ERR_INVALID_ARG;
    if (io.kind == H3C_UPD_WRITE && io.length && !io.payload) st = H3C_ERR_INVALID_ARG;
    if (syncing && (io.kind != H3C_UPD_WRITE || io.offset)) st = H3C_ERR_INVALID_ARG;
    if (st == H3C_OK && wcs != cs.chunk_size) st = H3C_ERR_CHUNK_SIZE_MISMATCH;
    // A6 on a TRUNCATE / EXTEND: create(type, <no data>, length) is {NONE, 0} (:193-207);
    // the Rust engine verifies only data (engine.rs:297)
    if (st == H3C_OK && !std_domain && io.kind != H3C_UPD_WRITE && io.checksum_type != H3C_TYPE_NONE && io.length)
      st = H3C_ERR_CHECKSUM_MISMATCH;
  }
  return st;
}

#ifndef H3C_PREP_TILE
#define H3C_PREP_TILE 1024  // items per prep-kernel tile (a power of two, 64..1024)
#endif
constexpr uint32_t kPrepTile = H3C_PREP_TILE;
constexpr uint32_t kFastChunksLds = 128;  // (= kFastCols: the chunks a fast-branch batch may name)
__global__ __launch_bounds__(kPrepTile) void uio_prep_kernel(
    const h3c_update_io *__restrict__ ios, uint32_t n, const h3c_chunk_state *__restrict__ chunks, uint32_t nchunks,
    uint8_t poly_type, uint32_t std_domain, uint32_t exact, uint32_t *__restrict__ status, uint32_t *__restrict__ key,
    uint32_t *__restrict__ idx, uint32_t *__restrict__ npieces, uint32_t *__restrict__ paycrc0,
    uint32_t *__restrict__ eacc, unsigned long long *__restrict__ ctr, uint32_t *__restrict__ misc,
    uint32_t *__restrict__ a6, uint32_t *__restrict__ fz, uint32_t fz_words, uint32_t *__restrict__ hhead,
    uint32_t hcap, uint32_t *__restrict__ gnext, uint32_t *__restrict__ fnext, uint32_t fcap,
    uint32_t *__restrict__ pbase, uint32_t *sstate, FastArgs fa) {
  __shared__ uint32_t s_w[kPrepTile / 64], s_last;
  // No tile waits on another (the last one to finish scans the tile totals), so tiles need no
  // ticket: one agent-scope atomic per tile on one address serialises beyond the XCDs' L2s.
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // the front kernel's initialisations, grid-strided (the grid may cover only the items)
  const uint32_t init_n = max(max(fz_words, hcap), fcap);
  for (uint32_t j = i; j < init_n; j += gridDim.x * blockDim.x) {
    if (j < fz_words) fz[j] = 0;        // the one-pass front's tile states (uio_front_kernel)
    if (j < hcap) hhead[j] = 0xFFFFFFFFu;  // ... its link hash's bucket heads
    if (j < fcap) {                     // ... its bucket lists' next pointers and the chains'
      gnext[j] = 0xFFFFFFFEu;           // (kPending)
      fnext[j] = 0xFFFFFFFFu;           // (kNil)
    }
  }
  if (i < kCtrN) ctr[i] = 0;
  if (i < kMiscSlow) misc[i] = i == kMiscT0 || i == kMiscT0 + 1 ? 0xFFFFFFFFu : 0u;  // (kMiscSlow: uio_zero_kernel)
  // the fast branch without the piece pass (not exact): only the validation feeds it (fast_prep_tile);
  // the general pipeline's arrays are not written (a batch that leaves the branch runs its own prep).
  // Its chunk table (<= kFastCols states) is read into LDS beside the ops' loads, so an op's chunk
  // state is not a second round trip after its op record.
  const bool lean = fa.head && !pbase;
  __shared__ h3c_chunk_state s_cs[kFastChunksLds];
  h3c_update_io io_pre{};
  if (i < n) io_pre = ios[i];
  if (lean) {
    if (threadIdx.x < nchunks && threadIdx.x < kFastChunksLds) s_cs[threadIdx.x] = chunks[threadIdx.x];
    __syncthreads();
  }
  // chunk items n + c for c < C = max(nchunks, 1) (the piece pass's NP = n + C items), then the
  // scan's extra entry: pbase[n + C] = total
  const uint32_t C = nchunks ? nchunks : 1u;
  uint32_t np = 0;
  if (!lean && i >= n && i < n + C) {
    const uint32_t c = i - n;
    if (c < nchunks) {
      const h3c_chunk_state cs = chunks[c];
      np = needs_init(cs, poly_type, exact) ? (cs.size + kPieceBytes - 1) / kPieceBytes : 0u;
    }
    npieces[i] = np;
    paycrc0[i] = 0;
  }
  if (!lean && i == n + C) npieces[i] = 0;
  h3c_update_io f_io{};
  h3c_chunk_state f_cs{};
  uint32_t f_st = H3C_ERR_INVALID_ARG;
  if (i < n) {
    if (!lean) {
      paycrc0[i] = 0;  // XOR accumulators of the piece and block kernels
      eacc[2 * i] = 0;
      eacc[2 * i + 1] = 0;
      a6[i] = 0;       // A6 verdicts (the early pass, the front / late checks, the block kernel)
    }
    const h3c_update_io io = io_pre;
    const uint32_t c = io.chunk;
    h3c_chunk_state cs_v{};
    if (c < nchunks && io.kind != H3C_UPD_COMMIT) cs_v = lean ? s_cs[c] : chunks[c];
    const uint32_t st = op_status(io, cs_v, nchunks, poly_type, std_domain);
    if (!lean) {
      status[i] = st;
      key[i] = c < nchunks ? c : nchunks;
      idx[i] = i;
      const bool cand = st == H3C_OK && fold_candidate(io, chunks[c], st);
      np = (st == H3C_OK && io.kind == H3C_UPD_WRITE && io.length && !cand) ? (io.length + kPieceBytes - 1) / kPieceBytes
                                                                            : 0;
      npieces[i] = np;
    }
    f_io = io;
    f_st = st;
    if (c < nchunks) f_cs = lean ? s_cs[c] : chunks[c];
  }
  if (fa.head) fast_prep_tile(fa, i, n, f_io, f_cs, f_st, poly_type, std_domain);  // (the whole workgroup)
  if (!pbase) return;
  // exclusive scan of the items' piece counts: in the tile, then the tile's base by look-back
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t x = np;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
  for (uint32_t w = 0; w < kPrepTile / 64; ++w) {
    if (w < wave) wpre += s_w[w];
    tot += s_w[w];
  }
  const uint32_t k = blockIdx.x, nscan = (n + C + 1 + kPrepTile - 1) / kPrepTile;
  if (k >= nscan) return;  // (whole tile: no item)
  uint32_t *tbase = sstate + 3;
  if (i <= n + C) pbase[i] = wpre + x - np;
  if (t == 0) {
    st_agent(&tbase[k], tot);
    stores_done();  // the tile total is at the coherence point before the count
    s_last = atomicAdd(&sstate[1], 1u) + 1 == nscan;
  }
  __syncthreads();
  if (!s_last) return;
  // the last tile: exclusive scan of the nscan tile totals, in place; thread t takes a contiguous
  // group of them (all its loads in flight at once), the group sums are scanned across the tile
  const uint32_t G = (nscan + kPrepTile - 1) / kPrepTile, g0 = t * G, g1 = min(g0 + G, nscan);
  uint32_t gsum = 0;
  for (uint32_t j = g0; j < g1; ++j) gsum += ld_agent(&tbase[j]);
  uint32_t y = gsum;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t z = (uint32_t)__shfl_up((int)y, o, 64);
    if (lane >= o) y += z;
  }
  __syncthreads();  // (s_w reuse)
  if (lane == 63) s_w[wave] = y;
  __syncthreads();
  uint32_t run = 0, all = 0;
  for (uint32_t w = 0; w < kPrepTile / 64; ++w) {
    if (w < wave) run += s_w[w];
    all += s_w[w];
  }
  run += y - gsum;  // this group's base
  for (uint32_t j = g0; j < g1; ++j) {
    const uint32_t v = ld_agent(&tbase[j]);
    st_agent(&tbase[j], run);
    run += v;
  }
  if (t == 0) st_agent(&sstate[2], all);
}

__device__ __forceinline__ bool applied_kind(uint8_t kind) {
  return kind == H3C_UPD_WRITE || kind == H3C_UPD_TRUNCATE || kind == H3C_UPD_EXTEND || kind == H3C_UPD_REMOVE;
}

// A6 (:193-207, engine.rs:297-312): the payload's raw CRC against the client's checksum.
// The verdicts go to a6[] and one flag: the sizes, cases and fragments are computed meanwhile
// assuming every check passes (a corrupted transfer is rare), and a failed check voids that
// speculative pass (the block kernel writes nothing; the host redoes from the sizes on).
__device__ __forceinline__ void verify_op(uint32_t i, const h3c_update_io *__restrict__ ios,
                                          const uint32_t *__restrict__ paycrc0, const PolyConsts *__restrict__ pc,
                                          uint32_t std_domain, const uint32_t *__restrict__ status,
                                          uint32_t *__restrict__ payraw, uint32_t *__restrict__ a6,
                                          uint32_t *__restrict__ misc, const h3c_chunk_state *__restrict__ skip_cand) {
  const h3c_update_io io = ios[i];
  // skip_cand: the early pass, which carries no fold candidate's payload (their verdicts come from
  // the block kernel or the front kernel, concurrently: a6[] of a skipped op is not written here;
  // the prep kernel zeroed it)
  if (io.kind == H3C_UPD_WRITE && status[i] == H3C_OK && !(skip_cand && fold_candidate(io, skip_cand[io.chunk], H3C_OK))) {
    const uint32_t poly = pc->poly;
    const uint32_t raw = io.length ? paycrc0[i] ^ dgf_mul_fast(0xFFFFFFFFu, dxpow8_fast(io.length, pc, poly), poly)
                                   : 0xFFFFFFFFu;
    payraw[i] = raw;
    const bool bad = io.checksum_type != H3C_TYPE_NONE && io.length && (std_domain ? ~raw : raw) != io.checksum_value;
    a6[i] = bad ? 1u : 0u;
    if (bad) atomicOr(&misc[kMiscA6], 1u);
  }
}

// After a failed A6: the verdicts into the statuses, and the flag cleared for the redo.
__global__ void uio_merge_a6_kernel(const uint32_t *__restrict__ a6, uint32_t n, uint32_t *__restrict__ status,
                                    uint32_t *__restrict__ misc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) misc[kMiscA6] = 0;
  if (i < n && a6[i] && status[i] == H3C_OK) status[i] = H3C_ERR_CHECKSUM_MISMATCH;
}

// The size / type map of one op.
__device__ __forceinline__ SzTy sz_elem_of(const h3c_update_io &io, uint32_t st, uint8_t poly_type,
                                           uint32_t std_domain) {
  SzTy e{0, 0, 0, 0, 0};
  if (st == H3C_OK && applied_kind(io.kind)) {
    switch (io.kind) {
      case H3C_UPD_WRITE:  // doRealWrite (:122-124); a syncing write sets meta.size = length (:289)
        if (io.flags & H3C_IO_SYNCING) {
          e.cst = 1;
          e.v = io.length;
        } else {
          e.v = io.offset + io.length;
        }
        e.tset = 1;
        e.t = std_domain ? poly_type : io.checksum_type;  // :392
        break;
      case H3C_UPD_TRUNCATE:  // :261-273: the new length either way
        e.cst = 1;
        e.v = io.length;
        break;
      case H3C_UPD_EXTEND:
        e.v = io.length;
        break;
      case H3C_UPD_REMOVE:  // case (i) with a NONE checksum (:334-336, :392)
        e.tset = 1;
        e.t = H3C_TYPE_NONE;
        break;
      default:
        break;
    }
    if (std_domain && io.kind != H3C_UPD_WRITE) {  // the engine reports every result as CRC32C (ChunkEngine.cc:66)
      e.tset = 1;
      e.t = poly_type;
    }
  }
  return e;
}

// The size / type map of each op, in sorted order.
__global__ void uio_sz_elem_kernel(const h3c_update_io *__restrict__ ios, const uint32_t *__restrict__ order, uint32_t n,
                                   const uint32_t *__restrict__ status, uint8_t poly_type, uint32_t std_domain,
                                   SzTy *__restrict__ el) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t i = order[p];
  el[p] = sz_elem_of(ios[i], status[i], poly_type, std_domain);
}

__device__ __forceinline__ uint32_t blocks_of(uint64_t base, uint32_t r0, uint32_t r1) {
  return r1 > r0 ? (uint32_t)(((base + r1 - 1) >> 12) - ((base + r0) >> 12) + 1) : 0u;
}

// The reference's case analysis for op i at sorted position p of chunk c (ChunkReplica.cc:246,
// 319-394; engine.rs:375-423 and chunk.rs:89-281 in the std domain), the maps' kinds, and the
// op's fragment range.  `ex` / `in` are the size / type maps of the chunk's ops before it and
// through it (identity: SzTy{}).  Returns the op's fragment count; *late: a fold candidate whose
// A6 check must happen before the block kernel.
__device__ __forceinline__ uint32_t classify_op(const h3c_update_io &io, uint32_t i, uint32_t st, uint32_t c,
                                                uint32_t nchunks, const h3c_chunk_state &cs, const SzTy &ex,
                                                const SzTy &in, uint8_t poly_type, uint32_t std_domain,
                                                uint32_t nofold, OpPos &r, bool &late) {
  r = OpPos{};
  r.op = i;
  r.status = st;
  late = false;
  if (c >= nchunks) return 0;  // names no chunk of the batch
  const uint32_t nb = ex.cst ? ex.v : (cs.size > ex.v ? cs.size : ex.v);
  const uint32_t tb = ex.tset ? ex.t : cs.type;
  const uint32_t na_scan = in.cst ? in.v : (cs.size > in.v ? cs.size : in.v);
  r.nb = nb;
  r.na = nb;
  r.tb = (uint8_t)tb;
  r.ta = (uint8_t)tb;
  r.tk = kT_IDENT;
  r.sk = kS_IDENT;
  const bool applied = r.status == H3C_OK && applied_kind(io.kind);
  if (applied) {
    const uint32_t na = na_scan;
    r.na = na;
    const uint32_t o = io.offset, len = io.length;
    const bool syncing = (io.flags & H3C_IO_SYNCING) != 0;
    if (io.kind == H3C_UPD_WRITE) {
      const bool full = syncing || (o == 0 && len >= nb);
      if (full) {
        r.tk = kT_FULL;
        r.r0 = 0;
        r.r1 = len;
      } else if (len || o > nb) {
        r.tk = kT_DELTA;
        r.r0 = o > nb ? nb : o;
        r.r1 = o + len;
      }
      if (!std_domain) {
        const uint8_t tw = io.checksum_type;
        r.ta = tw;
        if (tw == H3C_TYPE_NONE || na == 0) {  // (i)
          r.sk = kS_ZERO;
          r.ccode = kC_NONE;
        } else if (o == 0 && len == na) {  // (ii): the client's value, verified = raw(payload) = t'
          r.sk = kS_SET_T;
          r.ccode = kC_REUSE;
        } else if (tw == tb && nb > 0 && o == nb) {  // (iii)
          r.sk = kS_APPEND;
          r.ccode = kC_COMBINE;
        } else {  // (iv)
          r.sk = kS_SET_T;
          r.ccode = kC_READ;
        }
      } else {
        r.ta = poly_type;
        if (syncing || (len > 0 && o < nb)) {  // copy_on_write (engine.rs:377-391)
          r.sk = kS_SET_T;
          r.ccode = (syncing || (o == 0 && len >= nb)) ? kC_REUSE : kC_RECALC;  // chunk.rs:112,152-158
        } else if (na > nb) {  // safe_write append / zero pad (chunk.rs:200-276)
          r.sk = kS_APPEND;
          r.ccode = kC_COMBINE;
          const bool aligned = nb % kBlk == 0 && o % kBlk == 0 && (len == 0 || (io.payload % kBlk == 0 && len % kBlk == 0));
          r.ncomb = aligned ? (uint8_t)((o > nb ? 1 : 0) + (len ? 1 : 0)) : (uint8_t)1;
        } else {
          r.sk = kS_KEEP;
        }
      }
    } else if (io.kind == H3C_UPD_TRUNCATE || io.kind == H3C_UPD_EXTEND) {
      if (na < nb) {
        r.tk = kT_DELTA;
        r.r0 = na;
        r.r1 = nb;
      } else if (na > nb) {
        r.tk = kT_DELTA;
        r.r0 = nb;
        r.r1 = na;
      }
      if (!std_domain) {  // the write checksum is create(meta type, nullptr, 0), offset = size, len 0 (:328-332)
        if (tb == H3C_TYPE_NONE || na == 0) {
          r.sk = kS_ZERO;
          r.ccode = kC_NONE;
        } else if (nb > 0 && io.offset == nb) {  // isAppendWrite (:246): a combine of length 0 keeps the value
          r.sk = kS_KEEP;
          r.ccode = kC_COMBINE;
        } else {
          r.sk = kS_SET_T;
          r.ccode = kC_READ;
        }
      } else {
        r.ta = poly_type;
        if (io.kind == H3C_UPD_TRUNCATE && na < nb) {  // chunk.rs:184-197
          r.sk = kS_SET_T;
          r.ccode = kC_RECALC;
        } else if (na > nb) {  // zero pad (chunk.rs:205-218, 250-255)
          r.sk = kS_APPEND;
          r.ccode = kC_COMBINE;
          r.ncomb = 1;
        } else {
          r.sk = kS_KEEP;
        }
      }
    } else {  // REMOVE
      if (!std_domain) {
        r.sk = kS_ZERO;
        r.ccode = kC_NONE;
        r.ta = H3C_TYPE_NONE;
      } else {
        r.sk = kS_KEEP;  // engine.rs:376
        r.ta = poly_type;
      }
    }
  }
  // A6 of a fold candidate: in the block kernel when the op is local (keeps size and stored type),
  // else before it (late); nofold: every verdict is known already
  const bool cand = !nofold && fold_candidate(io, cs, r.status);
  const bool fold = cand && r.na == r.nb && r.ta == r.tb && r.tk != kT_IDENT;
  r.pf = fold ? kPosFold : 0;
  late = cand && !fold;
  return r.tk == kT_IDENT ? 0u : blocks_of(cs.base, r.r0, r.r1);
}

// classify_op over the sorted positions, from the segmented scan of the size / type maps.
__global__ void uio_classify_kernel(const h3c_update_io *__restrict__ ios, const uint32_t *__restrict__ order,
                                    const uint32_t *__restrict__ skey, uint32_t n, const h3c_chunk_state *__restrict__ chunks,
                                    uint32_t nchunks, const SzTy *__restrict__ scan, const uint32_t *__restrict__ status,
                                    uint8_t poly_type, uint32_t std_domain, uint32_t nofold, OpPos *__restrict__ pos,
                                    uint32_t *__restrict__ nfrag, uint32_t *__restrict__ late) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) {
    if (p == n) nfrag[n] = late[n] = 0;
    return;
  }
  const uint32_t i = order[p], c = skey[p];
  const SzTy id{0, 0, 0, 0, 0};
  const h3c_chunk_state cs = c < nchunks ? chunks[c] : h3c_chunk_state{};
  OpPos r;
  bool lt;
  nfrag[p] = classify_op(ios[i], i, status[i], c, nchunks, cs, (p > 0 && skey[p - 1] == c) ? scan[p - 1] : id,
                         scan[p], poly_type, std_domain, nofold, r, lt);
  late[i] = lt ? 1u : 0u;
  pos[p] = r;
}

// The late pass's verdicts: A6 of the fold candidates that were not folded (late[i] == 1).  Their
// payload CRCs were zeroed by the prep kernel and accumulated by the late piece pass.
__global__ void uio_late_verify_kernel(const h3c_update_io *__restrict__ ios, uint32_t n,
                                       const uint32_t *__restrict__ late, const uint32_t *__restrict__ paycrc0,
                                       const PolyConsts *__restrict__ pc, uint32_t std_domain,
                                       const uint32_t *__restrict__ status, uint32_t *__restrict__ payraw,
                                       uint32_t *__restrict__ a6, uint32_t *__restrict__ misc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && late[i]) verify_op(i, ios, paycrc0, pc, std_domain, status, payraw, a6, misc, nullptr);
}

// Before a redo after a failed A6: every typed WRITE's payload is CRC'd again, fold candidates
// included (n items; chunk items keep their t0), so that the redo runs with every verdict known.
__global__ void uio_redo_pieces_kernel(const h3c_update_io *__restrict__ ios, uint32_t n, uint32_t np_items,
                                       const uint32_t *__restrict__ status, uint32_t *__restrict__ npieces,
                                       uint32_t *__restrict__ paycrc0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const h3c_update_io io = ios[i];
    npieces[i] = (status[i] == H3C_OK && io.kind == H3C_UPD_WRITE && io.length)
                     ? (io.length + kPieceBytes - 1) / kPieceBytes : 0u;
    paycrc0[i] = 0;
  } else if (i <= np_items) {  // chunk items (their t0 is known) and the scan's extra entry
    npieces[i] = 0;
  }
}


__device__ __forceinline__ uint16_t rel_clamp(int64_t a, int64_t rel) {
  const int64_t x = a - rel;
  return (uint16_t)(x < 0 ? 0 : (x > (int64_t)kBlk ? (int64_t)kBlk : x));
}

// Fragment k: the j-th 4 KiB block (absolute) of op position p's range [base + r0, base + r1).
// The fragment kernels size their grids for a host guess `cap` and read the real count F =
// fbase[n] on the device: no mid-batch round trip.  F > cap: they do nothing (the block
// kernel then finds no chains) and the host redoes them with F known.
__device__ __forceinline__ uint32_t frag_count(const uint32_t *__restrict__ d_F, uint32_t cap) {
  const uint32_t F = *d_F;
  return F <= cap ? F : 0u;
}

// Fragment j of op position p (its j-th 4 KiB block) and the fragment's chain key.
// A fold fragment carries the client's checksum as the init-0 CRC its block image must have
// (payload bytes at [w0, w1), zeros elsewhere): the block kernel compares without a multiply.
// *praw receives the raw payload CRC the op has when its check passes (its t-map needs it).
__device__ __forceinline__ FragDesc make_frag(const OpPos &r, uint32_t p, uint32_t j, uint32_t c,
                                              const h3c_chunk_state &cs, const h3c_update_io &io,
                                              const PolyConsts *__restrict__ pc, uint32_t std_domain, bool solo,
                                              uint64_t &key, uint32_t &praw) {
  const uint64_t blk = (((cs.base + r.r0) >> 12) + j) << 12;
  const int64_t rel = (int64_t)blk - (int64_t)cs.base;  // chunk offset of the block's first byte
  FragDesc d{};
  d.blk = blk;
  d.p = p;
  d.k0 = rel_clamp(0, rel);
  d.k1 = rel_clamp(cs.chunk_size, rel);
  d.mult = dxpow8_fast((int64_t)r.na - (rel + (int64_t)kBlk), pc, pc->poly);
  auto range = [&](int64_t x0, int64_t x1, uint16_t &o0, uint16_t &o1) {
    o0 = rel_clamp(x0, rel);
    o1 = rel_clamp(x1, rel);
    if (o1 <= o0) o0 = o1 = 0;
  };
  if (io.kind == H3C_UPD_WRITE) {
    const int64_t o = io.offset, e = (int64_t)io.offset + io.length;
    d.src = io.payload + (uint64_t)rel - (uint64_t)io.offset;
    range(o, e, d.w0, d.w1);
    if (r.tk == kT_DELTA) {
      range(o, e < (int64_t)r.nb ? e : (int64_t)r.nb, d.q0, d.q1);
      if (o > (int64_t)r.nb) range(r.nb, o, d.z0, d.z1);
      if (d.w1 > d.w0) d.flags |= kFragCrc | (solo ? kFragSolo : 0u);
    }
    if (d.w1 > d.w0 || d.z1 > d.z0) d.flags |= kFragWrite;
    if (r.pf & kPosFold) {  // the op's only fragment: its A6 check happens in the block kernel
      const uint32_t poly = pc->poly;
      praw = std_domain ? ~io.checksum_value : io.checksum_value;
      const uint32_t c0 = praw ^ dgf_mul_fast(0xFFFFFFFFu, dxpow8_fast(io.length, pc, poly), poly);
      d.flags |= kFragA6;
      d.op = r.op;
      d.expect = dgf_mul_fast(c0, dxpow8_fast((int64_t)kBlk - d.w1, pc, poly), poly);
      d.len = io.length;
    }
  } else if (r.na < r.nb) {  // truncate: the cut bytes leave the CRC
    range(r.na, r.nb, d.q0, d.q1);
    if (d.q1 > d.q0) d.flags |= kFragCrc | (solo ? kFragSolo : 0u);
  } else {  // grow: zero fill
    range(r.nb, r.na, d.z0, d.z1);
    if (d.z1 > d.z0) d.flags |= kFragWrite;
  }
  key = ((uint64_t)c << 36) | (blk >> 12);
  return d;
}

__global__ void uio_frag_kernel(const OpPos *__restrict__ pos, const uint32_t *__restrict__ fbase, uint32_t n,
                                uint32_t cap, const h3c_update_io *__restrict__ ios, const uint32_t *__restrict__ skey,
                                const h3c_chunk_state *__restrict__ chunks, FragDesc *__restrict__ frags,
                                uint64_t *__restrict__ fkey, const PolyConsts *__restrict__ pc,
                                uint32_t *__restrict__ hhead, uint32_t hcap, uint32_t std_domain,
                                uint32_t *__restrict__ payraw, uint32_t *__restrict__ fnext) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < hcap) hhead[k] = kNil;  // the link hash's bucket heads (uio_tlink_kernel runs next)
  if (k < cap) fnext[k] = kNil;   // chain next pointers (uio_heads_kernel)
  const uint32_t F = frag_count(fbase + n, cap);
  if (k >= F) return;
  uint32_t a = 0, b = n;  // the last p with fbase[p] <= k
  while (b - a > 1) {
    const uint32_t m = (a + b) >> 1;
    if (fbase[m] <= k) a = m; else b = m;
  }
  const uint32_t p = a;
  const OpPos r = pos[p];
  const uint32_t c = skey[p];
  uint64_t key;
  uint32_t praw = 0;
  const FragDesc d = make_frag(r, p, k - fbase[p], c, chunks[c], ios[r.op], pc, std_domain,
                               fbase[p + 1] - fbase[p] == 1,
                               key, praw);
  frags[k] = d;
  fkey[k] = key;
  if (d.flags & kFragA6) payraw[r.op] = praw;
}

// ---- chain links: each fragment's previous fragment of the same (chunk, block) ----
// Tiles of kLinkTile consecutive fragments group by key in LDS (open addressing on the
// 64-bit key, per-key lists of tile positions); a fragment's predecessor inside its tile is
// the largest earlier listed position.  Each tile's last fragment of a key is pushed (one
// atomicExch) on its hash bucket's list in HBM; a fragment with no predecessor in its tile
// takes the largest listed index of its key below its own (h3c_update.hip uses the same
// scheme for block writes).  Fragments are numbered in (chunk, sequence) order, so index
// order within a key is sequence order.
constexpr uint32_t kLinkTile = 256;
constexpr unsigned long long kNoKey = ~0ull;

__device__ __forceinline__ uint32_t key_hash(uint64_t key) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32);
}

__global__ __launch_bounds__(kLinkTile) void uio_tlink_kernel(const uint64_t *__restrict__ fkey,
                                                              const uint32_t *__restrict__ d_F, uint32_t cap,
                                                              uint32_t *hhead, uint32_t hmask,
                                                              uint32_t *__restrict__ gnext, uint32_t *__restrict__ prev) {
  __shared__ unsigned long long gkey[2 * kLinkTile];
  __shared__ uint32_t ghead[2 * kLinkTile], gnx[kLinkTile];
  const uint32_t F = frag_count(d_F, cap);
  const uint32_t t = threadIdx.x, k0 = blockIdx.x * kLinkTile, k = k0 + t;
  if (k0 >= F) return;  // (whole workgroup: before any barrier)
  for (uint32_t e = t; e < 2 * kLinkTile; e += kLinkTile) {
    gkey[e] = kNoKey;
    ghead[e] = kNil;
  }
  __syncthreads();
  const unsigned long long key = k < F ? (unsigned long long)fkey[k] : kNoKey;
  uint32_t h = kNil;
  if (key != kNoKey) {
    h = key_hash(key) & (2 * kLinkTile - 1);
    for (;;) {
      const unsigned long long old = atomicCAS(&gkey[h], kNoKey, key);
      if (old == kNoKey || old == key) break;
      h = (h + 1) & (2 * kLinkTile - 1);
    }
    gnx[t] = atomicExch(&ghead[h], t);
  }
  __syncthreads();
  uint32_t pin = kNil;
  bool last = true;
  if (h != kNil)
    for (uint32_t u = ghead[h]; u != kNil; u = gnx[u]) {
      if (u < t && (pin == kNil || u > pin)) pin = u;
      if (u > t) last = false;
    }
  if (k < F) {
    prev[k] = pin == kNil ? kNil : k0 + pin;
    if (last) gnext[k] = atomicExch(&hhead[(key_hash(key) >> 7) & hmask], k);
  }
}

__global__ void uio_resolve_kernel(const uint64_t *__restrict__ fkey, const uint32_t *__restrict__ d_F, uint32_t cap,
                                   const uint32_t *__restrict__ hhead, uint32_t hmask,
                                   const uint32_t *__restrict__ gnext, uint32_t *__restrict__ prev) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= frag_count(d_F, cap) || prev[k] != kNil) return;
  const uint64_t key = fkey[k];
  uint32_t p = kNil;
  for (uint32_t j = hhead[(key_hash(key) >> 7) & hmask]; j != kNil; j = gnext[j])
    if (j < k && fkey[j] == key && (p == kNil || j > p)) p = j;
  prev[k] = p;
}

// next pointers and chain-head flags (a fragment with no predecessor on its block starts a
// chain; the block kernel walks the fragments and starts at the flagged ones)
__global__ void uio_heads_kernel(const uint32_t *__restrict__ prev, const uint32_t *__restrict__ d_F, uint32_t cap,
                                 FragDesc *__restrict__ frags, uint32_t *__restrict__ fnext) {
  const uint32_t F = frag_count(d_F, cap);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F) return;
  const uint32_t p = prev[k];
  if (p != kNil) fnext[p] = k;
  else frags[k].flags |= kFragHead;
}

// ---- the fast branch: prep-kernel part ----
__device__ __forceinline__ uint32_t fast_bucket(unsigned long long key, uint32_t mask) { return (key_hash(key) >> 7) & mask; }

// An op the fast branch takes: a typed WRITE (A6 checked on its payload in uio_fast_kernel) whose
// bytes lie in one 4 KiB block (absolute addresses) inside the chunk's current size, not a full
// rewrite and not syncing, into a chunk stored under the batch polynomial.  It keeps the chunk's
// size and stored type, and its stored checksum follows updateChecksum's case (iv) (raw domain,
// ChunkReplica.cc:356-390) or copy_on_write (std domain, chunk.rs:89-158): s' = t'.
__device__ __forceinline__ bool fast_op(const h3c_update_io &io, const h3c_chunk_state &cs, uint32_t st,
                                        uint8_t poly_type) {
  if (st != H3C_OK || io.kind != H3C_UPD_WRITE || io.checksum_type != poly_type || !io.length ||
      (io.flags & H3C_IO_SYNCING) || cs.type != poly_type || cs.size > cs.chunk_size)
    return false;
  if ((uint64_t)io.offset + io.length > cs.size || (io.offset == 0 && io.length >= cs.size)) return false;
  const uint64_t a = cs.base + io.offset;
  return (a >> 12) == ((a + io.length - 1) >> 12);
}

// Op i's fragment record and key, and the links of the tile's ops by block (called by every
// thread of a prep workgroup; i >= n: no op).
__device__ void fast_prep_tile(const FastArgs &fa, uint32_t i, uint32_t n, const h3c_update_io &io,
                               const h3c_chunk_state &cs, uint32_t st, uint8_t poly_type, uint32_t std_domain) {
  __shared__ unsigned long long f_key[2 * kPrepTile];
  __shared__ uint32_t f_head[2 * kPrepTile], f_nx[kPrepTile];
  const uint32_t t = threadIdx.x, base = blockIdx.x * kPrepTile;
  unsigned long long key = kNoKey;
  bool q = false;
  if (i < n) {
    q = fast_op(io, cs, st, poly_type);
    if (q) {  // (the fragment record itself is made by uio_fast_link_kernel)
      key = ((unsigned long long)io.chunk << 36) | ((cs.base + io.offset) >> 12);  // make_frag's key
      fa.key[i] = key;
    }
    fa.dv[i] = 0;
  }
  if (__syncthreads_or(i < n && !q) && t == 0) atomicOr(fa.slow, 1u);
  for (uint32_t e = t; e < 2 * kPrepTile; e += kPrepTile) {
    f_key[e] = kNoKey;
    f_head[e] = kNil;
  }
  __syncthreads();
  uint32_t h = kNil;
  if (key != kNoKey) {
    h = key_hash(key) & (2 * kPrepTile - 1);
    for (;;) {
      const unsigned long long old = atomicCAS(&f_key[h], kNoKey, key);
      if (old == kNoKey || old == key) break;
      h = (h + 1) & (2 * kPrepTile - 1);
    }
    f_nx[t] = atomicExch(&f_head[h], t);
  }
  __syncthreads();
  if (h == kNil) return;
  uint32_t pin = kNil, nin = kNil, fst = t;  // the tile's previous / next / first op of this block
  for (uint32_t u = f_head[h]; u != kNil; u = f_nx[u]) {
    if (u < t && (pin == kNil || u > pin)) pin = u;
    if (u > t && (nin == kNil || u < nin)) nin = u;
    fst = min(fst, u);
  }
  uint4 lk = make_uint4(pin == kNil ? kNil : base + pin, nin == kNil ? kNil : base + nin, kNil, 0u);
  if (nin == kNil) {  // the tile's last op of the block: listed for the later tiles' ops (uio_fast_kernel)
    lk.z = base + fst;
    lk.w = atomicExch(&fa.head[fast_bucket(key, fa.hmask)], i + 1);
  }
  fa.link[i] = lk;
}

// ---- one-pass front: sizes, cases, fragment numbering, fragments and chain links ----
// uio_front_kernel does in one launch what the scan-based stage does in ~10 (size-map scan,
// classify, fragment-count scan, fragments, tile links, link resolution, chain heads).  A
// workgroup takes a ticket k and owns sorted op positions [k T, (k+1) T); tiles are chained by
// decoupled look-back over per-tile states in HBM (ticket order: a tile only waits on tiles that
// are already running, so the chain cannot deadlock whatever the dispatch order):
//   1. the size / type maps of the tile's ops, a segmented scan in LDS; the tile's last run is
//      published (aggregate), the carry into its first run read back from earlier tiles, the
//      inclusive state published;
//   2. each op's case (classify_op), its fragment count; a fold candidate that is not local gets
//      its A6 check here (one thread per op, a table-driven CRC of <= 4 KiB);
//   3. fragment numbering: the tile's count published, its base read back the same way;
//   4. the tile's fragments, grouped by (chunk, block) in LDS for the links inside the tile; each
//      group's last fragment pushed on its hash bucket's list (next pointer first, then a CAS on
//      the head, so a list read concurrently is always well formed); the tile's links flag set;
//   5. once every earlier tile has set its flag, the fragments with no predecessor in their tile
//      walk their bucket's list for the largest earlier fragment of their key.
// Waits are bounded: a tile that gives up sets bit 1 of misc[kMiscA6] -- the pass is void, the
// block kernel writes nothing and the host redoes the batch on the scan-based stage.
constexpr uint32_t kFrontTile = 1024;
constexpr uint32_t kFrontSpin = 1u << 21;
constexpr uint32_t kPending = 0xFFFFFFFEu;  // gnext[] entry pushed, its next pointer not yet stored
constexpr uint32_t kMiscVoid = 2;  // misc[kMiscA6] bit: a front tile gave up waiting
struct FrontSlot {
  uint32_t sz_flag, nf_flag, ln_flag, whole;  // 0: nothing yet, 1: aggregate, 2: inclusive (ln: 1 = published)
  uint32_t key, nf_agg, nf_incl, pad;         // the tile's last chunk key; fragment counts
  SzTy sz_agg, sz_incl;                       // the tile's last run of `key`: alone / with everything before
};
static_assert(sizeof(FrontSlot) == 48, "FrontSlot is 48 bytes");

__device__ __forceinline__ uint64_t sz_bits(const SzTy &a) {
  uint64_t b;
  __builtin_memcpy(&b, &a, 8);
  return b;
}
__device__ __forceinline__ SzTy sz_from_bits(uint64_t b) {
  SzTy a;
  __builtin_memcpy(&a, &b, 8);
  return a;
}
// spin until *f != 0; 0 after kFrontSpin polls (the caller voids the pass).  force (test hook
// H3C_HOOK_UPD_GIVEUP): give up at once, as a wait starved of its predecessor's CU would.
__device__ __forceinline__ uint32_t wait_flag(uint32_t *f, bool force = false) {
  if (force) return 0;
  uint32_t v;
  for (uint32_t spins = 0; (v = ld_agent(f)) == 0;) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > kFrontSpin) return 0;
  }
  return v;
}

// t0 per chunk: the raw CRC of no bytes, the trusted stored value, or the bytes' CRC.
// Also copies the chunk table to the output table, whose entries of chunks with ops the result
// kernel replaces (the same chunks on a redone pass, so the copy is made once).
__device__ __forceinline__ void t0_chunk(uint32_t c, const h3c_chunk_state *__restrict__ chunks, uint8_t poly_type,
                                         uint32_t exact, uint32_t std_domain, const uint32_t *__restrict__ crc0,
                                         const PolyConsts *__restrict__ pc, uint32_t *__restrict__ t0v,
                                         h3c_chunk_state *__restrict__ chunks_out) {
  const h3c_chunk_state cs = chunks[c];
  chunks_out[c] = cs;
  uint32_t t0;
  if (cs.size == 0 || cs.size > cs.chunk_size) {
    t0 = 0xFFFFFFFFu;
  } else if (needs_init(cs, poly_type, exact)) {
    t0 = crc0[c] ^ dgf_mul_fast(0xFFFFFFFFu, dxpow8_fast(cs.size, pc, pc->poly), pc->poly);
  } else {
    t0 = std_domain ? ~cs.value : cs.value;
  }
  t0v[c] = t0;
}

// SzTy <-> two dwords (v; cst | tset << 8 | t << 16 | segment-head flag << 24) for shuffles
__device__ __forceinline__ uint32_t sz_pack(const SzTy &a, uint32_t head) {
  return (uint32_t)a.cst | ((uint32_t)a.tset << 8) | ((uint32_t)a.t << 16) | (head << 24);
}
__device__ __forceinline__ SzTy sz_unpack(uint32_t v, uint32_t w) {
  return SzTy{v, (uint8_t)(w & 1u), (uint8_t)((w >> 8) & 1u), (uint8_t)((w >> 16) & 255u), 0};
}
// (head, map) pairs of a segmented scan: a, then b
__device__ __forceinline__ void seg_combine(uint32_t av, uint32_t aw, uint32_t &bv, uint32_t &bw) {
  if (bw >> 24) return;  // b starts a segment
  const SzTy r = SzTyOp()(sz_unpack(av, aw), sz_unpack(bv, bw));
  bv = r.v;
  bw = sz_pack(r, aw >> 24);
}

// The raw CRC of a payload of at most a few KiB by one thread: 16-byte granules (edges masked)
// into four dword streams stepped by x^(8*16) (PolyConsts::tab1), folded with x^-32 (red[0]); the
// zero pad past the end removed with x^-(8 pad); the ~0 start's share added (init ~0, no final
// XOR).  For the rare fold candidates that are not local (appends, first writes); tables read
// from HBM through the caches.
__device__ uint32_t thread_raw_crc(uint64_t S, uint32_t len, const PolyConsts *__restrict__ pc, uint32_t poly) {
  const uint64_t E = S + len;
  auto tstep = [&](uint32_t x) {
    return pc->tab1[0][x & 255u] ^ pc->tab1[1][(x >> 8) & 255u] ^ pc->tab1[2][(x >> 16) & 255u] ^ pc->tab1[3][x >> 24];
  };
  auto tred = [&](uint32_t x) {
    return pc->red[0][0][x & 255u] ^ pc->red[0][1][(x >> 8) & 255u] ^ pc->red[0][2][(x >> 16) & 255u] ^
           pc->red[0][3][x >> 24];
  };
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (uint64_t a = S & ~uint64_t(15); a < E; a += 16) {
    const uint4 v = load_masked(a, S, E);
    s0 = tstep(s0 ^ v.x);
    s1 = tstep(s1 ^ v.y);
    s2 = tstep(s2 ^ v.z);
    s3 = tstep(s3 ^ v.w);
  }
  uint32_t v = tred(s3) ^ s2;
  v = tred(v) ^ s1;
  v = tred(v) ^ s0;
  const uint32_t pad = (uint32_t)(((E + 15) & ~uint64_t(15)) - E);
  if (pad) v = dgf_mul(v, pc->fixz[pad], poly);
  return v ^ dgf_mul_fast(0xFFFFFFFFu, dxpow8_fast(len, pc, poly), poly);
}

__global__ __launch_bounds__(kFrontTile) void uio_front_kernel(
    const h3c_update_io *__restrict__ ios, const uint32_t *__restrict__ order, const uint32_t *__restrict__ skey,
    uint32_t n, const h3c_chunk_state *__restrict__ chunks, uint32_t nchunks, const uint32_t *__restrict__ status,
    uint8_t poly_type, uint32_t std_domain, const PolyConsts *__restrict__ pc, OpPos *__restrict__ pos,
    uint32_t *__restrict__ nfrag, uint32_t *__restrict__ fbase, uint32_t *__restrict__ late,
    uint32_t *__restrict__ payraw, uint32_t *__restrict__ a6, uint32_t *misc, FragDesc *frags, uint64_t *fkey,
    uint32_t cap, uint32_t *hhead, uint32_t hmask, uint32_t *gnext, uint32_t *prev, uint32_t *fnext, FrontSlot *slots,
    const uint32_t *__restrict__ paycrc0, uint32_t exact, uint32_t *__restrict__ t0v,
    h3c_chunk_state *__restrict__ chunks_out, const uint32_t *sstate, uint32_t force_giveup) {
  constexpr uint32_t T = kFrontTile, NW = T / 64;
  __shared__ uint32_t s_key[T], s_v[T], s_w[T];         // keys; the inclusive maps (v, packed)
  __shared__ uint32_t s_fex[T + 1];                     // exclusive fragment counts of the tile
  __shared__ uint32_t s_op[T], s_nb[T], s_na[T], s_r0[T], s_r1[T], s_kind[T];
  __shared__ uint32_t s_wv[NW], s_ww[NW], s_wn[NW];
  __shared__ unsigned long long s_gkey[2 * T];          // link grouping of a fragment sub-tile
  __shared__ uint32_t s_ghead[2 * T], s_gnx[T];
  __shared__ uint32_t s_tile, s_cv, s_cw, s_cnf, s_void;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) {
    s_tile = atomicAdd(&misc[kMiscTicket], 1u);
    s_void = 0;
  }
  __syncthreads();
  const uint32_t k = s_tile;
  const uint32_t p0 = k * T;
  if (p0 >= n) return;  // (whole workgroup)
  const uint32_t cnt = min(T, n - p0), tlast = cnt - 1;
  const uint32_t poly = pc->poly;
#define FRONT_MARK(i) ((void)0)
  const bool valid = t < cnt;
  const uint32_t p = p0 + t;
  const uint32_t c = valid ? skey[p] : 0xFFFFFFFFu;
  const uint32_t i = valid ? order[p] : 0u;
  h3c_update_io io{};
  uint32_t st = H3C_ERR_INVALID_ARG;
  if (valid) {
    io = ios[i];
    st = status[i];
  }
  if (sstate) {
    // the serial path: the A6 verdicts of the ops the piece pass read (the fold candidates' come
    // later), t0 per chunk (and the output table's copy)
    if (valid) verify_op(i, ios, paycrc0, pc, std_domain, status, payraw, a6, misc, chunks);
    for (uint32_t cc = k * T + t; cc < nchunks; cc += gridDim.x * T)
      t0_chunk(cc, chunks, poly_type, exact, std_domain, paycrc0 + n, pc, t0v, chunks_out);
  }
  const SzTy id{0, 0, 0, 0, 0};
  const SzTy e = valid ? sz_elem_of(io, st, poly_type, std_domain) : id;
  s_key[t] = c;
  __syncthreads();
  const uint32_t c0 = s_key[0];

  // 1. segmented inclusive scan of the maps over the tile (a head where the key changes)
  uint32_t xv = e.v, xw = sz_pack(e, (t == 0 || c != s_key[t - 1]) ? 1u : 0u);
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t yv = (uint32_t)__shfl_up((int)xv, o, 64), yw = (uint32_t)__shfl_up((int)xw, o, 64);
    if (lane >= o) seg_combine(yv, yw, xv, xw);
  }
  if (lane == 63) {
    s_wv[wave] = xv;
    s_ww[wave] = xw;
  }
  __syncthreads();
  {  // the earlier waves' totals combined in order, then into this lane

    uint32_t pv = 0, pw = 0;  // identity, no head
    for (uint32_t w = 0; w < wave; ++w) {
      uint32_t bv = s_wv[w], bw = s_ww[w];
      seg_combine(pv, pw, bv, bw);
      pv = bv;
      pw = bw;
    }
    if (wave) seg_combine(pv, pw, xv, xw);
  }
  // the tile's last run, published as its aggregate
  if (t == tlast) {
    FrontSlot &sl = slots[k];
    st_agent(&sl.key, c);
    st_agent(&sl.whole, c == c0 ? 1u : 0u);
    st_agent(reinterpret_cast<uint64_t *>(&sl.sz_agg), sz_bits(sz_unpack(xv, xw)));
    pub_flag(&sl.sz_flag, 1u);
  }
  // the carry into the tile's first run: the maps of the positions before it with key c0
  if (wave == 0) {
    SzTy carry = id;
    bool done = k == 0;
    for (int64_t j0 = (int64_t)k - 1; !done; j0 -= 64) {
      const int64_t j = j0 - (int64_t)lane;
      uint32_t fl = 3, key = 0xFFFFFFFFu, whole = 0, v = 0, w = 0;
      if (j >= 0) {
        FrontSlot &sl = slots[j];
        fl = wait_flag(&sl.sz_flag, force_giveup && k == 1);
        key = ld_agent(&sl.key);
        whole = ld_agent(&sl.whole);
        const SzTy a = sz_from_bits(ld_agent(reinterpret_cast<uint64_t *>(fl == 2 ? &sl.sz_incl : &sl.sz_agg)));
        v = a.v;
        w = sz_pack(a, 0);
      }
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t fl_l = (uint32_t)__builtin_amdgcn_readlane((int)fl, (int)l);
        if (fl_l == 3) {  // before tile 0
          done = true;
          break;
        }
        if (fl_l == 0) {  // gave up waiting
          if (lane == 0) s_void = 1;
          done = true;
          break;
        }
        if ((uint32_t)__builtin_amdgcn_readlane((int)key, (int)l) != c0) {
          done = true;
          break;
        }
        carry = SzTyOp()(sz_unpack((uint32_t)__builtin_amdgcn_readlane((int)v, (int)l),
                                   (uint32_t)__builtin_amdgcn_readlane((int)w, (int)l)), carry);
        if (fl_l == 2 || !__builtin_amdgcn_readlane((int)whole, (int)l)) {
          done = true;
          break;
        }
      }
    }
    if (lane == 0) {
      s_cv = carry.v;
      s_cw = sz_pack(carry, 0);
    }
  }
  __syncthreads();
  FRONT_MARK(1);
  const SzTy carry = sz_unpack(s_cv, s_cw);
  SzTy in = sz_unpack(xv, xw);
  if (c == c0) in = SzTyOp()(carry, in);
  s_v[t] = in.v;
  s_w[t] = sz_pack(in, 0);
  if (t == tlast) {
    st_agent(reinterpret_cast<uint64_t *>(&slots[k].sz_incl), sz_bits(in));
    pub_flag(&slots[k].sz_flag, 2u);
  }
  __syncthreads();

  // 2. each op's case and fragment count
  const SzTy ex = (t > 0 && s_key[t - 1] == c) ? sz_unpack(s_v[t - 1], s_w[t - 1]) : (c == c0 ? carry : id);
  OpPos r{};
  bool lt = false;
  uint32_t f = 0;
  h3c_chunk_state cs{};
  if (valid) {
    if (c < nchunks) cs = chunks[c];
    f = classify_op(io, i, st, c, nchunks, cs, ex, in, poly_type, std_domain, 0u, r, lt);
    if (lt) {  // A6 before the block kernel (a failure voids the speculative pass: the host redoes it)
      const uint32_t raw = thread_raw_crc(io.payload, io.length, pc, poly);
      payraw[i] = raw;
      const bool bad = (std_domain ? ~raw : raw) != io.checksum_value;
      a6[i] = bad ? 1u : 0u;
      if (bad) atomicOr(&misc[kMiscA6], 1u);
    }
    late[i] = 0;
  }

  // 3. fragment numbering: exclusive counts in the tile, the tile's base from the tiles before
  uint32_t fx = f;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)fx, o, 64);
    if (lane >= o) fx += y;
  }
  if (lane == 63) s_wn[wave] = fx;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
  for (uint32_t w = 0; w < NW; ++w) {
    if (w < wave) wpre += s_wn[w];
    tot += s_wn[w];
  }
  const uint32_t fex = wpre + fx - f;
  s_fex[t] = fex;
  if (t == 0) {
    s_fex[T] = tot;
    st_agent(&slots[k].nf_agg, tot);
    pub_flag(&slots[k].nf_flag, 1u);
  }
  if (wave == 0) {
    uint32_t base = 0;
    bool done = k == 0;
    for (int64_t j0 = (int64_t)k - 1; !done; j0 -= 64) {
      const int64_t j = j0 - (int64_t)lane;
      uint32_t fl = 3, v = 0;
      if (j >= 0) {
        FrontSlot &sl = slots[j];
        fl = wait_flag(&sl.nf_flag);
        v = ld_agent(fl == 2 ? &sl.nf_incl : &sl.nf_agg);
      }
      const uint64_t stop = __builtin_amdgcn_ballot_w64(fl != 1);  // inclusive, before tile 0, or gave up
      const uint32_t first = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
      uint32_t x = lane <= first && fl != 3 && fl != 0 ? v : 0u;
#pragma unroll
      for (uint32_t o = 32; o >= 1; o >>= 1) x += (uint32_t)__shfl_xor((int)x, (int)o, 64);
      base += x;
      if (stop) {
        done = true;
        if (first < 64 && (uint32_t)__builtin_amdgcn_readlane((int)fl, (int)first) == 0 && lane == 0) s_void = 1;
      }
    }
    if (lane == 0) s_cnf = base;
  }
  __syncthreads();
  FRONT_MARK(2);
  const uint32_t F0 = s_cnf, FT = s_fex[T];
  if (t == 0) {
    st_agent(&slots[k].nf_incl, F0 + tot);
    pub_flag(&slots[k].nf_flag, 2u);
  }
  if (valid) {
    pos[p] = r;
    nfrag[p] = f;
    fbase[p] = F0 + fex;
    if (p == n - 1) fbase[n] = F0 + tot;  // F: read by the block kernel and the host
  }
  s_op[t] = r.op;
  s_nb[t] = r.nb;
  s_na[t] = r.na;
  s_r0[t] = r.r0;
  s_r1[t] = r.r1;
  s_kind[t] = (uint32_t)r.tk | ((uint32_t)r.pf << 8) | ((uint32_t)r.sk << 16);
  __syncthreads();

  // 4. the tile's fragments and the links inside it, in sub-tiles of T fragments
  for (uint32_t s0 = 0; s0 < FT; s0 += T) {
    for (uint32_t q = t; q < 2 * T; q += T) {
      s_gkey[q] = kNoKey;
      s_ghead[q] = kNil;
    }
    __syncthreads();
    const uint32_t kk = s0 + t, g = F0 + kk;
    const bool fv = kk < FT && g < cap;
    unsigned long long key = kNoKey;
    uint32_t h = kNil;
    if (fv) {
      uint32_t a = 0, b = cnt;  // the last position q of the tile with s_fex[q] <= kk
      while (b - a > 1) {
        const uint32_t m = (a + b) >> 1;
        if (s_fex[m] <= kk) a = m; else b = m;
      }
      OpPos rq{};
      rq.op = s_op[a];
      rq.nb = s_nb[a];
      rq.na = s_na[a];
      rq.r0 = s_r0[a];
      rq.r1 = s_r1[a];
      rq.tk = (uint8_t)(s_kind[a] & 255u);
      rq.pf = (uint8_t)((s_kind[a] >> 8) & 255u);
      const uint32_t cq = s_key[a];
      uint64_t k64;
      uint32_t praw = 0;
      const FragDesc d = make_frag(rq, p0 + a, kk - s_fex[a], cq, chunks[cq], ios[rq.op], pc, std_domain,
                                   s_fex[a + 1] - s_fex[a] == 1, k64, praw);
      frags[g] = d;  // plain stores: only this thread writes the record (its head flag below)
      st_agent(reinterpret_cast<unsigned long long *>(&fkey[g]), (unsigned long long)k64);  // read by later tiles
      if (d.flags & kFragA6) payraw[rq.op] = praw;
      key = k64;
      h = key_hash(key) & (2 * T - 1);
      for (;;) {
        const unsigned long long old = atomicCAS(&s_gkey[h], kNoKey, key);
        if (old == kNoKey || old == key) break;
        h = (h + 1) & (2 * T - 1);
      }
      s_gnx[t] = atomicExch(&s_ghead[h], t);
    }
    __syncthreads();
    uint32_t pin = kNil;
    bool lastk = true;
    if (h != kNil)
      for (uint32_t u = s_ghead[h]; u != kNil; u = s_gnx[u]) {
        if (u < t && (pin == kNil || u > pin)) pin = u;
        if (u > t) lastk = false;
      }
    if (fv) {
      prev[g] = pin == kNil ? kNil : F0 + s0 + pin;
      // next pointers are written through: a later tile may set this tile's last ones (step 5)
      if (pin != kNil) st_agent(&fnext[F0 + s0 + pin], g);
      if (lastk) {
        // publish on the bucket: this entry's key at the coherence point first, then one exchange
        // for the old head, then the next pointer (gnext[] starts as kPending, prep kernel: a
        // reader that reaches this entry before its next pointer lands waits for it)
        uint32_t *bucket = &hhead[(key_hash(key) >> 7) & hmask];
        stores_done();
        const uint32_t old = __hip_atomic_exchange(bucket, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_agent(&gnext[g], old);
      }
    }
    __syncthreads();  // (the sub-tile's LDS groups are reused)
  }
  stores_done();  // every thread's fkey / gnext / CAS traffic is out before the flag
  __syncthreads();
  if (t == 0) pub_flag(&slots[k].ln_flag, 1u);
  FRONT_MARK(3);

  // 5. predecessors in earlier tiles, once every earlier tile has published its links
  if (wave == 0) {
    for (int64_t j0 = (int64_t)k - 1; j0 >= 0; j0 -= 64) {
      const int64_t j = j0 - (int64_t)lane;
      const uint32_t fl = j >= 0 ? wait_flag(&slots[j].ln_flag) : 1u;
      if (__builtin_amdgcn_ballot_w64(fl == 0) && lane == 0) s_void = 1;
    }
  }
  __syncthreads();
  FRONT_MARK(4);
  if (s_void) {  // the pass is void: no chain is run, the host redoes the batch
    if (t == 0) atomicOr(&misc[kMiscA6], kMiscVoid);
    return;
  }
  for (uint32_t s0 = 0; s0 < FT; s0 += T) {
    const uint32_t kk = s0 + t, g = F0 + kk;
    if (kk >= FT || g >= cap || prev[g] != kNil) continue;
    const unsigned long long key = ld_agent(reinterpret_cast<unsigned long long *>(&fkey[g]));
    uint32_t pr = kNil;
    bool gave_up = false;
    // an entry's key reached the coherence point before the exchange that made it reachable, and
    // each load here depends on the one before; a next pointer still kPending is waited for
    for (uint32_t j = ld_agent(&hhead[(key_hash(key) >> 7) & hmask]); j != kNil;) {
      if (j < g && ld_agent(reinterpret_cast<unsigned long long *>(&fkey[j])) == key && (pr == kNil || j > pr)) pr = j;
      uint32_t nx = ld_agent(&gnext[j]);
      for (uint32_t spins = 0; nx == kPending && !gave_up; nx = ld_agent(&gnext[j])) {
        __builtin_amdgcn_s_sleep(1);
        gave_up = ++spins > kFrontSpin;
      }
      if (gave_up) break;
      j = nx;
    }
    if (gave_up) {
      atomicOr(&misc[kMiscA6], kMiscVoid);  // the pass is void (the block kernel skips it)
      continue;
    }
    if (pr != kNil) {
      prev[g] = pr;
      st_agent(&fnext[pr], g);
    } else {
      frags[g].flags |= kFragHead;  // this thread wrote the record (step 4)
    }
  }
}

// ---- the block kernel ----
__device__ __forceinline__ uint4 mask16(uint32_t rel, uint32_t s, uint32_t e) {
  return make_uint4(byte_mask(rel, s, e), byte_mask(rel + 4, s, e), byte_mask(rel + 8, s, e), byte_mask(rel + 12, s, e));
}
__device__ __forceinline__ uint4 and4(uint4 a, uint4 m) { return make_uint4(a.x & m.x, a.y & m.y, a.z & m.z, a.w & m.w); }
__device__ __forceinline__ uint4 andn4(uint4 a, uint4 m) {
  return make_uint4(a.x & ~m.x, a.y & ~m.y, a.z & ~m.z, a.w & ~m.w);
}
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }
__device__ __forceinline__ uint4 or4(uint4 a, uint4 b) { return make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w); }

__device__ __forceinline__ uint32_t alb(uint32_t hi, uint32_t lo, uint32_t r) {
  return __builtin_amdgcn_alignbyte(hi, lo, r);
}
// bytes [s, s+16) of lo || hi (s in 1..15, wave-uniform)
__device__ __forceinline__ uint4 funnel16(uint4 lo, uint4 hi, uint32_t s) {
  const uint32_t r = s & 3u;
  switch (s >> 2) {
    case 0: return make_uint4(alb(lo.y, lo.x, r), alb(lo.z, lo.y, r), alb(lo.w, lo.z, r), alb(hi.x, lo.w, r));
    case 1: return make_uint4(alb(lo.z, lo.y, r), alb(lo.w, lo.z, r), alb(hi.x, lo.w, r), alb(hi.y, hi.x, r));
    case 2: return make_uint4(alb(lo.w, lo.z, r), alb(hi.x, lo.w, r), alb(hi.y, hi.x, r), alb(hi.z, hi.y, r));
    default: return make_uint4(alb(hi.x, lo.w, r), alb(hi.y, hi.x, r), alb(hi.z, hi.y, r), alb(hi.w, hi.z, r));
  }
}

__device__ __forceinline__ uint4 load_plain(uint64_t a) {
  const v4u v = *(gv4p)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// The byte mask of [s, e) over this lane's 16 bytes at block offset rel, in row `row` (1 KiB
// at 1024 row).  s, e and row are wave-uniform: a range that misses or covers the whole row is
// decided by a scalar branch, and only partial rows pay the per-byte compares.
__device__ __forceinline__ uint4 row_mask(uint32_t row, uint32_t rel, uint32_t s, uint32_t e) {
  const uint32_t r0 = 1024u * row, r1 = r0 + 1024u;
  if (e <= s || e <= r0 || s >= r1) return make_uint4(0, 0, 0, 0);
  if (s <= r0 && e >= r1) return make_uint4(~0u, ~0u, ~0u, ~0u);
  return mask16(rel, s, e);
}
__device__ __forceinline__ bool row_none(uint32_t row, uint32_t s, uint32_t e) {
  return e <= s || e <= 1024u * row || s >= 1024u * row + 1024u;
}
__device__ __forceinline__ bool row_full(uint32_t row, uint32_t s, uint32_t e) {
  return s <= 1024u * row && e >= 1024u * row + 1024u;
}

// Block bytes [rel, rel+16) of the new data (payload address src + rel), only those in
// [w0, w1); granules with no wanted byte are not dereferenced.
__device__ __forceinline__ uint4 load_new(uint64_t src, uint32_t row, uint32_t rel, uint32_t w0, uint32_t w1) {
  if (row_none(row, w0, w1)) return make_uint4(0, 0, 0, 0);
  const uint32_t s = (uint32_t)(src & 15u);
  const uint64_t a = src + rel;
  if (row_full(row, w0, w1) && s == 0) return load_row_rmw(a);
  if (rel + 16 <= w0 || rel >= w1) return make_uint4(0, 0, 0, 0);
  uint4 v;
  if (s == 0) {
    v = load_row_rmw(a);
  } else {
    const uint64_t a0 = a & ~uint64_t(15);
    const uint64_t wb = src + (rel > w0 ? rel : w0), we = src + (rel + 16 < w1 ? rel + 16 : w1);
    const uint4 lo = a0 + 16 > wb ? load_row_rmw(a0) : make_uint4(0, 0, 0, 0);
    const uint4 hi = a0 + 16 < we ? load_row_rmw(a0 + 16) : make_uint4(0, 0, 0, 0);
    v = funnel16(lo, hi, s);
  }
  return row_full(row, w0, w1) ? v : and4(v, mask16(rel, w0, w1));
}

// Waves per block-kernel workgroup (one per CU: the LDS tables take 156 KiB).  16 waves leave
// 128 registers a lane; 12 leave 168.
#ifndef H3C_UIO_BLOCK_WAVES
#define H3C_UIO_BLOCK_WAVES 16
#endif
constexpr uint32_t kBlkWaves = H3C_UIO_BLOCK_WAVES, kBlkThreads = 64 * kBlkWaves;
// Write-back store policy per kernel (1: nontemporal, 0: plain; profiles/r05s_rmw_policy_ab.txt):
#ifndef H3C_UIO_NT_STORES
#define H3C_UIO_NT_STORES 1  // uio_block_kernel (the general pipeline)
#endif
#ifndef H3C_FAST_NT_STORES
#define H3C_FAST_NT_STORES 1  // uio_fast_kernel (the chain-based fast branch)
#endif
#ifndef H3C_AF_NT_STORES
#define H3C_AF_NT_STORES 0  // uio_afused_kernel (the aligned sub-branch): plain, 265 -> 244 us
#endif
template <bool kNt = H3C_UIO_NT_STORES>
__device__ __forceinline__ void store_masked(uint64_t blk, uint32_t rel, uint4 v, uint32_t k0, uint32_t k1) {
  if (rel >= k0 && rel + 16 <= k1) {
    v4u w = {v.x, v.y, v.z, v.w};
    if (kNt)
      __builtin_nontemporal_store(w, (v4u __attribute__((address_space(1))) *)(blk + rel));
    else
      *(v4u __attribute__((address_space(1))) *)(blk + rel) = w;
  } else if (rel + 16 > k0 && rel < k1) {  // a word shared with a neighbouring chunk: its own bytes only
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint8_t *p = reinterpret_cast<uint8_t *>(blk + rel);
    for (uint32_t b = 0; b < 16; ++b)
      if (rel + b >= k0 && rel + b < k1) p[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
  }
}

// The block rows this lane holds (4 x 16 B at 1024 r + 16 lane) and, for a fragment with new
// bytes, the matching payload rows.
struct BlockRows {
  uint4 img[4], nw[4];
};

__device__ __forceinline__ void load_task_rows(uint64_t blk, uint32_t k0, uint32_t k1, uint64_t src, uint32_t w0,
                                               uint32_t w1, uint32_t lane, BlockRows &b) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t rel = 1024u * r + 16u * lane;
    b.img[r] = (rel + 16 > k0 && rel < k1) ? load_plain(blk + rel) : make_uint4(0, 0, 0, 0);
    b.nw[r] = load_new(src, r, rel, w0, w1);
  }
}

// The fold check's per-fragment inputs (kFragA6) and outputs.
struct FoldIo {
  uint32_t op, expect, len;
  uint32_t std_domain;
  const PolyConsts *pc;
  uint32_t *payraw, *a6;
};

// Where apply_fragment's results go (lane 0 calls them): the general pipeline's E accumulators
// and A6 verdicts (GenSink), or the fast branch's per-op granules (FastSink, uio_fast_kernel).
struct GenSink {
  uint32_t *eacc, *a6;
  uint32_t poly;
  __device__ void fail(uint32_t op) const { a6[op] = 1u; }
  __device__ void crc(uint32_t p, uint32_t v, uint32_t mult, uint32_t flags) const {
    if (flags & kFragSolo) {
      *reinterpret_cast<uint2 *>(eacc + 2 * p) = make_uint2(v, mult);
    } else {
      const uint32_t cv = dgf_mul_fast(v, mult, poly);
      if (cv) atomicXor(&eacc[2 * p], cv);
    }
  }
};

// One fragment on the block rows: its delta CRC (new ^ old) moved to its op's end goes to
// eacc[p]; then its zero fill and new bytes are applied.  Returns the rows it wrote.
// kFragA6 (a fold op): the payload's own CRC is folded beside the old bytes' (crc0 is linear:
// crc0(new ^ old) = crc0(new) ^ crc0(old)), its raw value checked against the client's checksum
// (ChunkReplica.cc:193-207, engine.rs:297-308); a failed op contributes nothing and writes nothing.
template <class Sink>
__device__ __forceinline__ uint32_t apply_fragment(uint4 (&img)[4], const uint4 (&nw)[4], uint32_t flags, uint32_t w,
                                                   uint32_t q, uint32_t z, uint32_t mult, uint32_t p, uint32_t lane,
                                                   const char *lb, const LaneLut &L, const uint32_t *red,
                                                   const FoldIo &fx, const Sink &sink) {
  const uint32_t w0 = w & 0xFFFFu, w1 = w >> 16, q0 = q & 0xFFFFu, q1 = q >> 16, z0 = z & 0xFFFFu, z1 = z >> 16;
  if (flags & kFragA6) {
    Streams sn{0, 0, 0, 0};  // the new bytes alone (one stream set at a time: the registers are full)
#pragma unroll
    for (int r = 0; r < 4; ++r) consume(sn, nw[r], lb, L);
    // the payload's init-0 CRC in its block image against the client's, precomputed (make_frag)
    const bool bad = __builtin_amdgcn_readfirstlane(wave_fold_tab(sn, lane, red)) != fx.expect;
    if (bad) {
      if (lane == 0) sink.fail(fx.op);
      return 0u;
    }
  }
  if (flags & kFragCrc) {
    Streams st{0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t rel = 1024u * r + 16u * lane;
      const uint4 old = row_full(r, q0, q1) ? img[r] : and4(img[r], row_mask(r, rel, q0, q1));
      consume(st, xor4(nw[r], old), lb, L);
    }
    const uint32_t v = wave_fold_tab(st, lane, red);
    if (lane == 0) sink.crc(p, v, mult, flags);
  }
  uint32_t dirty = 0;
  if (flags & kFragWrite) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t rel = 1024u * r + 16u * lane;
      if (row_full(r, w0, w1)) {
        img[r] = nw[r];
      } else {
        if (!row_none(r, z0, z1)) img[r] = andn4(img[r], row_mask(r, rel, z0, z1));
        if (!row_none(r, w0, w1)) img[r] = or4(andn4(img[r], row_mask(r, rel, w0, w1)), nw[r]);
      }
      if (!row_none(r, w0, w1) || !row_none(r, z0, z1)) dirty |= 1u << r;
    }
  }
  return dirty;
}

// One wave per chain (a block's fragments in sequence order): the block is loaded once, each
// fragment's delta CRC goes to its op's E, the new bytes are applied in order, and the rows
// that changed are stored once.  Waves take contiguous fragment ranges; per group of 64 lane
// k loads fragment g0 + k's record (one vector load round trip instead of a chain of
// dependent scalar loads per chain) and the wave walks the group's chain heads with readlane,
// keeping the next head's block and payload rows in flight while the current chain is folded
// and stored.  Chains longer than one fragment (blocks written more than once in the batch)
// continue with uniform loads.
__device__ __forceinline__ void uio_block_body(const FragDesc *__restrict__ frags, const uint32_t *__restrict__ fnext,
                                               const uint32_t *__restrict__ d_F,
                                               uint32_t cap, const PolyConsts *__restrict__ pc,
                                               uint32_t *__restrict__ eacc, const uint32_t *__restrict__ misc,
                                               uint32_t *lds, uint32_t std_domain, uint32_t *__restrict__ payraw,
                                               uint32_t *__restrict__ a6, uint32_t *misc_w) {
  auto fill_lds = [&]() {  // the stride and fold tables (156 KiB), then a barrier
    fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, threadIdx.x, kBlkThreads);
    if (threadIdx.x == 0) lds[kLdsWords + kRedWords] = 0;  // the waves' range counter (H3C_UIO_GRAB)
    __syncthreads();
  };
  constexpr bool kEarlyRows = true;  // first rows before the fill
  if (!kEarlyRows) fill_lds();
  const uint32_t F = misc[kMiscA6] ? 0u : frag_count(d_F, cap);  // a failed A6: this pass writes nothing
  const uint32_t *red = lds + kLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kBlkWaves + wave;
  const uint64_t nw = (uint64_t)gridDim.x * kBlkWaves;
  const uint32_t lo = (uint32_t)(gw * F / nw), hi = (uint32_t)((gw + 1) * F / nw);
  if (!kEarlyRows && lo >= hi) return;
  const uint32_t poly = pc->poly;
  const GenSink sink{eacc, a6, poly};
  const LaneLut L = make_lut(lane);
  // Every field comes from uniform (scalar) loads: the wave walks its fragments in order, the
  // rows of fragment g + 1 in flight while g is processed and the addresses of g + 2 loaded
  // meanwhile.  No per-lane copies of the records: 128 VGPRs hold the rows with no spill (a
  // spill's reload at the loop top waits, in vmcnt order, for the previous stores' acks).
  const uint4 *rec = reinterpret_cast<const uint4 *>(frags);  // 4 x 16 bytes per record
  auto addr_of = [&](uint32_t g, uint64_t &blk, uint64_t &src, uint32_t &w, uint32_t &k) {
    const uint4 a = rec[4 * (size_t)g], b = rec[4 * (size_t)g + 1], c = rec[4 * (size_t)g + 2];
    blk = (uint64_t)a.x | ((uint64_t)a.y << 32);
    src = (uint64_t)a.z | ((uint64_t)a.w << 32);
    w = b.z;
    k = c.y;
  };
  // fragment g's chain on the block rows in `cb` (its fields by scalar loads)
  auto process = [&](uint32_t g, uint64_t blk, uint32_t kk, BlockRows &cb) {
    const uint4 f1 = rec[4 * (size_t)g + 1], f2 = rec[4 * (size_t)g + 2];  // {p, rsv, w, q}, {z, k, mult, flags}
    const uint32_t flags = f2.w;
    if (flags & kFragHead) {
      const uint32_t k0 = kk & 0xFFFFu, k1 = kk >> 16;
      FoldIo fx{0, 0, 0, std_domain, pc, payraw, a6};
      if (flags & kFragA6) {  // a fold fragment's op / checksum / length
        const uint4 f3 = rec[4 * (size_t)g + 3];
        fx.op = f3.x;
        fx.expect = f3.y;
        fx.len = f3.z;
      }
      uint32_t dirty = apply_fragment(cb.img, cb.nw, flags, f1.z, f1.w, f2.x, f2.z, f1.x, lane, lb, L, red, fx, sink);
      for (uint32_t f = fnext[g]; f != kNil;) {  // later fragments of the same block
        const FragDesc d = frags[f];
        uint4 nw4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) nw4[r] = load_new(d.src, r, 1024u * r + 16u * lane, d.w0, d.w1);
        const FoldIo fd{d.op, d.expect, d.len, std_domain, pc, payraw, a6};
        dirty |= apply_fragment(cb.img, nw4, d.flags, (uint32_t)d.w0 | ((uint32_t)d.w1 << 16),
                                (uint32_t)d.q0 | ((uint32_t)d.q1 << 16), (uint32_t)d.z0 | ((uint32_t)d.z1 << 16),
                                d.mult, d.p, lane, lb, L, red, fd, sink);
        f = fnext[f];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (dirty & (1u << r)) store_masked(blk, 1024u * r + 16u * lane, cb.img[r], k0, k1);
    }
  };
  uint64_t c_blk, c_src, n_blk = 0, n_src = 0;
  uint32_t c_w, c_k, n_w = 0, n_k = 0;
  BlockRows cur, nxt;
  // the first fragment's rows are in flight while the workgroup fills its LDS tables (a wave with
  // no fragment still takes part in the fill's barrier)
  if (lo < hi) {
    addr_of(lo, c_blk, c_src, c_w, c_k);
    load_task_rows(c_blk, c_k & 0xFFFFu, c_k >> 16, c_src, c_w & 0xFFFFu, c_w >> 16, lane, cur);
    if (lo + 1 < hi) addr_of(lo + 1, n_blk, n_src, n_w, n_k);
  }
  if (kEarlyRows) fill_lds();
  if (lo >= hi) return;
  for (uint32_t g = lo; g < hi; ++g) {
    const uint64_t blk = c_blk;
    const uint32_t kk = c_k;
    if (g + 1 < hi) {
      // the next fragment's rows in flight while this one is processed (a fragment that is not a
      // chain head -- a later write to an already written block -- loads them in vain)
      load_task_rows(n_blk, n_k & 0xFFFFu, n_k >> 16, n_src, n_w & 0xFFFFu, n_w >> 16, lane, nxt);
      c_blk = n_blk;
      c_k = n_k;
      if (g + 2 < hi) addr_of(g + 2, n_blk, n_src, n_w, n_k);
    }
    process(g, blk, kk, cur);
    cur = nxt;
  }
}

// ts (nullable): [0] the earliest workgroup start, [1] the latest workgroup end (wall clock).
__global__ __launch_bounds__(kBlkThreads) void uio_block_kernel(const FragDesc *__restrict__ frags, const uint32_t *__restrict__ fnext,
                                                             const uint32_t *__restrict__ d_F, uint32_t cap,
                                                             const PolyConsts *__restrict__ pc,
                                                             uint32_t *__restrict__ eacc,
                                                             const uint32_t *__restrict__ misc,
                                                             unsigned long long *ts, uint32_t std_domain,
                                                             uint32_t *__restrict__ payraw, uint32_t *__restrict__ a6,
                                                             uint32_t *__restrict__ pbz, uint32_t pbz_words,
                                                             uint32_t *__restrict__ misc_w) {
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRedWords + 1];
  if (ts && threadIdx.x == 0) atomicMin(&ts[0], (unsigned long long)wall_clock64());
  if (blockIdx.x == 0) {  // uio_phaseb_kernel's tile states and ticket, fresh for every attempt
    for (uint32_t i = threadIdx.x; i < pbz_words; i += blockDim.x) pbz[i] = 0;
    if (threadIdx.x == 0) misc_w[kMiscPBVoid] = misc_w[kMiscPBDone] = 0;
  }
  uio_block_body(frags, fnext, d_F, cap, pc, eacc, misc, lds, std_domain, payraw, a6, misc_w);
  if (ts) {  // one stamp per workgroup, once all its waves are done
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&ts[1], (unsigned long long)wall_clock64());
  }
}

// A fold op whose A6 check failed in the block kernel (it changed nothing).
__device__ __forceinline__ bool fold_failed(const OpPos &r, const uint32_t *__restrict__ a6) {
  return (r.pf & kPosFold) && a6[r.op];
}

__device__ __forceinline__ Aff t_map(const OpPos &r, const uint32_t *__restrict__ eacc, const uint32_t *__restrict__ payraw,
                                     uint32_t p, const PolyConsts *__restrict__ pc, const uint32_t *__restrict__ a6) {
  if (fold_failed(r, a6)) return Aff{kOne, 0u};
  if (r.tk == kT_DELTA) {
    const uint2 w = *reinterpret_cast<const uint2 *>(eacc + 2 * p);  // (a solo fragment's shift: kFragSolo)
    return Aff{dxpow8_fast((int64_t)r.na - (int64_t)r.nb, pc, pc->poly), w.y ? dgf_mul_fast(w.x, w.y, pc->poly) : w.x};
  }
  if (r.tk == kT_FULL) return Aff{0u, payraw[r.op]};
  return Aff{kOne, 0u};
}

// t map per op position.
struct TMapFn {
  const OpPos *pos;
  const uint32_t *eacc, *payraw;
  const PolyConsts *pc;
  const uint32_t *a6;
  __device__ Aff operator()(uint32_t p) const { return t_map(pos[p], eacc, payraw, p, pc, a6); }
};

// s map per op position, from each op's t after it (the chunk's t0 through the t scan).
struct SMapFn {
  const OpPos *pos;
  const uint32_t *skey;
  uint32_t nchunks;
  const Aff *tscan;
  const uint32_t *t0v, *eacc, *payraw;
  const PolyConsts *pc;
  const uint32_t *a6;
  __device__ Aff operator()(uint32_t p) const {
    const OpPos r = pos[p];
    const uint32_t c = skey[p];
    if (c >= nchunks || fold_failed(r, a6)) return Aff{kOne, 0u};
    switch (r.sk) {
      case kS_ZERO:
        return Aff{0u, 0u};
      case kS_SET_T: {
        const Aff t = tscan[p];
        return Aff{0u, hd_gf_mul(t0v[c], t.m, pc->poly) ^ t.e};
      }
      case kS_APPEND:
        return t_map(r, eacc, payraw, p, pc, a6);
      default:
        return Aff{kOne, 0u};
    }
  }
};

template <class Fn>
__global__ void uio_elem_kernel(Fn fn, uint32_t n, Aff *__restrict__ out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) out[p] = fn(p);
}

// Per op result (IOResult.checksum, ChunkReplica.cc:174,311; ChunkEngine.cc:61-67), each chunk's
// final state (its last op), and the counters.
// Position p's result (IOResult.checksum, ChunkReplica.cc:174,311; ChunkEngine.cc:61-67) from its
// s-scan value, the chunk's final state when p is the chunk's last op, and the counter increments.
__device__ __forceinline__ void result_at(uint32_t p, OpPos r, uint32_t c, bool last_of_chunk, const Aff &x,
                                          const h3c_chunk_state *__restrict__ chunks,
                                          h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks,
                                          const uint32_t *__restrict__ t0v, uint8_t poly_type, uint32_t std_domain,
                                          uint32_t poly, h3c_update_result *__restrict__ res,
                                          const uint32_t *__restrict__ a6, uint32_t (&v)[8]) {
  if (fold_failed(r, a6)) r.status = H3C_ERR_CHECKSUM_MISMATCH;  // checked in the block kernel
  h3c_update_result o{};
  o.status = r.status;
  const bool applied = r.status == H3C_OK && r.sk != kS_IDENT;
  if (r.status == H3C_ERR_INVALID_ARG) v[6] = 1;
  if (r.status == H3C_ERR_CHECKSUM_MISMATCH) v[5] = 1;
  if (applied) {
    v[0] = r.ccode == kC_NONE;
    v[1] = r.ccode == kC_REUSE;
    v[3] = r.ccode == kC_READ;
    v[4] = r.ccode == kC_RECALC;
    v[2] = r.ccode == kC_COMBINE ? (std_domain ? r.ncomb : 1u) : 0u;
  }
  if (c < nchunks) {
    const h3c_chunk_state cs = chunks[c];
    const uint32_t t0 = t0v[c];
    uint32_t s0 = std_domain ? ~cs.value : cs.value;
    if (std_domain && cs.type != poly_type) s0 = t0;  // the engine's checksum is always crc32c of the bytes
    const uint32_t s = hd_gf_mul(s0, x.m, poly) ^ x.e;
    o.size = applied ? r.na : r.nb;
    if (r.status == H3C_ERR_CHECKSUM_MISMATCH || r.status == H3C_ERR_CHUNK_SIZE_MISMATCH) {
      // both fail after :174 set result.checksum = meta.checksum()
      o.type = std_domain ? poly_type : r.tb;
      o.value = std_domain ? 0u : s;  // engine.rs:303 returns before out_checksum is set
    } else if (applied) {
      o.type = r.ta;
      o.value = std_domain ? ~s : s;
    }
    if (last_of_chunk) {
      h3c_chunk_state fin = cs;
      fin.size = o.size;
      fin.type = r.ta;
      fin.value = std_domain ? ~s : s;
      chunks_out[c] = fin;
    }
  }
  res[r.op] = o;
}

// Per op result, each chunk's final state (its last op), and the counters.
__global__ void uio_result_kernel(const OpPos *__restrict__ pos, const uint32_t *__restrict__ skey, uint32_t n,
                                  const Aff *__restrict__ sscan, const h3c_chunk_state *__restrict__ chunks,
                                  h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks,
                                  const uint32_t *__restrict__ t0v, uint8_t poly_type, uint32_t std_domain,
                                  uint32_t poly, h3c_update_result *__restrict__ res,
                                  unsigned long long *__restrict__ ctr, const uint32_t *__restrict__ d_F,
                                  uint32_t *__restrict__ misc, const uint32_t *__restrict__ a6) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p == 0) {  // the pass's outcome, for the host's one read-back
    misc[kMiscOutF] = *d_F;
    misc[kMiscOutA6] = misc[kMiscA6];
  }
  uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (p < n) {
    const uint32_t c = skey[p];
    result_at(p, pos[p], c, p + 1 == n || skey[p + 1] != c, sscan[p], chunks, chunks_out, nchunks, t0v, poly_type,
              std_domain, poly, res, a6, v);
  }
  __shared__ unsigned int sh[8];
  ctr_add_block(sh, ctr, v);
}

// ---- one-pass phase B: the t-scan, the s-scan and the results in one launch ----
// uio_phaseb_kernel replaces the elem / scan_by_key / elem / scan_by_key / result launches: per
// ticket-ordered tile of sorted positions, a segmented scan of the t maps in LDS, the carry from
// earlier tiles by decoupled look-back (as in uio_front_kernel), the s maps from each op's t, a
// second scan and look-back, then each position's result.  Its tile states and ticket are zeroed by
// the block kernel that runs just before it, on every attempt.
struct PhaseBSlot {
  uint32_t flag[2];  // [0] t-scan, [1] s-scan: 0 nothing yet, 1 aggregate, 2 inclusive
  uint32_t whole, key;
  unsigned long long agg[2], incl[2];
};
static_assert(sizeof(PhaseBSlot) == 48, "PhaseBSlot is 48 bytes");
constexpr uint32_t kPhaseBTile = 1024;

__device__ __forceinline__ unsigned long long aff_bits(const Aff &a) {
  return (unsigned long long)a.m | ((unsigned long long)a.e << 32);
}

// Segmented inclusive scan of (head, map) over a 1024-thread tile; `sw` holds 3 x 16 words of LDS.
__device__ __forceinline__ Aff aff_tile_scan(Aff x, uint32_t head, uint32_t poly, uint32_t lane, uint32_t wave,
                                             uint32_t *sw) {
  const AffOp op{poly};
  uint32_t h = head;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const Aff y{(uint32_t)__shfl_up((int)x.m, o, 64), (uint32_t)__shfl_up((int)x.e, o, 64)};
    const uint32_t yh = (uint32_t)__shfl_up((int)h, o, 64);
    if (lane >= o && !h) {
      x = op(y, x);
      h = yh;
    }
  }
  if (lane == 63) {
    sw[wave] = x.m;
    sw[16 + wave] = x.e;
    sw[32 + wave] = h;
  }
  __syncthreads();
  if (!h) {  // no head at or before this lane in its wave: the earlier waves' run continues into it
    Aff pre{kOne, 0u};
    uint32_t ph = 0;
    for (uint32_t w = 0; w < wave; ++w) {
      const Aff y{sw[w], sw[16 + w]};
      if (sw[32 + w]) {
        pre = y;
        ph = 1;
      } else {
        pre = op(pre, y);
      }
    }
    (void)ph;
    x = op(pre, x);
  }
  __syncthreads();
  return x;
}

// The carry into the tile's first run (key c0) of scan `which`, from earlier tiles (wave 0).
__device__ Aff aff_carry(PhaseBSlot *slots, uint32_t k, uint32_t c0, int which, uint32_t poly, uint32_t lane,
                         uint32_t *gave_up, bool force = false) {
  const AffOp op{poly};
  Aff carry{kOne, 0u};
  bool done = k == 0;
  for (int64_t j0 = (int64_t)k - 1; !done; j0 -= 64) {
    const int64_t j = j0 - (int64_t)lane;
    uint32_t fl = 3, key = 0xFFFFFFFFu, whole = 0;
    unsigned long long a = 0;
    if (j >= 0) {
      PhaseBSlot &sl = slots[j];
      fl = wait_flag(&sl.flag[which], force);
      key = ld_agent(&sl.key);
      whole = ld_agent(&sl.whole);
      a = ld_agent(fl == 2 ? &sl.incl[which] : &sl.agg[which]);
    }
    for (uint32_t l = 0; l < 64; ++l) {
      const uint32_t fl_l = (uint32_t)__builtin_amdgcn_readlane((int)fl, (int)l);
      if (fl_l == 3) {
        done = true;
        break;
      }
      if (fl_l == 0) {
        if (lane == 0) *gave_up = 1;
        done = true;
        break;
      }
      if ((uint32_t)__builtin_amdgcn_readlane((int)key, (int)l) != c0) {
        done = true;
        break;
      }
      const Aff al{(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a, (int)l),
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a >> 32), (int)l)};
      carry = op(al, carry);
      if (fl_l == 2 || !__builtin_amdgcn_readlane((int)whole, (int)l)) {
        done = true;
        break;
      }
    }
  }
  return carry;
}

// s map of position p (SMapFn) given its t-scan value.
__device__ __forceinline__ Aff s_map_at(const OpPos &r, uint32_t c, uint32_t nchunks, const Aff &t,
                                        const uint32_t *__restrict__ t0v, const uint32_t *__restrict__ eacc,
                                        const uint32_t *__restrict__ payraw, uint32_t p,
                                        const PolyConsts *__restrict__ pc, const uint32_t *__restrict__ a6) {
  if (c >= nchunks || fold_failed(r, a6)) return Aff{kOne, 0u};
  switch (r.sk) {
    case kS_ZERO:
      return Aff{0u, 0u};
    case kS_SET_T:
      return Aff{0u, hd_gf_mul(t0v[c], t.m, pc->poly) ^ t.e};
    case kS_APPEND:
      return t_map(r, eacc, payraw, p, pc, a6);
    default:
      return Aff{kOne, 0u};
  }
}

__global__ __launch_bounds__(kPhaseBTile) void uio_phaseb_kernel(
    const OpPos *__restrict__ pos, const uint32_t *__restrict__ skey, uint32_t n, const uint32_t *__restrict__ eacc,
    const uint32_t *__restrict__ payraw, const PolyConsts *__restrict__ pc, const uint32_t *__restrict__ a6,
    const uint32_t *__restrict__ t0v, const h3c_chunk_state *__restrict__ chunks,
    h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks, uint8_t poly_type, uint32_t std_domain,
    h3c_update_result *__restrict__ res, unsigned long long *__restrict__ ctr, const uint32_t *__restrict__ d_F,
    uint32_t *misc, PhaseBSlot *slots, uint32_t *ticket, uint32_t *hout, uint32_t force_giveup) {
  constexpr uint32_t T = kPhaseBTile;
  __shared__ uint32_t s_key[T + 1], sw[48], s_c[2], s_tile, s_void;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t poly = pc->poly;
  const AffOp op{poly};
  if (t == 0) {
    s_tile = atomicAdd(ticket, 1u);
    s_void = 0;
  }
  __syncthreads();
  const uint32_t k = s_tile, p0 = k * T;
  if (p0 >= n) return;  // (whole workgroup)
  const uint32_t cnt = min(T, n - p0), tlast = cnt - 1;
  const bool valid = t < cnt;
#define PB_MARK(j) ((void)0)
  const uint32_t p = p0 + t;
  const uint32_t c = valid ? skey[p] : 0xFFFFFFFFu;
  OpPos r{};
  if (valid) r = pos[p];
  s_key[t] = c;
  if (t == 0) s_key[T] = p0 + T < n ? skey[p0 + T] : 0xFFFFFFFFu;  // the next tile's first key
  __syncthreads();
  const uint32_t c0 = s_key[0];
  const uint32_t head = (t == 0 || c != s_key[t - 1]) ? 1u : 0u;
  PhaseBSlot &me = slots[k];
  PB_MARK(1);
  // t-scan
  Aff tin = aff_tile_scan(valid ? t_map(r, eacc, payraw, p, pc, a6) : Aff{kOne, 0u}, head, poly, lane, wave, sw);
  if (t == tlast) {
    st_agent(&me.key, c);
    st_agent(&me.whole, c == c0 ? 1u : 0u);
    st_agent(&me.agg[0], aff_bits(tin));
    pub_flag(&me.flag[0], 1u);
  }
  if (wave == 0) {
    const Aff cy = aff_carry(slots, k, c0, 0, poly, lane, &s_void, force_giveup && k == 1);
    if (lane == 0) {
      s_c[0] = cy.m;
      s_c[1] = cy.e;
    }
  }
  __syncthreads();
  if (c == c0) tin = op(Aff{s_c[0], s_c[1]}, tin);
  if (t == tlast) {
    st_agent(&me.incl[0], aff_bits(tin));
    pub_flag(&me.flag[0], 2u);
  }
  __syncthreads();  // (s_c is reused below)
  PB_MARK(2);
  // s-scan, from each op's t
  Aff sin = aff_tile_scan(valid ? s_map_at(r, c, nchunks, tin, t0v, eacc, payraw, p, pc, a6) : Aff{kOne, 0u}, head,
                          poly, lane, wave, sw);
  if (t == tlast) {
    st_agent(&me.agg[1], aff_bits(sin));
    pub_flag(&me.flag[1], 1u);
  }
  if (wave == 0) {
    const Aff cy = aff_carry(slots, k, c0, 1, poly, lane, &s_void);
    if (lane == 0) {
      s_c[0] = cy.m;
      s_c[1] = cy.e;
    }
  }
  __syncthreads();
  if (c == c0) sin = op(Aff{s_c[0], s_c[1]}, sin);
  if (t == tlast) {
    st_agent(&me.incl[1], aff_bits(sin));
    pub_flag(&me.flag[1], 2u);
  }
  PB_MARK(3);
  // results
  if (p == 0) {  // the pass's outcome, for the host's one read-back (written through: the last tile copies it)
    st_agent(&misc[kMiscOutF], *d_F);
    st_agent(&misc[kMiscOutA6], ld_agent(&misc[kMiscA6]));
  }
  uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (valid) result_at(p, r, c, s_key[t + 1] != c, sin, chunks, chunks_out, nchunks, t0v, poly_type, std_domain, poly,
                       res, a6, v);
  __shared__ unsigned int sh[8];
  ctr_add_block(sh, ctr, v);
  if (s_void && t == 0) atomicOr(&misc[kMiscPBVoid], 1u);  // the host reruns phase B the scan-based way
  if (hout && t == 0) {
    // the last tile to finish hands the outcome words straight to the caller's pinned host buffer
    // (no device-to-host copy after the kernel); every tile's misc traffic is at the coherence
    // point before its count (write-through stores and device atomics, then the vmcnt wait)
    stores_done();
    if (atomicAdd(&misc[kMiscPBDone], 1u) + 1 == (n + T - 1) / T) {
#pragma unroll
      for (uint32_t w = kMiscOutF; w < kMiscN; ++w) hout[w - kMiscOutF] = ld_agent(&misc[w]);
    }
  }
}

// ---- the fast branch: the blocks and A6 checks in one launch, the checksums and results in another ----
// A fast-branch batch (fast_op: every op one block, no size or type change, case (iv) / copy_on_write)
// runs, after the prep kernel and uio_fast_link_kernel, in place of the sort, the piece pass, the front
// kernel, the block kernel and phase B:
//   uio_fast_kernel: a wave takes a contiguous range of ops in sequence order and runs the chains its
//     ops start (an op starts its block's chain when no earlier op of the batch writes the block): the
//     block loaded once, each op's A6 check on its payload rows, its delta CRC (new ^ old), its bytes
//     applied, the block stored once; a chain's later ops come from chain[].  Each op's delta (or its
//     failed check) goes to dv[op].  Nothing waits: the kernel ends when its slowest wave does.
//   uio_fast_sum_kernel + uio_fast_res_kernel (the tail): per 1,024-op tile, each op's delta moved to its
//     chunk's end (x^(8e), one op per lane), the per-chunk XORs in sequence order (<= 128 chunks, checked
//     by the host), every op's result t0 ^ the XOR of its chunk's deltas up to it, the final states, the
//     commit (device-table entry) and the outcome words (to the host buffer).
// (One kernel with the sums chained across workgroups by look-back measured 320-330 us against this
// form's ~300 us: its waves that finished early waited on chains run late by other waves, polling.)
// uio_fast_recover_kernel recomputes the results from dv[] when a pass reports itself void (kept for
// the test hook H3C_HOOK_UPD_GIVEUP bit 2; the two-launch tail has no wait to give up).
// the bucket walks over the tiles' last ops (uio_fast_kernel; restrict pointers, so that uniform
// walks compile to scalar loads)
__device__ __forceinline__ bool fast_listed_before(const uint4 *__restrict__ link, const unsigned long long *__restrict__ keys,
                                                   const uint32_t *__restrict__ bhead, uint32_t hmask,
                                                   unsigned long long key, uint32_t j) {
  for (uint32_t e = bhead[fast_bucket(key, hmask)]; e != 0; e = link[e - 1].w)
    if (e - 1 < j && keys[e - 1] == key) return true;
  return false;
}
// the next op of `key` after m, the last op of the block in m's tile: the first op of the block in the
// next tile that has one (that tile's last op of the block is listed, with the tile's first beside it)
__device__ __forceinline__ uint32_t fast_cross_next(const uint4 *__restrict__ link,
                                                    const unsigned long long *__restrict__ keys,
                                                    const uint32_t *__restrict__ bhead, uint32_t hmask,
                                                    unsigned long long key, uint32_t m) {
  uint32_t best = kNil;
  for (uint32_t e = bhead[fast_bucket(key, hmask)]; e != 0; e = link[e - 1].w) {
    const uint32_t j = e - 1;
    if (j > m && j < best && keys[j] == key) best = j;
  }
  return best == kNil ? kNil : link[best].z;
}
// Per op: whether it starts its block's chain (no earlier op of the block in its tile, none listed by an
// earlier tile) and the block's next op (in its tile, else the first in the next tile that has one).
// One thread per op, between the prep kernel and uio_fast_kernel: the bucket walks' dependent loads run
// here, all at once, instead of in front of uio_fast_kernel's first row loads and between a chain's ops.
// It also makes op j's fragment record (make_frag: the op's one block), whose table lookups and GF(2)
// multiplies overlap the walks' round trips.
__global__ void uio_fast_link_kernel(const uint4 *__restrict__ link, const unsigned long long *__restrict__ keys,
                                     const uint32_t *__restrict__ bhead, uint32_t hmask, uint32_t n,
                                     const uint32_t *__restrict__ slow, uint4 *__restrict__ chain,
                                     const h3c_update_io *__restrict__ ios, const h3c_chunk_state *__restrict__ chunks,
                                     uint32_t nchunks, uint8_t poly_type, uint32_t std_domain,
                                     const PolyConsts *__restrict__ pc, FragDesc *__restrict__ frag,
                                     uint32_t *__restrict__ heavy, uint32_t *heavy_n) {
  // the chunk table (<= 128 states) into LDS beside the op's own loads: its chunk state is not a
  // second round trip after the op record
  __shared__ h3c_chunk_state s_cs[kFastChunksLds];
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  h3c_update_io io{};
  uint4 lk{};
  unsigned long long key = 0;
  if (j < n) {
    io = ios[j];
    lk = link[j];
    key = keys[j];
  }
  if (threadIdx.x < nchunks && threadIdx.x < kFastChunksLds) s_cs[threadIdx.x] = chunks[threadIdx.x];
  __syncthreads();
  if (j >= n || *slow) return;  // (an abandoned batch: uio_fast_kernel returns at once)
  const h3c_chunk_state cs = s_cs[io.chunk];  // (the host sends only batches of <= 128 chunks here)
  const uint32_t lane = threadIdx.x & 63;
  {
    OpPos r{};
    r.op = j;
    r.status = H3C_OK;
    r.nb = r.na = cs.size;
    r.r0 = io.offset;
    r.r1 = io.offset + io.length;
    r.tk = kT_DELTA;
    r.sk = kS_SET_T;
    r.tb = r.ta = poly_type;
    r.pf = kPosFold;
    uint64_t k64;
    uint32_t praw;
    frag[j] = make_frag(r, j, 0, io.chunk, cs, io, pc, std_domain, false, k64, praw);
  }
  const bool start = lk.x == kNil && !fast_listed_before(link, keys, bhead, hmask, key, j);
  const uint32_t next = lk.y != kNil ? lk.y : fast_cross_next(link, keys, bhead, hmask, key, j);
  uint4 e = make_uint4(start ? 1u << 31 : 0u, next, 0u, 0u);
  if (next != kNil) {  // the next op's payload rows (its record is another thread's, being written now;
    const h3c_update_io nio = ios[next];  // its chunk is this op's)
    const uint64_t blk = (cs.base + nio.offset) & ~(uint64_t)(kBlk - 1);
    const int64_t rel = (int64_t)blk - (int64_t)cs.base;
    const uint64_t src = nio.payload + (uint64_t)rel - (uint64_t)nio.offset;
    const uint32_t w0 = rel_clamp(nio.offset, rel), w1 = rel_clamp((int64_t)nio.offset + nio.length, rel);
    e.x |= w0 | (w1 << 13);
    e.z = (uint32_t)src;
    e.w = (uint32_t)(src >> 32);
  }
  chain[j] = e;
  // the starts of chains with later ops, listed per 64-op segment (this wave's; no atomics: heavy[64 s + k],
  // heavy_n[s] the count): uio_fast_kernel deals the segments out round-robin over its workgroups, whose
  // contiguous ranges would otherwise carry the batch's early starts' later ops -- early ranges ran ~10 %
  // more ops than late ones (profiles/r04_updio_fast_wg_ends.txt)
  if (heavy) {
    const bool hv = start && next != kNil;
    const uint64_t m = __builtin_amdgcn_ballot_w64(hv);
    const uint32_t seg = j >> 6;
    if (hv) heavy[64 * seg + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1))] = j;
    if (lane == 0) heavy_n[seg] = (uint32_t)__builtin_popcountll(m);  // (lane 0 is active: j = 64 seg < n)
  }
}

struct FastSink {  // apply_fragment's results on the fast branch: dv[op] = {1, unshifted delta} or {2, 0}
  unsigned long long *dv;
  __device__ void fail(uint32_t op) const { st_agent(&dv[op], 2ull << 32); }
  __device__ void crc(uint32_t p, uint32_t v, uint32_t, uint32_t) const { st_agent(&dv[p], (1ull << 32) | v); }
};
#ifndef H3C_FAST_TRACE
#define H3C_FAST_TRACE 0  // 1: workgroups 0, 1, the middle one and the last print their step times (diagnostics)
#endif
#if H3C_FAST_TRACE == 3
// each workgroup's start and end of the last uio_fast_kernel launch (diagnostics; h3c_diag_fast_wg,
// scripts/fast_wg_trace.py)
__device__ unsigned long long g_fast_wg[2 * 1024];
__device__ uint32_t g_fast_rot;  // workgroup b takes range (b + g_fast_rot) % grid (h3c_diag_fast_rot)
#endif
#if H3C_FAST_TRACE
#define FAST_MARK(i) (ftr[i] = wall_clock64())
#else
#define FAST_MARK(i) ((void)0)
#endif
constexpr uint32_t kFastCols = 128;  // chunks a fast-branch batch may name (lane c: chunks c, c + 64)
// FastScratch words: [0] the chain-based fast branch's slow word; [64, 128) the aligned sub-branch's control
// words (kACtlWords); [128, ...) its look-back granules (kAGranRows rows of kFastCols u64) and per-ticket
// throughput records (kAGranRows x 3 words); then the fast
// branch's bucket heads (hcap words, zero between batches) and the aligned sub-branch's (hcap words,
// epoch-tagged).  A layout for another hcap starts from a zeroed scratch.
constexpr uint32_t kAGranRows = 1024;  // aligned workgroups at most
constexpr uint32_t kScratchACtl = 64, kScratchAGran = 128;
constexpr uint32_t kScratchAStat = kScratchAGran + 2 * kAGranRows * kFastCols;
constexpr uint32_t kScratchHeads = kScratchAStat + 3 * kAGranRows;
constexpr uint32_t kAEpochBatches = 240;  // aligned batches between zeroings (epochs are 8 bits)
#ifndef H3C_FAST_WG_MULT
#define H3C_FAST_WG_MULT 1  // uio_fast_kernel workgroups per CU over the launch (one resident at a time)
#endif
constexpr unsigned long long kGranApplied = 4ull << 32;  // look-back granule bit: some op of the chunk applied


// t0 of chunk c: the trusted stored value, or (H3C_UPD_EXACT) the CRC of its bytes (prep / piece pass)
__device__ __forceinline__ uint32_t fast_t0(const h3c_chunk_state &cs, uint32_t c, uint32_t exact, uint32_t std_domain,
                                            const uint32_t *__restrict__ crc0, const PolyConsts *__restrict__ pc) {
  if (exact && cs.size && cs.size <= cs.chunk_size)
    return crc0[c] ^ dgf_mul_fast(0xFFFFFFFFu, dxpow8_fast(cs.size, pc, pc->poly), pc->poly);
  return std_domain ? ~cs.value : cs.value;
}

__global__ __launch_bounds__(kBlkThreads) void uio_fast_kernel(uint32_t n, uint32_t std_domain,
                                                             const PolyConsts *__restrict__ pc,
                                                             const FragDesc *__restrict__ frag,
                                                             const uint4 *__restrict__ chain, unsigned long long *dv,
                                                             const uint32_t *__restrict__ slow, unsigned long long *ts,
                                                             const unsigned long long *__restrict__ keys,
                                                             uint32_t *heads, uint32_t hmask,
                                                             const uint32_t *__restrict__ heavy,
                                                             const uint32_t *__restrict__ heavy_n) {
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRedWords];
  const uint32_t t = threadIdx.x, lane = t & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6);
  if (*slow) return;  // not a fast-branch batch: the host runs the general pipeline
  if (ts && t == 0) atomicMin(&ts[0], (unsigned long long)wall_clock64());
#if H3C_FAST_TRACE
  uint64_t ftr[8];
  FAST_MARK(0);
#endif
  const uint64_t gw = (uint64_t)blockIdx.x * kBlkWaves + wave, nw = (uint64_t)gridDim.x * kBlkWaves;
  const uint32_t lo = (uint32_t)(gw * n / nw), hi = (uint32_t)((gw + 1) * n / nw);
  const uint32_t *red = lds + kLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const LaneLut Lt = make_lut(lane);
  const FastSink sink{dv};
  const uint4 *__restrict__ rec = reinterpret_cast<const uint4 *>(frag);  // 4 x 16 bytes per record
  // the chain starts of the group at g0 (lanes: one op each) and, among them, those whose block has
  // later ops in the batch (their chains run without the next start's rows in flight: the registers
  // hold the block, one payload and the next start's rows only when the chain is one op)
  auto starts = [&](uint32_t g0, uint64_t &cm) -> uint64_t {
    const uint32_t j = g0 + lane;
    bool hd = false, cn = false;
    if (j < hi) {
      const uint4 ch = chain[j];
      hd = (ch.x >> 31) != 0;
      cn = hd && ch.y != kNil;
    }
    cm = __builtin_amdgcn_ballot_w64(cn);
    return __builtin_amdgcn_ballot_w64(hd);
  };
  // the next chain start at or after group g0 (g0 and the masks advance): kNil when none is left
  auto next_start = [&](uint32_t &g0, uint64_t &hm, uint64_t &cm, bool &cont) -> uint32_t {
    while (!hm) {
      g0 += 64;
      if (g0 >= hi) return kNil;
      hm = starts(g0, cm);
    }
    const uint32_t b = (uint32_t)__builtin_ctzll(hm);
    cont = (cm >> b) & 1u;
    hm &= hm - 1;
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(g0 + b));
  };
  // 1 + 2: the wave's chains in order.  A one-op chain runs with the next start's rows in flight (and
  // the addresses of the one after it loaded); a longer one walks its block's later ops (their payload
  // rows into cur.nw) with nothing else in flight.  The first chain's rows load before the workgroup
  // fills its LDS tables.  One apply site for every op keeps the registers within 128.
  struct Addr {
    uint64_t blk, src;
    uint32_t w, k;
  };
  auto addr_of = [&](uint32_t g, Addr &d) {  // (scalar record loads)
    const uint4 x = rec[4 * (size_t)g], y = rec[4 * (size_t)g + 1], z = rec[4 * (size_t)g + 2];
    d.blk = (uint64_t)x.x | ((uint64_t)x.y << 32);
    d.src = (uint64_t)x.z | ((uint64_t)x.w << 32);
    d.w = y.z;
    d.k = z.y;
  };
  auto rows_at = [&](const Addr &d, BlockRows &b) {
    load_task_rows(d.blk, d.k & 0xFFFFu, d.k >> 16, d.src, d.w & 0xFFFFu, d.w >> 16, lane, b);
  };
  BlockRows cur, nxt;
  uint32_t g0 = lo, op = kNil, nh = kNil, nh2 = kNil;
  uint64_t hm = 0, cm = 0;
  bool cont = false, ncont = false, ncont2 = false;
  Addr an{}, an2{};
  // Dynamic: a chain's later ops run on the wave of its start, so static ranges leave waves with a few
  // chains more than others finishing last.  The workgroup's ops [wlo, whi) are handed out one at a
  // time by an LDS counter (a wave skips the ops that do not start a chain); each wave's first op is
  // wlo + wave, whose rows load (speculatively: ~95 % start a chain) before the table fill.
  (void)next_start, (void)g0, (void)hm, (void)cm;  // (the static form's)
  auto is_start = [&](uint32_t j, bool &cn) -> bool {
    const uint4 ch = chain[j];
    cn = ch.y != kNil;
    return (ch.x >> 31) != 0;
  };
  __shared__ uint32_t s_grab;
#if H3C_FAST_TRACE == 3
  const uint32_t rb = (blockIdx.x + g_fast_rot) % gridDim.x;  // (diagnostics: the range a workgroup takes, rotated)
#else
  const uint32_t rb = blockIdx.x;
#endif
  const uint32_t wlo = (uint32_t)((uint64_t)rb * kBlkWaves * n / nw);
  const uint32_t whi = (uint32_t)((uint64_t)(rb + 1) * kBlkWaves * n / nw);
  const uint32_t first = wlo + wave;
  if (first < whi) {
    Addr a0;
    addr_of(first, a0);
    rows_at(a0, cur);
  }
  if (t == 0) s_grab = wlo + kBlkWaves;  // (the LPT form resets it below)
  // Longest first: after the static first ops, the counter hands out the starts of chains with later ops
  // (their continuations' exposed round trips), a second counter then the one-op chains, so the
  // workgroup's last waves end on short work.  The chains with later ops come from the link kernel's list,
  // dealt round-robin (entries rb, rb + grid, ...): by range, the batch's early ranges would run most of
  // them (a block's first write starts its chain).
  __shared__ uint32_t s_grab2;
  if (t == 0) {
    s_grab2 = wlo + kBlkWaves;
    s_grab = 0;  // (the list counter)
  }
  const uint32_t nseg = heavy ? (n + 63) / 64 : 0u;
  bool one_ops = false;  // (this wave has moved on to the second counter)
  auto grab = [&](bool &cn) -> uint32_t {
    for (;;) {
      uint32_t j = 0;
      if (lane == 0) j = atomicAdd(one_ops ? &s_grab2 : &s_grab, 1u);
      j = (uint32_t)__builtin_amdgcn_readfirstlane((int)j);
      if (!one_ops) {  // the list: entry j & 63 of segment rb + (j >> 6) * grid
        const uint64_t sg = (uint64_t)rb + (uint64_t)(j >> 6) * gridDim.x;
        if (sg >= nseg) {
          one_ops = true;
          continue;
        }
        if ((j & 63u) < heavy_n[sg]) {
          cn = true;
          return heavy[64 * sg + (j & 63u)];
        }
        if (lane == 0) atomicMax(&s_grab, (j | 63u) + 1u);  // (the segment's rest is empty: skip it)
        continue;
      }
      if (j >= whi) return kNil;
      bool c;
      if (is_start(j, c) && !c) {  // (a start with later ops is on the list)
        cn = false;
        return j;
      }
    }
  };
  FAST_MARK(1);
  fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, t, kBlkThreads);
  __syncthreads();
  FAST_MARK(2);
  if (first < whi && is_start(first, cont) && !cont) {  // (LPT: those are on the list)
    op = first;
  } else {
    op = grab(cont);
    if (op != kNil) {
      Addr a0;
      addr_of(op, a0);
      rows_at(a0, cur);
    }
  }
  if (op != kNil) {
    nh = grab(ncont);
    if (nh != kNil) {
      addr_of(nh, an);
      nh2 = grab(ncont2);
      if (nh2 != kNil) addr_of(nh2, an2);
    }
  }
  uint32_t head_op = op, dirty = 0;
  while (op != kNil) {
    if (op == head_op && nh != kNil) rows_at(an, nxt);  // the next chain's rows, in flight meanwhile
    uint4 cx = make_uint4(0u, kNil, 0u, 0u);
    if (cont) cx = chain[op];  // the block's next op and its payload address: the load overlaps the apply
    {
      const uint4 f1 = rec[4 * (size_t)op + 1], f2 = rec[4 * (size_t)op + 2], f3 = rec[4 * (size_t)op + 3];
      const FoldIo fx{f3.x, f3.y, f3.z, std_domain, pc, nullptr, nullptr};
      dirty |= apply_fragment(cur.img, cur.nw, f2.w, f1.z, f1.w, f2.x, f2.z, f1.x, lane, lb, Lt, red, fx, sink);
    }
    // the op's bucket head cleared for the next batch (FastScratch; uio_fast_link_kernel, its only reader,
    // has ended)
    if (lane == 0) heads[fast_bucket(keys[op], hmask)] = 0;
    if (cont) {  // the block's next op
      const uint32_t nx = cx.y;
      if (nx != kNil) {
        const uint64_t src = (uint64_t)cx.z | ((uint64_t)cx.w << 32);
        const uint32_t w0 = cx.x & 0x1FFFu, w1 = (cx.x >> 13) & 0x1FFFu;
#pragma unroll
        for (int r = 0; r < 4; ++r) cur.nw[r] = load_new(src, r, 1024u * r + 16u * lane, w0, w1);
        op = nx;
        continue;
      }
    }
    {  // the chain is done: its block's changed rows, once
      const uint4 a = rec[4 * (size_t)head_op], c2 = rec[4 * (size_t)head_op + 2];
      const uint64_t blk = (uint64_t)a.x | ((uint64_t)a.y << 32);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (dirty & (1u << r)) store_masked<H3C_FAST_NT_STORES>(blk, 1024u * r + 16u * lane, cur.img[r], c2.y & 0xFFFFu, c2.y >> 16);
    }
    dirty = 0;
    if (nh == kNil) break;
    cur = nxt;
    op = head_op = nh;
    cont = ncont;
    nh = nh2;
    an = an2;
    ncont = ncont2;
    nh2 = kNil;
    if (nh != kNil) {  // the addresses two chains ahead
      nh2 = grab(ncont2);
      if (nh2 != kNil) addr_of(nh2, an2);
    }
  }
#if H3C_FAST_TRACE
  FAST_MARK(3);
  if (lane == 0 && ((blockIdx.x < 2 || blockIdx.x == gridDim.x / 2 || blockIdx.x + 1 == gridDim.x) && wave < 2))
    printf("fast wg %u wave %u start %llu first-rows %llu fill %llu chains %llu (ticks)\n", blockIdx.x, wave,
           (unsigned long long)ftr[0], (unsigned long long)(ftr[1] - ftr[0]), (unsigned long long)(ftr[2] - ftr[0]),
           (unsigned long long)(ftr[3] - ftr[0]));
#endif
  if (ts) {  // one stamp per workgroup, once all its waves are done
    __syncthreads();
    if (t == 0) atomicMax(&ts[1], (unsigned long long)wall_clock64());
#if H3C_FAST_TRACE == 3
    if (t == 0 && blockIdx.x < 1024) {
      g_fast_wg[2 * blockIdx.x] = ftr[0];
      g_fast_wg[2 * blockIdx.x + 1] = wall_clock64();
    }
#endif
  }
}

// The outcome words into the caller's pinned host buffer, the fast-branch word last: the host polls
// it (update_core) and reads the others once it is set.
__device__ __forceinline__ void fast_outcome_to_host(const uint32_t *misc, uint32_t *hout, uint32_t fs) {
#pragma unroll
  for (uint32_t w = kMiscOutF; w < kMiscN; ++w)
    if (w != kMiscFast) hout[w - kMiscOutF] = ld_agent(&misc[w]);
  __threadfence_system();
  __hip_atomic_store(&hout[kMiscFast - kMiscOutF], fs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kTailTile = 1024;  // ops per tile of the tail kernels

// The tail in two launches with no waiting: uio_fast_sum_kernel writes each tile's per-chunk sums (one row
// of gran per tile) and each op's XOR within its tile; uio_fast_res_kernel reads, per tile, the rows of
// the tiles before it -- complete at the launch boundary -- and writes the results; its last tile the
// final states, its last to finish the commit and the outcome words.  (Round 4's first form, one launch
// chaining the tiles by look-back, took ~27 us against ~19 us: most of it waiting on late-starting tiles.)
// They also keep the fast scratch clean for the next batch (FastScratch: the slow word and bucket heads
// are zero between batches): uio_fast_kernel clears the bucket of every op it runs; when the batch was
// not a fast one, the sum kernel clears every bucket and the results kernel's last tile the slow word.
__global__ __launch_bounds__(kTailTile) void uio_fast_sum_kernel(uint32_t n, const PolyConsts *__restrict__ pc,
                                                                const FragDesc *__restrict__ frag,
                                                                const unsigned long long *__restrict__ keys,
                                                                const unsigned long long *__restrict__ dv,
                                                                const uint32_t *__restrict__ slow,
                                                                uint32_t *__restrict__ heads, uint32_t hmask,
                                                                unsigned long long *__restrict__ gran,
                                                                uint2 *__restrict__ part, uint32_t *merr) {
  constexpr uint32_t NW = kTailTile / 64;
  __shared__ uint32_t wagg[NW * kFastCols], wapp[NW * kFastCols], lv[kTailTile];
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6, k = blockIdx.x;
  const uint32_t j = k * kTailTile + t;
  // the op's loads issued before the slow word is known (their round trips overlap)
  unsigned long long kj = 0, g = 0;
  uint32_t mult = 0;
  if (j < n) {
    kj = keys[j];
    g = dv[j];
    mult = frag[j].mult;
  }
  if (*slow) {  // not a fast-branch batch (keys may be partial): every bucket head cleared
    for (uint32_t i = k * kTailTile + t; i <= hmask; i += gridDim.x * kTailTile) heads[i] = 0;
    return;
  }
  const uint32_t poly = pc->poly;
  uint32_t c = kNil, v = 0, st = 0;
  if (j < n) {  // each op's delta moved to its chunk's end
    c = (uint32_t)(kj >> 36);
    st = (uint32_t)(g >> 32);
    if (st == 1) v = dgf_mul_fast((uint32_t)g, mult, poly);
  }
  // in the wave: each op's inclusive XOR of its chunk's deltas (lanes at or before this one with the
  // same chunk, from 8 ballots over the chunk index); the wave's per-chunk sums into LDS
  lv[t] = v;
  uint64_t same = __builtin_amdgcn_ballot_w64(c != kNil);
#pragma unroll
  for (uint32_t b = 0; b < 8; ++b) {
    const uint64_t m = __builtin_amdgcn_ballot_w64((c >> b) & 1u);
    same &= ((c >> b) & 1u) ? m : ~m;
  }
  uint32_t ip = 0;
  for (uint64_t m = same & (lane == 63 ? ~0ull : ((2ull << lane) - 1)); m; m &= m - 1)
    ip ^= lv[(t & ~63u) + (uint32_t)__builtin_ctzll(m)];
  const bool top = c != kNil && (same >> lane) <= 1;  // no higher lane with this chunk
  const uint64_t okm = __builtin_amdgcn_ballot_w64(st == 1);
  wagg[wave * kFastCols + lane] = 0;
  wagg[wave * kFastCols + 64 + lane] = 0;
  wapp[wave * kFastCols + lane] = 0;
  wapp[wave * kFastCols + 64 + lane] = 0;
  __builtin_amdgcn_wave_barrier();
  if (top) {
    wagg[wave * kFastCols + c] = ip;
    wapp[wave * kFastCols + c] = (same & okm) ? 1u : 0u;
  }
  // (an op with no delta cannot happen after a complete uio_fast_kernel: the call then fails)
  const int bad = __syncthreads_or(j < n && st != 1 && st != 2);
  if (t < kFastCols) {  // the tile's row: per chunk {some op applied, XOR of the deltas}
    uint32_t a = 0, p = 0;
    for (uint32_t w = 0; w < NW; ++w) {
      a ^= wagg[w * kFastCols + t];
      p |= wapp[w * kFastCols + t];
    }
    gran[(uint64_t)k * kFastCols + t] = (p ? kGranApplied : 0ull) | a;
  }
  if (j < n) {  // the op's XOR within the tile (earlier waves' sums of its chunk, then the wave's)
    uint32_t sv = ip;
    for (uint32_t w = 0; w < wave; ++w) sv ^= wagg[w * kFastCols + c];
    part[j] = make_uint2(sv, c | (st << 8));
  }
  if (t == 0 && bad) atomicOr(merr, 1u);
}

__global__ __launch_bounds__(kTailTile) void uio_fast_res_kernel(
    const h3c_chunk_state *__restrict__ chunks, h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks, uint32_t n,
    uint8_t poly_type, uint32_t std_domain, uint32_t exact, const uint32_t *__restrict__ crc0,
    const PolyConsts *__restrict__ pc, const unsigned long long *__restrict__ gran, const uint2 *__restrict__ part,
    uint32_t *misc, uint32_t *slow, h3c_update_result *__restrict__ res, unsigned long long *__restrict__ ctr,
    uint32_t *hout, uint32_t force_giveup, h3c_chunk_state *commit) {
  constexpr uint32_t NR = kTailTile / kFastCols;  // row groups read in parallel (thread t: column t % 128)
  __shared__ uint32_t px[NR * kFastCols], pq[NR * kFastCols], wbase[kFastCols], wsz[kFastCols];
  __shared__ uint32_t s_last;
  const uint32_t t = threadIdx.x, k = blockIdx.x, ntiles = gridDim.x;
  // the op's and the chunk table's loads issued before the slow word is known (round trips overlap)
  const uint32_t j = k * kTailTile + t;
  uint2 pj = make_uint2(0u, 0u);
  if (j < n) pj = part[j];
  h3c_chunk_state cs{};
  if (t < nchunks && t < kFastCols) cs = chunks[t];
  if (ld_agent(slow)) {  // not a fast-branch batch: nothing was done; the outcome says so
    if (t == 0 && atomicAdd(&misc[kMiscFDone], 1u) + 1 == ntiles) {  // (every tile has read the slow word)
      st_agent(slow, 0u);
      misc[kMiscFast] = kFastAbort;
      if (hout) fast_outcome_to_host(misc, hout, kFastAbort);
    }
    return;
  }
  uint32_t t0 = 0;
  if (t < nchunks && t < kFastCols) t0 = fast_t0(cs, t, exact, std_domain, crc0, pc);
  {  // the earlier tiles' rows: column t % 128, rows t / 128 + NR i, 8 loads in flight per thread
    const uint32_t col = t % kFastCols, r0 = t / kFastCols;
    uint32_t x = 0, q = 0;
    constexpr uint32_t kU = 8;
    for (uint32_t rb = r0; rb < k; rb += kU * NR) {
      unsigned long long g[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t r = rb + u * NR;
        g[u] = r < k ? gran[(uint64_t)r * kFastCols + col] : 0ull;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        x ^= (uint32_t)g[u];
        q |= (g[u] & kGranApplied) ? 1u : 0u;
      }
    }
    px[r0 * kFastCols + col] = x;
    pq[r0 * kFastCols + col] = q;
  }
  __syncthreads();
  if (t < kFastCols) {
    uint32_t e = 0, q = 0;
    for (uint32_t r = 0; r < NR; ++r) {
      e ^= px[r * kFastCols + t];
      q |= pq[r * kFastCols + t];
    }
    wbase[t] = t0 ^ e;
    wsz[t] = cs.size;
    if (k + 1 == ntiles && t < nchunks) {  // the final states: the earlier tiles, then this tile's own row
      const unsigned long long own = gran[(uint64_t)k * kFastCols + t];
      const uint32_t a = e ^ (uint32_t)own;
      const bool p = q || (own & kGranApplied);
      h3c_chunk_state f = cs;
      if (p) {  // (a chunk whose ops all failed A6 keeps its stored value)
        f.value = std_domain ? ~(t0 ^ a) : (t0 ^ a);
        f.type = poly_type;
      }
      unsigned long long fw[sizeof(h3c_chunk_state) / 8];
      __builtin_memcpy(fw, &f, sizeof f);
      unsigned long long *o = reinterpret_cast<unsigned long long *>(chunks_out + t);
#pragma unroll
      for (uint32_t w = 0; w < sizeof(h3c_chunk_state) / 8; ++w) st_agent(&o[w], fw[w]);
      if (exact && cs.size && cs.type == poly_type && t0 != (std_domain ? ~cs.value : cs.value))
        atomicAdd(&ctr[kCtrStale], 1ull);
      stores_done();
    }
  }
  __syncthreads();
  const uint32_t c = pj.y & 0xFFu, st = pj.y >> 8;
  if (j < n) {  // every op's result: t0 ^ its chunk's deltas up to it
    const uint32_t sv = wbase[c] ^ pj.x;
    h3c_update_result o{};
    o.status = st == 1 ? H3C_OK : H3C_ERR_CHECKSUM_MISMATCH;
    o.size = wsz[c];
    o.type = poly_type;  // (a failed op reports the stored type: the batch polynomial here)
    o.value = st == 1 ? (std_domain ? ~sv : sv) : (std_domain ? 0u : sv);  // engine.rs:303 / ChunkReplica.cc:174
    res[j] = o;
  }
  {
    uint32_t v8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    v8[std_domain ? kCtrRecalc : kCtrRead] = j < n && st == 1;  // updateChecksum (iv) (:389) / copy_on_write (chunk.rs:153)
    v8[kCtrMismatch] = j < n && st == 2;
    __shared__ unsigned int sh[8];
    ctr_add_block(sh, ctr, v8);
  }
  // Every wave's result and counter stores complete (each wave waits for its own) before the tile
  // counts itself done: the count is what the last tile's outcome word stands on.
  stores_done();
  __syncthreads();
  if (t == 0) {
    // test hook (H3C_HOOK_UPD_GIVEUP bit 2): tile 1 reports the pass void, as the look-back form's
    // starved tile did, so that uio_fast_recover_kernel stays covered
    if (force_giveup && k == 1) atomicOr(&misc[kMiscFVoid], 1u);
    stores_done();
    s_last = atomicAdd(&misc[kMiscFDone], 1u) + 1 == ntiles;
  }
  __syncthreads();
  if (!s_last) return;
  const uint32_t fs = ld_agent(&misc[kMiscFVoid]) ? (uint32_t)kFastVoid : (uint32_t)kFastDone;
  const bool ok = fs == kFastDone && !ld_agent(&misc[kMiscErr]);
  if (commit && ok && t < nchunks) {
    const unsigned long long *in = reinterpret_cast<const unsigned long long *>(chunks_out + t);
    unsigned long long *o = reinterpret_cast<unsigned long long *>(commit + t);
#pragma unroll
    for (uint32_t w = 0; w < sizeof(h3c_chunk_state) / 8; ++w) o[w] = ld_agent(&in[w]);
  }
  // The outcome word ends the batch for the host: update_core returns on it and the leases holding
  // misc and chunks_out go back to their pools.  So every wave of this tile has finished reading misc
  // and chunks_out, and its commit stores are complete, before thread 0 publishes it (the commit of
  // chunks 64..127 is wave 1's; __threadfence_system() orders only wave 0's own accesses).
  stores_done();
  __syncthreads();
  if (t == 0) {
    st_agent(&misc[kMiscFast], fs);
    if (hout) fast_outcome_to_host(misc, hout, fs);
  }
}


// After a void fast pass (a workgroup gave up waiting): the results, final states and counters again
// from dv[], which the pass completed, by one workgroup walking the ops in tiles of 1,024.
__global__ __launch_bounds__(1024) void uio_fast_recover_kernel(
    const h3c_chunk_state *__restrict__ chunks, h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks, uint32_t n,
    uint8_t poly_type, uint32_t std_domain, uint32_t exact, const uint32_t *__restrict__ crc0,
    const PolyConsts *__restrict__ pc, FastArgs fa, uint32_t *misc, h3c_update_result *__restrict__ res,
    unsigned long long *__restrict__ ctr) {
  __shared__ uint32_t wagg[16][kFastCols], run[kFastCols], t0s[kFastCols], szs[kFastCols];
  __shared__ unsigned int app[kFastCols], cnt_ok, cnt_bad, bad_state;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6, poly = pc->poly;
  if (t < kFastCols) {
    run[t] = 0;
    app[t] = 0;
    t0s[t] = 0;
    szs[t] = 0;
    if (t < nchunks) {
      t0s[t] = fast_t0(chunks[t], t, exact, std_domain, crc0, pc);
      szs[t] = chunks[t].size;
    }
  }
  if (t == 0) cnt_ok = cnt_bad = bad_state = 0;
  __syncthreads();
  for (uint32_t b = 0; b < n; b += 1024) {
    const uint32_t j = b + t;
    uint32_t c = kNil, v = 0, st = 0;
    if (j < n) {
      c = (uint32_t)(fa.key[j] >> 36);
      const unsigned long long g = ld_agent(&fa.dv[j]);
      st = (uint32_t)(g >> 32);
      if (st == 1) v = dgf_mul_fast((uint32_t)g, fa.frag[j].mult, poly);
      if (st == 1) atomicAdd(&cnt_ok, 1u);
      else if (st == 2) atomicAdd(&cnt_bad, 1u);
      else atomicOr(&bad_state, 1u);
      if (st == 1 && c < kFastCols) atomicOr(&app[c], 1u);
    }
    uint32_t acc0 = 0, acc1 = 0, ip = 0;
    for (uint32_t u = 0; u < 64; ++u) {
      const uint32_t cu = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)u);
      const uint32_t vu = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)u);
      if (lane >= u && c == cu) ip ^= vu;
      if (cu == lane) acc0 ^= vu;
      if (cu == lane + 64) acc1 ^= vu;
    }
    wagg[wave][lane] = acc0;
    wagg[wave][64 + lane] = acc1;
    __syncthreads();
    if (j < n && c < kFastCols) {
      uint32_t e = run[c];
      for (uint32_t w = 0; w < wave; ++w) e ^= wagg[w][c];
      const uint32_t sv = t0s[c] ^ e ^ ip;
      h3c_update_result o{};
      o.status = st == 1 ? H3C_OK : H3C_ERR_CHECKSUM_MISMATCH;
      o.size = szs[c];
      o.type = poly_type;
      o.value = st == 1 ? (std_domain ? ~sv : sv) : (std_domain ? 0u : sv);
      res[j] = o;
    }
    __syncthreads();
    if (t < kFastCols) {
      uint32_t x = 0;
      for (uint32_t w = 0; w < 16; ++w) x ^= wagg[w][t];
      run[t] ^= x;
    }
    __syncthreads();
  }
  if (t < nchunks) {
    const h3c_chunk_state cs = chunks[t];
    h3c_chunk_state f = cs;
    if (app[t]) {
      f.value = std_domain ? ~(t0s[t] ^ run[t]) : (t0s[t] ^ run[t]);
      f.type = poly_type;
    }
    chunks_out[t] = f;
  }
  __syncthreads();
  if (t == 0) {
    uint32_t stale = 0;
    for (uint32_t c = 0; c < nchunks; ++c) {
      const h3c_chunk_state cs = chunks[c];
      stale += exact && cs.size && cs.type == poly_type && t0s[c] != (std_domain ? ~cs.value : cs.value);
    }
    for (int k = 0; k < kCtrN; ++k) ctr[k] = 0;
    ctr[std_domain ? kCtrRecalc : kCtrRead] = cnt_ok;
    ctr[kCtrMismatch] = cnt_bad;
    ctr[kCtrStale] = stale;
    misc[kMiscFast] = kFastDone;
    misc[kMiscFVoid] = 0;
    if (bad_state) misc[kMiscErr] = 1u;  // an op with no published delta: cannot happen after a complete pass
  }
}

// After the piece pass: A6 per op and t0 per chunk (the chunk CRCs are items n + c), one launch
// of max(n, nchunks) threads.
__global__ void uio_verify_t0_kernel(const h3c_update_io *__restrict__ ios, uint32_t n,
                                     const h3c_chunk_state *__restrict__ chunks, uint32_t nchunks, uint8_t poly_type,
                                     uint32_t exact, uint32_t std_domain, const uint32_t *__restrict__ crc0,
                                     const PolyConsts *__restrict__ pc, const uint32_t *__restrict__ status,
                                     uint32_t *__restrict__ payraw, uint32_t *__restrict__ a6,
                                     uint32_t *__restrict__ misc, uint32_t *__restrict__ t0v,
                                     h3c_chunk_state *__restrict__ chunks_out, uint32_t skip_cand) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) verify_op(i, ios, crc0, pc, std_domain, status, payraw, a6, misc, skip_cand ? chunks : nullptr);
  if (i < nchunks) t0_chunk(i, chunks, poly_type, exact, std_domain, crc0 + n, pc, t0v, chunks_out);
}

// h3c_update_ios_dev: the final chunk states over the input table, unless the pass is redone
// (a short fragment guess or a failed A6): the redo starts from the original states.
__global__ void uio_commit_kernel(const h3c_chunk_state *__restrict__ fin, h3c_chunk_state *__restrict__ chunks,
                                  uint32_t nchunks, const uint32_t *__restrict__ out, uint32_t cap) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  // out: kMiscOutF, kMiscOutA6, ... kMiscPBVoid (a void phase B is redone before its outputs count)
  // (and the fast branch, when it ran, finished with valid results; no kernel met a corrupt table)
  if (c < nchunks && out[0] <= cap && !out[1] && !out[kMiscPBVoid - kMiscOutF] &&
      out[kMiscFast - kMiscOutF] <= kFastDone && !out[kMiscErr - kMiscOutF])
    chunks[c] = fin[c];
}

// H3C_UPD_EXACT: chunks whose stored checksum of the batch polynomial disagrees with the bytes.
__global__ void uio_stale_kernel(const h3c_chunk_state *__restrict__ chunks, uint32_t nchunks,
                                 const uint32_t *__restrict__ t0v, uint8_t poly_type, uint32_t std_domain,
                                 unsigned long long *__restrict__ ctr) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t stale = 0;
  if (c < nchunks) {
    const h3c_chunk_state cs = chunks[c];
    if (cs.size && cs.type == poly_type) stale = t0v[c] != (std_domain ? ~cs.value : cs.value);
  }
  __shared__ unsigned int sh[8];
  const uint32_t v[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, stale};
  ctr_add_block(sh, ctr, v);
}

// ---- the aligned sub-branch: BASELINE config 3's block-aligned 4 KiB WRITEs in two launches ----
// A fast-branch batch whose every op is a full, block-aligned 4 KiB typed WRITE (aligned_op: config 3
// exactly) runs as uio_aprep_kernel + uio_afused_kernel instead of the chain-based fast branch's five
// launches.  It is the block-update scheme of h3c_update.hip (upd_tlink_kernel + upd_fused_kernel) with
// UpdateIO's A6 check and results added:
//   uio_aprep_kernel, per tile of 256 ops: validation (op_status) and aligned_op, each op's key (chunk,
//     block), its previous op of the block in the tile (LDS hash), and the tile's last op of each block
//     pushed on its bucket's list.  An op that does not qualify marks the batch (kASlow); the host then
//     runs the chain-based fast branch (or the general pipeline) from the original tables.
//   uio_afused_kernel, persistent: each wave takes a contiguous range of ops in sequence order (workgroups
//     in ticket order); per op: the old bytes are the previous op's payload, or the block for the block's
//     first op (speculated "no earlier op", the bucket walk overlapped with the first rows); crc0(new) is
//     the A6 check (ChunkReplica.cc:193-207), crc0(new ^ old) the delta of updateChecksum case (iv)
//     (:356-390, the checksum moved by linearity); a block's only op writes its bytes; of several, the
//     first op (which reads the block) and the last op (whose bytes are final) meet in an exchange word,
//     and the second to arrive writes the block (the last op from its rows, or the first op from the last
//     op's payload).  Each op's delta shifted to its chunk's end is XORed into the workgroup's per-chunk
//     aggregate (LDS), published as soon as the loop ends; then per group of 64 ops the shifted deltas
//     are folded into per-chunk XORs held in the lanes; workgroups chain their per-chunk aggregates by
//     decoupled look-back; every op's result is written directly; the last workgroup to
//     finish writes the final states, the counters, the commit and the outcome word.
// Nothing is zeroed per batch: the bucket heads and granules carry the batch's epoch (kAEpoch, advanced by
// the last workgroup), the ticket and done words are reset by the last workgroup.  An A6 failure (a
// corrupted transfer), a block whose last op fails its check, or a look-back that gave up makes the pass
// void: the bytes are right or deferred (kADefer list), and uio_afix_kernel recomputes every result from
// the per-op records (dv, pv) and writes the deferred blocks.
#ifndef H3C_AF_TRACE
#define H3C_AF_TRACE 0  // 1: per-workgroup wall-clock stamps of the last launch (h3c_diag_af_trace, diagnostics)
#endif
#if H3C_AF_TRACE
// per ticket: start, tables filled, last wave's ops done, look-back done, end; each wave's ops done;
// the workgroup's blockIdx and hardware XCC id
__device__ unsigned long long g_af_wg[1024 * 5];
__device__ unsigned long long g_af_wave[1024 * 16];
__device__ uint32_t g_af_blk[1024 * 4];  // per ticket: blockIdx, XCC, range start, range end
__device__ uint32_t g_af_fin[1024 * 16];  // per wave: its ops whose block has later writes (the fin path)
__device__ unsigned long long g_af_entry[1024 * 2];  // per blockIdx: kernel entry, ticket taken
#endif
#ifndef H3C_ATILE
#define H3C_ATILE 256
#endif
constexpr uint32_t kATile = H3C_ATILE;       // uio_aprep_kernel ops per workgroup
constexpr uint32_t kAMaxOps = (1u << 24) - 2;  // bucket entries: epoch << 24 | (op index + 1)
// control words: [kAAcc, +1] one u64: tickets taken << 40 | the workgroups' range weights summed (ranges are
// cut in ticket order, each sized by its class's weight); [kAW, +8) the range weight of each workgroup class
// (blockIdx % 8, one XCD each: 16.16 fixed point, 0 = 1.0), learnt from the previous batch's per-class
// throughput (the stat records) by uio_aprep_kernel's first workgroup
// [kAHas, +8): exact mode's chunks that some op of the batch writes, one 128-bit set per epoch parity (set by
// uio_aprep_kernel; the batch's last workgroup clears the other parity's set for the next batch)
enum { kAEpoch = 0, kADone = 2, kASlow = 3, kADefer = 4, kAAcc = 8, kAW = 16, kAHas = 32, kACtlWords = 64 };
constexpr uint32_t kAClasses = 8;
constexpr uint32_t kAOne = 1u << 16;  // weight 1.0
__device__ uint32_t g_aw_seed[kAClasses];  // the device's last learnt weights (0: none yet), seeding new scratches
constexpr uint32_t kADoneVoid = 1u << 12;    // kADone: finished workgroups (low 12 bits) + void reports << 12
constexpr uint32_t kASpin = 1u << 22;        // bounded look-back spins (about a quarter second)
#ifndef H3C_AF_LOOK_WIN
#define H3C_AF_LOOK_WIN 4
#endif
constexpr uint32_t kALookWin = H3C_AF_LOOK_WIN;  // look-back rows read per column per round trip

struct AlignedArgs {
  uint32_t *ctl;                  // kACtlWords control words (the thread's FastScratch)
  uint32_t *head;                 // bucket heads, hmask + 1 of them (FastScratch; epoch-tagged, never cleared)
  uint32_t hmask;
  unsigned long long *gran;       // look-back granules, kFastCols per workgroup (FastScratch; epoch-tagged)
  unsigned long long *key;        // per op: (chunk << 36) | block address >> 12
  uint4 *link;                    // per op: {previous op of the block in the op's tile (kNil: none), the bucket
                                  //  list's next entry (the tile's last op of a block), 0, 0}
  unsigned long long *dv;         // per op: {state << 32 | crc0(new ^ old)}; state 1 applied, 2 failed A6
  uint2 *pv;                      // per op: {crc0(new), the resolved previous op of the block (kNil: none)}
  uint32_t *inp;                  // per op: its chunk's XOR of shifted deltas in the wave's range up to it
  uint2 *defer;                   // blocks whose first op deferred the write-back: {first op, last op}
  uint4 *rec;                     // per op, 2 x 16 bytes (uio_afused_kernel's phase 0 -> 1): new bytes, old bytes
                                  //  (| 1: the block's first op), the block's final bytes, the A6 expectations; in
                                  //  the addresses' top 16 bits the op's shift to its chunk's end and its chunk
  uint2 *pr;                      // per op (phase 1 -> 2): {its delta moved to its chunk's end (0: a failed
                                  //  check), chunk | passed << 31}
  uint32_t *stat;                 // per ticket (FastScratch): {epoch << 8 | class, ops, wall-clock ticks of its ops}
  uint32_t *hand;                 // per op (FastScratch; epoch-tagged): the hand-over word of a block's last op
                                  //  between it and the block's first op (kHandRead / kHandPending)
  const uint32_t *crc0;           // H3C_UPD_EXACT: each chunk's crc0 of its bytes before the batch (the piece
                                  //  pass), t0 from the bytes; null: the stored checksums are trusted
};

// An op the aligned sub-branch takes: a fast-branch op (fast_op) that writes one whole 4 KiB block at a
// block-aligned address from a 16-byte-aligned payload, both below 2^48 (the records carry 16 bits in the
// addresses' top bits; device addresses are 48-bit).
__device__ __forceinline__ bool aligned_op(const h3c_update_io &io, const h3c_chunk_state &cs, uint32_t st,
                                           uint8_t poly_type) {
  return io.length == kBlk && ((cs.base + io.offset) & (kBlk - 1)) == 0 && (io.payload & 15) == 0 &&
         (io.payload >> 48) == 0 && ((cs.base + io.offset) >> 48) == 0 && fast_op(io, cs, st, poly_type);
}
__device__ __forceinline__ bool aentry_valid(uint32_t e, uint32_t E) { return (e >> 24) == E && (e & 0xFFFFFFu) != 0; }
// crc0 of an op's 4 KiB payload as its client checksum says it is (raw register, init ~0:
// raw = crc0(data) ^ ~0 * x^(8 * 4096); the std domain's value is ~raw)
__device__ __forceinline__ uint32_t aexpect(uint32_t value, uint32_t std_domain, uint32_t k4096) {
  return (std_domain ? ~value : value) ^ k4096;
}
// A chunk's base checksum t0 (raw domain): its stored value, or in exact mode the CRC of its bytes (fast_t0)
__device__ __forceinline__ uint32_t at0(const h3c_chunk_state &cs, uint32_t c, const AlignedArgs &aa,
                                        uint32_t std_domain, const PolyConsts *__restrict__ pc) {
  return fast_t0(cs, c, aa.crc0 ? 1u : 0u, std_domain, aa.crc0, pc);
}
// exact mode: whether some op of the batch (epoch E) writes chunk c
__device__ __forceinline__ bool ahas(const AlignedArgs &aa, uint32_t E, uint32_t c) {
  return (aa.ctl[kAHas + 4 * (E & 1u) + (c >> 5)] >> (c & 31u)) & 1u;
}

// Exact mode's piece table for the aligned sub-branch: the chunks' bytes only, as items 0..C-1 of a piece pass
// with no payload items (the ops' payloads are CRC'd by uio_afused_kernel itself; a piece then finds its item
// in a table of C + 1 entries), its total, and the chunks' crc0 accumulators zeroed.  One thread.
__global__ void uio_apiece_kernel(const h3c_chunk_state *__restrict__ chunks, uint32_t nchunks, uint8_t poly_type,
                                  uint32_t *__restrict__ pbase, uint32_t *__restrict__ total, uint32_t *__restrict__ crc0) {
  if (threadIdx.x != 0) return;
  const uint32_t C = nchunks ? nchunks : 1u;
  uint32_t acc = 0;
  for (uint32_t c = 0; c < C; ++c) {
    pbase[c] = acc;
    crc0[c] = 0;
    if (c < nchunks && needs_init(chunks[c], poly_type, 1u)) acc += (chunks[c].size + kPieceBytes - 1) / kPieceBytes;
  }
  pbase[C] = acc;
  *total = acc;
}

__global__ __launch_bounds__(kATile) void uio_aprep_kernel(const h3c_update_io *__restrict__ ios, uint32_t n,
                                                           const h3c_chunk_state *__restrict__ chunks,
                                                           uint32_t nchunks, uint8_t poly_type, uint32_t std_domain,
                                                           uint32_t *__restrict__ misc, unsigned long long *__restrict__ ctr,
                                                           AlignedArgs aa) {
  __shared__ h3c_chunk_state s_cs[kFastChunksLds];
  __shared__ unsigned long long g_key[2 * kATile];
  __shared__ uint32_t g_head[2 * kATile], g_nx[kATile];
  // block 0: the range weights (first dispatched, so its chain of loads does not end the launch); the
  // ops' tiles are blocks 1..
  const uint32_t t = threadIdx.x, base = (blockIdx.x - 1u) * kATile, i = blockIdx.x ? base + t : n;
  h3c_update_io io{};
  if (i < n) io = ios[i];
  if (t < nchunks && t < kFastChunksLds) s_cs[t] = chunks[t];
  const uint32_t E = aa.ctl[kAEpoch] & 0xFFu;  // (written by the previous batch's last workgroup)
  if (blockIdx.x == 0 && t < kMiscWords) misc[t] = t == kMiscT0 || t == kMiscT0 + 1 ? 0xFFFFFFFFu : 0u;
  if (blockIdx.x == 0 && t < kCtrN) ctr[t] = 0;
  if (blockIdx.x == 0) {  // (a block of its own, no ops) the workgroup classes' range weights from the
                         // previous batch's throughput
    __shared__ unsigned long long w_ops[kAClasses], w_ticks[kAClasses];
    static_assert(kAGranRows % kATile == 0, "whole rows per thread");
    constexpr uint32_t kR = kAGranRows / kATile;
    uint32_t ra[kR], ro[kR], rt[kR];  // (every row's words loaded before any is used: one round trip)
#pragma unroll
    for (uint32_t u = 0; u < kR; ++u) {
      const uint32_t r = t + u * kATile;
      ra[u] = aa.stat[3 * r];
      ro[u] = aa.stat[3 * r + 1];
      rt[u] = aa.stat[3 * r + 2];
    }
    if (t < kAClasses) w_ops[t] = w_ticks[t] = 0;
    __syncthreads();
    const uint32_t Ep = (E + 0xFFu) & 0xFFu;  // (the previous batch's epoch)
#pragma unroll
    for (uint32_t u = 0; u < kR; ++u) {
      if ((ra[u] >> 8) != Ep || (ra[u] & 0xFFu) >= kAClasses) continue;
      atomicAdd(&w_ops[ra[u] & 0xFFu], (unsigned long long)ro[u]);
      atomicAdd(&w_ticks[ra[u] & 0xFFu], (unsigned long long)rt[u]);
    }
    __syncthreads();
    if (t == 0) {
      double rate[kAClasses], mean = 0;
      uint32_t have = 0;
      for (uint32_t r = 0; r < kAClasses; ++r) {
        rate[r] = w_ticks[r] ? (double)w_ops[r] / (double)w_ticks[r] : 0.0;
        if (rate[r] > 0) {
          mean += rate[r];
          ++have;
        }
      }
      if (have == kAClasses) {  // every class measured: w <- (w + rate / mean rate) / 2, within [0.5, 2]
        mean /= kAClasses;
        for (uint32_t r = 0; r < kAClasses; ++r) {
          const uint32_t w0 = aa.ctl[kAW + r] ? aa.ctl[kAW + r] : kAOne;
          double w = (double)w0 / kAOne + H3C_W_GAIN * (-(double)w0 / kAOne + rate[r] / mean);
          w = w < 0.5 ? 0.5 : w > 2.0 ? 2.0 : w;
          aa.ctl[kAW + r] = (uint32_t)(w * kAOne);
          __hip_atomic_store(&g_aw_seed[r], (uint32_t)(w * kAOne), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {  // a new scratch (no weights yet): the device's last learnt ones, from any thread's scratch
        bool none = true;
        for (uint32_t r = 0; r < kAClasses; ++r) none = none && aa.ctl[kAW + r] == 0;
        if (none)
          for (uint32_t r = 0; r < kAClasses; ++r)
            aa.ctl[kAW + r] = __hip_atomic_load(&g_aw_seed[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  __shared__ uint32_t s_has[4];
  for (uint32_t e = t; e < 2 * kATile; e += kATile) {
    g_key[e] = kNoKey;
    g_head[e] = kNil;
  }
  if (t < 4) s_has[t] = 0;
  __syncthreads();
  unsigned long long key = kNoKey;
  bool q = false;
  if (i < n) {
    const uint32_t c = io.chunk;
    h3c_chunk_state cs{};
    if (c < nchunks && c < kFastChunksLds) cs = s_cs[c];
    const uint32_t st = op_status(io, cs, nchunks, poly_type, std_domain);
    q = c < kFastChunksLds && aligned_op(io, cs, st, poly_type);
    if (q) key = ((unsigned long long)c << 36) | ((cs.base + io.offset) >> 12);
    if (q && aa.crc0) atomicOr(&s_has[c >> 5], 1u << (c & 31u));
    aa.key[i] = key;
  }
  if (__syncthreads_or(i < n && !q) && t == 0) st_agent(&aa.ctl[kASlow], 0x100u | E);
  uint32_t h = kNil;
  if (key != kNoKey) {
    h = key_hash(key) & (2 * kATile - 1);
    for (;;) {
      const unsigned long long old = atomicCAS(&g_key[h], kNoKey, key);
      if (old == kNoKey || old == key) break;
      h = (h + 1) & (2 * kATile - 1);
    }
    g_nx[t] = atomicExch(&g_head[h], t);
  }
  __syncthreads();
  if (aa.crc0 && t < 4 && s_has[t]) atomicOr(&aa.ctl[kAHas + 4 * (E & 1u) + t], s_has[t]);
  if (i >= n) return;
  uint32_t pin = kNil;
  bool last = true;
  if (h != kNil)
    for (uint32_t u = g_head[h]; u != kNil; u = g_nx[u]) {
      if (u < t && (pin == kNil || u > pin)) pin = u;
      if (u > t) last = false;
    }
  uint4 lk = make_uint4(pin == kNil ? kNil : base + pin, 0u, 0u, 0u);
  if (h != kNil && last) {  // (listed: .z marks it)
    lk.y = atomicExch(&aa.head[fast_bucket(key, aa.hmask)], (E << 24) | (i + 1));
    lk.z = 1;
  }
  aa.link[i] = lk;
}

// The hand-over of a block's final bytes between its first op (which reads the block) and its last op (whose
// bytes are final): each exchanges its mark into the last op's word; whichever comes second writes the block
// -- the last op from its own rows if the first op has read the block, else the first op from the last op's
// payload.  The words carry the batch's epoch (trusted in the zeroed FastScratch only).
__device__ __forceinline__ uint32_t ahand(uint32_t E, uint32_t state) { return 0x01000000u | (E << 8) | state; }
constexpr uint32_t kHandRead = 1, kHandPending = 2;
__device__ __forceinline__ unsigned long long agran(uint32_t E, uint32_t state, uint32_t v) {
  return ((unsigned long long)((E << 8) | state) << 32) | v;
}
// a granule's state in batch E (0: not published in this batch)
__device__ __forceinline__ uint32_t agran_state(unsigned long long g, uint32_t E) {
  const uint32_t hi = (uint32_t)(g >> 32);
  return (hi >> 8) == E ? (hi & 3u) : 0u;
}

__global__ __launch_bounds__(kBlkThreads) void uio_afused_kernel(
    const h3c_update_io *__restrict__ ios, uint32_t n, const h3c_chunk_state *__restrict__ chunks,
    h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks, uint8_t poly_type, uint32_t std_domain,
    const PolyConsts *__restrict__ pc, AlignedArgs aa, uint32_t *misc, h3c_update_result *__restrict__ res,
    unsigned long long *__restrict__ ctr, uint32_t *hout, h3c_chunk_state *commit, uint32_t force_void) {
  __shared__ alignas(16) uint32_t lds[kLdsWords + kRedWords];
  __shared__ h3c_chunk_state s_cs[kFastChunksLds];
  __shared__ uint32_t s_ticket, s_E, s_slow, s_last, s_void, s_prev, s_grab, s_wlo, s_whi;
  __shared__ uint32_t s_agg[kFastCols];  // the workgroup's per-chunk XOR of its ops' deltas at their chunks' ends
  __shared__ uint32_t s_stale;           // (the last workgroup, exact mode: chunks whose stored value is stale)
  __shared__ uint64_t s_t_start;
  const uint32_t t = threadIdx.x, lane = t & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t cls = blockIdx.x % kAClasses;  // (one XCD per class: workgroups are dealt round-robin)
  // the kernel's own span (bench / profiling): the first-dispatched workgroup's entry (one store, not one
  // atomic per workgroup on one address) and the last workgroup's end
  if (t == 0 && blockIdx.x == 0) *reinterpret_cast<unsigned long long *>(misc + kMiscT0) = wall_clock64();
#if H3C_AF_TRACE
  if (t == 0 && blockIdx.x < 1024) g_af_entry[2 * blockIdx.x] = wall_clock64();
#endif
  if (t == 0) {
    s_E = ld_agent(&aa.ctl[kAEpoch]) & 0xFFu;
    s_slow = ld_agent(&aa.ctl[kASlow]);
    s_void = 0;
    // the ticket and the range: workgroups take tickets in order, and ticket L's range is the next slice
    // of the batch, sized by its class's weight (a slower XCD gets fewer ops)
    uint64_t wt = 0, wmine = 0;
    for (uint32_t r = 0; r < kAClasses; ++r) {
      const uint32_t w = aa.ctl[kAW + r] ? aa.ctl[kAW + r] : kAOne;
      const uint32_t cnt = gridDim.x > r ? (gridDim.x - 1 - r) / kAClasses + 1 : 0u;
      wt += (uint64_t)cnt * w;
      if (r == cls) wmine = w;
    }
    const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long *>(aa.ctl + kAAcc),
                                             (1ull << 40) | wmine);
    const uint64_t cum = old & ((1ull << 40) - 1);
    s_ticket = (uint32_t)(old >> 40);
#if H3C_AF_TRACE
    if (blockIdx.x < 1024) g_af_entry[2 * blockIdx.x + 1] = wall_clock64();
#endif
    s_wlo = (uint32_t)(cum * n / wt);
    s_whi = s_ticket + 1 == gridDim.x ? n : (uint32_t)((cum + wmine) * n / wt);
  }
  if (t < nchunks && t < kFastChunksLds) s_cs[t] = chunks[t];
  if (t < kFastCols) s_agg[t] = 0;
  if (t == 0) s_stale = 0;
  __syncthreads();  // (the ticket; the CRC tables fill beside phase 0, below)
  const uint32_t E = s_E, L = s_ticket, nwg = gridDim.x;
#if H3C_AF_TRACE
  if (t < 16 && L < 1024) g_af_fin[16 * L + t] = 0;
  if (t == 0 && L < 1024) {
    g_af_wg[5 * L] = wall_clock64();
    g_af_blk[4 * L] = blockIdx.x;
    g_af_blk[4 * L + 2] = s_wlo;
    g_af_blk[4 * L + 3] = s_whi;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_af_blk[4 * L + 1] = xcc;
  }
#endif
  const uint32_t poly = pc->poly;
  // the end of the batch, by the last workgroup to finish (every other one has counted itself done):
  // the control words reset for the next batch, the epoch advanced, the outcome words to the host
  auto finish = [&](uint32_t outcome) {
    if (t == 0) {
      st_agent(reinterpret_cast<unsigned long long *>(aa.ctl + kAAcc), 0ull);
      st_agent(&aa.ctl[kADone], 0u);
      st_agent(&aa.ctl[kAEpoch], (E + 1) & 0xFFu);
      for (uint32_t k = 0; k < 4; ++k) st_agent(&aa.ctl[kAHas + 4 * ((E + 1) & 1u) + k], 0u);
      misc[kMiscFast] = outcome;
      stores_done();
      if (hout) fast_outcome_to_host(misc, hout, outcome);
    }
  };
  if (s_slow == (0x100u | E)) {  // not an aligned batch: nothing was done
    if (t == 0) s_last = (atomicAdd(&aa.ctl[kADone], 1u) & 0xFFFu) + 1 == nwg;
    __syncthreads();
    if (s_last) finish(kFastAbort);
    return;
  }
  const uint32_t k4096 = dgf_mul(0xFFFFFFFFu, pc->pow8[12], poly);  // ~0 * x^(8 * 4096)
  // the workgroup's ops [wlo, whi) (ticket order) and, for the prefix, each wave's contiguous share
  const uint32_t wlo = s_wlo, whi = s_whi;
  const uint32_t wn_ops = whi - wlo;
  const uint32_t lo = wlo + (uint32_t)((uint64_t)wave * wn_ops / kBlkWaves);
  const uint32_t hi = wlo + (uint32_t)((uint64_t)(wave + 1) * wn_ops / kBlkWaves);
  const uint32_t lo16 = 16u * lane;  // (32 bits: a wave-uniform base plus this offset is one saddr load)
  // ---- phase 0, one thread per op of the workgroup, beside the table fill: each op's old bytes (the
  // previous op of its block: in its tile, else the last listed one of an earlier tile; none: the block
  // itself, and the op writes the block back -- with the block's last op's bytes), its A6 expectations;
  // one 32-byte record per op for phase 1's scalar loads ----
  // the CRC tables fill beside phase 0, by the waves its first pass leaves idle (they fill before loading their
  // first op's rows: vmcnt is counted in order); by every thread after phase 0 when no wave is idle
  const uint32_t p0w = (wn_ops + 63) / 64;  // waves with ops in phase 0's first pass
  if (p0w < kBlkWaves && wave >= p0w)
    fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, t - 64 * p0w, kBlkThreads - 64 * p0w);
  // (each wave's first op is wlo + wave: its new rows and (speculated) block rows load before phase 0)
  uint4 vn[4], vo[4];
  const uint32_t j0 = wlo + wave;
  uint64_t spec_old = 0;
  if (j0 < whi) {
    const h3c_update_io io = ios[j0];  // (scalar: wave-uniform)
    spec_old = s_cs[io.chunk].base + io.offset;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vn[u] = load_row_rmw(io.payload + (uint32_t)(u * kRowBytes + lo16));
      vo[u] = load_row_old(spec_old + (uint32_t)(u * kRowBytes + lo16), true);
    }
  }
  uint4 wn[4], wo[4];  // (the next op's rows)
  for (uint32_t j = wlo + t; j < whi; j += kBlkThreads) {
    const h3c_update_io io = ios[j];
    const uint4 lk = aa.link[j];
    const h3c_chunk_state &cs = s_cs[io.chunk];  // (aprep: every op's chunk is < nchunks <= 128)
    const uint32_t exp = aexpect(io.checksum_value, std_domain, k4096);
    // the block's previous op (in this tile, else the last listed one of an earlier tile) and, for an op listed
    // as its tile's last of the block, whether a later tile lists the block too (fmax: the largest listed op)
    uint32_t prev = lk.x, fmax = j;
    const bool tile_first = prev == kNil, listed = lk.z != 0;
    uint64_t old = 0, f = 0;
    if (tile_first || listed) {
      const unsigned long long key = aa.key[j];
      for (uint32_t e = aa.head[fast_bucket(key, aa.hmask)]; aentry_valid(e, E); e = aa.link[(e & 0xFFFFFFu) - 1].y) {
        const uint32_t i = (e & 0xFFFFFFu) - 1;
        if (i >= n) break;  // (cannot happen: this batch's entries name its ops)
        if (aa.key[i] != key) continue;
        if (tile_first && i < j && (prev == kNil || i > prev)) prev = i;
        fmax = max(fmax, i);
      }
    }
    if (prev == kNil) {  // the block's first op; of several: its last op's index (the hand-over word)
      old = (cs.base + io.offset) | 1u;
      if (fmax != j) f = ((uint64_t)fmax << 2) | 1u;
    } else {
      old = ios[prev].payload;
      if (listed && fmax == j) f = (cs.base + io.offset) | 2u;  // the block's last op of several: the block
    }
    // x^(8(size - offset - 4096)): the op's delta moved to its chunk's end (phase 1 applies it)
    const uint32_t xs = dxpow8_fast((int64_t)cs.size - (int64_t)io.offset - (int64_t)kBlk, pc, poly);
    aa.rec[2 * (size_t)j] = make_uint4((uint32_t)io.payload, (uint32_t)(io.payload >> 32) | (xs & 0xFFFF0000u),
                                       (uint32_t)old, (uint32_t)(old >> 32) | (xs << 16));
    aa.rec[2 * (size_t)j + 1] = make_uint4((uint32_t)f, (uint32_t)(f >> 32) | (io.chunk << 16), exp, 0u);
    aa.pv[j].y = prev;  // (uio_afix_kernel's input; crc0(new) follows in .x)
  }
  if (p0w >= kBlkWaves) fill_tables(lds, pc->tab, &pc->red[0][0][0], kRedWords, t, kBlkThreads);
  if (t == 0) s_grab = wlo + kBlkWaves;  // (each wave's first op is wlo + wave)
  stores_done();
  __syncthreads();
  if (t == 0) s_t_start = wall_clock64();
#if H3C_AF_TRACE
  if (t == 0 && L < 1024) g_af_wg[5 * L + 1] = wall_clock64();
#endif
  const uint32_t *red = lds + kLdsWords;
  const char *lb = reinterpret_cast<const char *>(lds);
  const LaneLut Lt = make_lut(lane);
  // ---- phase 1: the workgroup's ops, taken one at a time from an LDS counter by whichever wave is free
  // (static shares left waves up to ~30 us apart): per op the A6 CRC of the new bytes and the delta CRC of
  // new ^ old, the block write-back by the block's first op, {state, delta} and crc0(new) published ----
  struct Rec {
    uint64_t pnew, pold, f;  // f: 0; (the block's last op << 2) | 1 (a first op of several); the block | 2 (a last op)
    uint32_t exp, xs, c;
    bool first;
  };
  auto rec_of = [&](uint32_t j, Rec &r) {  // (scalar loads: j is wave-uniform)
    const uint4 a = aa.rec[2 * (size_t)j], b = aa.rec[2 * (size_t)j + 1];
    r.pnew = (uint64_t)a.x | ((uint64_t)(a.y & 0xFFFFu) << 32);
    const uint64_t o = (uint64_t)a.z | ((uint64_t)(a.w & 0xFFFFu) << 32);
    r.pold = o & ~uint64_t(1);
    r.first = (o & 1u) != 0;
    r.f = (uint64_t)b.x | ((uint64_t)(b.y & 0xFFFFu) << 32);
    r.exp = b.z;
    r.xs = (a.y & 0xFFFF0000u) | (a.w >> 16);
    r.c = b.y >> 16;
  };
  auto grab = [&]() -> uint32_t {
    uint32_t j = 0;
    if (lane == 0) j = atomicAdd(&s_grab, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)j);
  };
  uint32_t wave_void = 0;
  uint32_t jc = j0 < whi ? j0 : kNil;
  Rec rc{}, rn{};
  if (jc != kNil) {
    rec_of(jc, rc);
    if (rc.pold != spec_old) {  // the first op was not its block's first: its old rows are a payload
#pragma unroll
      for (int u = 0; u < 4; ++u) vo[u] = load_row_rmw(rc.pold + (uint32_t)(u * kRowBytes + lo16));
    }
  }
  uint32_t jn = jc != kNil ? grab() : kNil;
  if (jn >= whi) jn = kNil;
  if (jn != kNil) rec_of(jn, rn);
  while (jc != kNil) {
    const bool nvalid = jn != kNil;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      wn[u] = nvalid ? load_row_rmw(rn.pnew + (uint32_t)(u * kRowBytes + lo16)) : make_uint4(0, 0, 0, 0);
      wo[u] = nvalid ? load_row_old(rn.pold + (uint32_t)(u * kRowBytes + lo16), rn.first) : make_uint4(0, 0, 0, 0);
    }
    uint32_t jnn = nvalid ? grab() : kNil;  // (the op after next: its record loads meanwhile)
    if (jnn >= whi) jnn = kNil;
    Rec rnn{};
    if (jnn != kNil) rec_of(jnn, rnn);
    const bool solo = rc.first && rc.f == 0;  // the block's only write
    if (solo) {
#pragma unroll
      for (int u = 0; u < 4; ++u) store_masked<H3C_AF_NT_STORES>(rc.pold, u * kRowBytes + lo16, vn[u], 0u, kBlk);
    }
    Streams s2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      consume(s2[0], vn[u], lb, Lt);
      consume(s2[1], xor4(vn[u], vo[u]), lb, Lt);
    }
    uint32_t fv[2];
    wave_fold_tab_n<2>(s2, lane, red, fv);
    const uint32_t P = (uint32_t)__builtin_amdgcn_readfirstlane((int)fv[0]);
    const uint32_t D = (uint32_t)__builtin_amdgcn_readfirstlane((int)fv[1]);
    const bool pass = P == rc.exp;
    if (solo && !pass) {  // the block's only write fails its check: the early store undone (old rows back)
#pragma unroll
      for (int u = 0; u < 4; ++u) store_masked<H3C_AF_NT_STORES>(rc.pold, u * kRowBytes + lo16, vo[u], 0u, kBlk);
    }
    if (rc.f & 1u) {  // the first op of several: the block is read (its rows are folded into D: the asm
                      // keeps the exchange after that), hand over to the block's last op
      asm volatile("" ::"s"(D) : "memory");
      const uint32_t fm = (uint32_t)(rc.f >> 2);
      uint32_t o = 0;
      if (lane == 0) o = atomicExch(&aa.hand[fm], ahand(E, kHandRead));
      if ((uint32_t)__builtin_amdgcn_readfirstlane((int)o) == ahand(E, kHandPending)) {
        // the last op came first (and passed its check): its bytes to the block, from its payload
#if H3C_AF_TRACE
        if (lane == 0 && L < 1024) atomicAdd(&g_af_fin[16 * L + wave], 1u);
#endif
        const uint64_t lp = ios[fm].payload;
#pragma unroll
        for (int u = 0; u < 4; ++u) vo[u] = load_row_rmw(lp + (uint32_t)(u * kRowBytes + lo16));
#pragma unroll
        for (int u = 0; u < 4; ++u) store_masked<H3C_AF_NT_STORES>(rc.pold, u * kRowBytes + lo16, vo[u], 0u, kBlk);
      }
    } else if (rc.f & 2u) {  // the last op of several: its bytes are the block's final bytes
      if (pass) {
        uint32_t o = 0;
        if (lane == 0) o = atomicExch(&aa.hand[jc], ahand(E, kHandPending));
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)o) == ahand(E, kHandRead)) {  // the block is read
          const uint64_t blk = rc.f & ~uint64_t(3);
#pragma unroll
          for (int u = 0; u < 4; ++u) store_masked<H3C_AF_NT_STORES>(blk, u * kRowBytes + lo16, vn[u], 0u, kBlk);
        }
      } else {  // it fails A6: uio_afix_kernel writes the last passing op's bytes (if any)
        if (lane == 0) {
          const uint32_t d = atomicAdd(&aa.ctl[kADefer], 1u);
          aa.defer[d] = make_uint2(jc, 0u);
        }
        wave_void = 1;
      }
    }
    // the delta moved to the chunk's end: phase 2's input, and the workgroup's per-chunk XOR (published as
    // its aggregate as soon as the loop ends)
    const uint32_t v = pass ? dgf_mul(D, rc.xs, poly) : 0u;
    if (lane == 0) {
      aa.dv[jc] = ((unsigned long long)(pass ? 1u : 2u) << 32) | D;
      aa.pv[jc].x = P;
      aa.pr[jc] = make_uint2(v, rc.c | (pass ? 0x80000000u : 0u));
      atomicXor(&s_agg[rc.c], v);
    }
    if (!pass) wave_void = 1;
    jc = jn;
    rc = rn;
    jn = jnn;
    rn = rnn;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vn[u] = wn[u];
      vo[u] = wo[u];
    }
  }
#if H3C_AF_TRACE
  if (lane == 0 && L < 1024) g_af_wave[16 * L + wave] = wall_clock64();
#endif
  if (wave_void && lane == 0) atomicOr(&s_void, 1u);
  stores_done();
  __syncthreads();  // every op of the workgroup published (the CRC tables are done with: their LDS is free)
  // the workgroup's aggregate, at once: a successor's look-back waits for nothing after this loop
  unsigned long long *row = aa.gran + (uint64_t)L * kFastCols;
  const bool two = nchunks > 64;
  if (wave == 0 && L > 0) {
    if (lane < nchunks) st_agent(&row[lane], agran(E, 1u, s_agg[lane]));
    if (two && lane + 64 < nchunks) st_agent(&row[64 + lane], agran(E, 1u, s_agg[64 + lane]));
  }
  if (t == 0 && L < kAGranRows) {  // this workgroup's throughput, for the next batch's range weights
    const uint64_t t1 = wall_clock64();
    aa.stat[3 * L] = (E << 8) | cls;
    aa.stat[3 * L + 1] = whi - wlo;
    aa.stat[3 * L + 2] = (uint32_t)(t1 - s_t_start);
  }
#if H3C_AF_TRACE
  if (t == 0 && L < 1024) g_af_wg[5 * L + 2] = wall_clock64();
#endif
  uint32_t acc0 = 0, acc1 = 0;
  uint32_t my_ip = 0, my_pass = 0, my_c = kNil;
  auto phase2 = [&]() {
    // ---- phase 2: per wave, its contiguous share of the workgroup's ops in sequence order: each op's delta
    // moved to its chunk's end, the chunk XOR right after it (lanes: one op each, in groups of 64), the
    // running per-chunk XORs (lane c: chunks c and c + 64) ----
    for (uint32_t g0 = lo; g0 < hi; g0 += 64) {
      const uint32_t cnt = min(64u, hi - g0), k = g0 + lane;
      uint32_t v = 0;
      my_c = kNil;
      my_pass = 0;
      if (lane < cnt) {  // (the workgroup's own stores, before the barrier)
        const uint2 q = aa.pr[k];
        v = q.x;
        my_c = q.y & 0x7FFFFFFFu;
        my_pass = q.y >> 31;
      }
      const uint32_t src = my_c & 63;
      const uint32_t r0 = __shfl(acc0, src, 64), r1 = __shfl(acc1, src, 64);
      my_ip = my_c < 64 ? r0 : r1;
      for (uint32_t u0 = 0; u0 < cnt; ++u0) {
        const uint32_t ct = __builtin_amdgcn_readlane(my_c, u0), vt = __builtin_amdgcn_readlane(v, u0);
        if (lane >= u0 && my_c == ct) my_ip ^= vt;
        if (ct == lane) acc0 ^= vt;
        if (ct == lane + 64) acc1 ^= vt;
      }
      if (hi - lo > 64 && lane < cnt) aa.inp[k] = my_ip;
    }
  };
  // the chunks' base checksums (trusted stored values), one per lane (chunks lane, lane + 64)
  auto t0_of = [&](uint32_t c) -> uint32_t { return c < nchunks ? at0(s_cs[c], c, aa, std_domain, pc) : 0u; };
  const uint32_t rb0 = t0_of(lane), rb1 = t0_of(64 + lane);
  // ---- chunk aggregates: waves of the workgroup (LDS), then workgroups (look-back in ticket order) ----
  uint32_t *wagg = lds;                                 // [16][128]
  uint32_t *wexcl = lds + kBlkWaves * kFastCols;        // [128]: the workgroup's exclusive prefix
  auto lookback = [&]() {  // wave 0: the look-back (the aggregate is out), the inclusive sums
    if (wave == 0) {
      const uint32_t a0 = s_agg[lane], a1 = s_agg[64 + lane];
      uint32_t x0 = 0, x1 = 0;
      if (L > 0) {
        int j0 = lane < nchunks ? (int)L - 1 : -1, j1 = two && lane + 64 < nchunks ? (int)L - 1 : -1;
        const uint32_t limit = (force_void & 1) && L == 1 ? 0u : kASpin;  // (test hook: ticket 1 gives up at once)
        for (uint32_t spins = 0; __builtin_amdgcn_ballot_w64(j0 >= 0 || j1 >= 0) != 0;) {
          bool moved = false;
          auto look = [&](int &j, uint32_t &x, uint32_t col) {
            if (j < 0) return;
            const int top = j;
            unsigned long long g[kALookWin];
  #pragma unroll
            for (int w = 0; w < (int)kALookWin; ++w)
              g[w] = top - w >= 0 ? ld_agent(&aa.gran[(uint64_t)(top - w) * kFastCols + col]) : 0ull;
  #pragma unroll
            for (int w = 0; w < (int)kALookWin; ++w) {
              const uint32_t state = agran_state(g[w], E);
              if (top - w >= 0 && j == top - w && state) {
                x ^= (uint32_t)g[w];
                j = state == 2u ? -1 : j - 1;
                moved = true;
              }
            }
          };
          look(j0, x0, lane);
          look(j1, x1, 64 + lane);
          if (__builtin_amdgcn_ballot_w64(moved) == 0 || limit == 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > limit) {  // a predecessor never published: the pass is void (uio_afix_kernel)
              if (lane == 0) s_void = 1;
              break;
            }
          }
        }
      }
      if (lane < nchunks) st_agent(&row[lane], agran(E, 2u, x0 ^ a0));
      if (two && lane + 64 < nchunks) st_agent(&row[64 + lane], agran(E, 2u, x1 ^ a1));
      wexcl[lane] = x0;
      wexcl[64 + lane] = x1;
  #if H3C_AF_TRACE
      if (lane == 0 && L < 1024) g_af_wg[5 * L + 3] = wall_clock64();
  #endif
    }
  };
  phase2();
  wagg[wave * kFastCols + lane] = acc0;
  wagg[wave * kFastCols + 64 + lane] = acc1;
  __syncthreads();
  lookback();
  __syncthreads();
  // every op's result: its chunk's checksum right after it (ChunkReplica.cc:174, :311; a failed op reports
  // the stored checksum unchanged, engine.rs:303 in the std domain)
  uint32_t e0 = wexcl[lane], e1 = wexcl[64 + lane];
  for (uint32_t w = 0; w < wave; ++w) {
    e0 ^= wagg[w * kFastCols + lane];
    e1 ^= wagg[w * kFastCols + 64 + lane];
  }
  const uint32_t be0 = rb0 ^ e0, be1 = rb1 ^ e1;
  auto result = [&](uint32_t j, uint32_t c, uint32_t ip, bool pass) {
    const uint32_t x0 = __shfl(be0, c & 63, 64), x1 = __shfl(be1, c & 63, 64);
    if (j >= hi) return;
    const uint32_t sv = (c < 64 ? x0 : x1) ^ ip;
    h3c_update_result o{};
    o.status = pass ? H3C_OK : H3C_ERR_CHECKSUM_MISMATCH;
    o.size = s_cs[c].size;
    o.type = poly_type;
    o.value = pass ? (std_domain ? ~sv : sv) : (std_domain ? 0u : sv);
    res[j] = o;
  };
  if (hi - lo <= 64) {  // one group (the common case): its chunks and XORs are still in registers
    result(lo + lane, my_c, my_ip, my_pass != 0);
  } else {
    for (uint32_t i0 = lo; i0 < hi; i0 += 64) {
      const uint32_t j = i0 + lane;
      uint32_t c = 0, ip = 0;
      bool pass = false;
      if (j < hi) {
        c = ios[j].chunk;
        ip = aa.inp[j];
        pass = (uint32_t)(aa.dv[j] >> 32) == 1u;
      }
      result(j, c, ip, pass);
    }
  }
  stores_done();
  __syncthreads();
#if H3C_AF_TRACE
  if (t == 0 && L < 1024) g_af_wg[5 * L + 4] = wall_clock64();
#endif
  if (t == 0) {
    const uint32_t w = atomicAdd(&aa.ctl[kADone], 1u + (s_void ? kADoneVoid : 0u));
    s_last = (w & 0xFFFu) + 1 == nwg;
    s_prev = (w >> 12) + (s_void ? 1u : 0u);  // void reports, this one included
  }
  __syncthreads();
  if (!s_last) return;
  // the last workgroup to finish: the totals are the last ticket's inclusive granules
  const bool vd = s_prev != 0 || force_void;
  // the counters (a pass that is not void has no failed check: every op is updateChecksum case (iv),
  // :389, or copy_on_write, chunk.rs:153; uio_afix_kernel writes them for a void pass)
  if (t < kCtrN) ctr[t] = !vd && t == (std_domain ? kCtrRecalc : kCtrRead) ? n : 0u;
  if (t == 0) *reinterpret_cast<unsigned long long *>(misc + kMiscT1) = wall_clock64();
  if (t < nchunks && !vd) {  // (exact mode: a chunk no op writes keeps its stored value, stale or not)
    const unsigned long long g = ld_agent(&aa.gran[(uint64_t)(nwg - 1) * kFastCols + t]);
    const uint32_t a = (uint32_t)g;
    h3c_chunk_state f = s_cs[t];
    const uint32_t t0 = at0(f, t, aa, std_domain, pc);
    if (aa.crc0 && f.size && f.type == poly_type && t0 != (std_domain ? ~f.value : f.value)) atomicAdd(&s_stale, 1u);
    if (!aa.crc0 || ahas(aa, E, t)) {
      f.value = std_domain ? ~(t0 ^ a) : (t0 ^ a);
      f.type = poly_type;
    }
    chunks_out[t] = f;
    if (commit) commit[t] = f;
  }
  stores_done();
  __syncthreads();
  if (t == 0 && !vd && aa.crc0) ctr[kCtrStale] = s_stale;
  finish(vd ? kFastVoid : kFastDone);
}

// After a void aligned pass: the deferred blocks' bytes (the last op of the block that passes A6, if any),
// then every op's result from the per-op records -- its delta against the last passing op before it on
// its block, or the block's original bytes (crc0 = the first op's crc0(new ^ old) ^ crc0(new)) -- the final
// states, the counters and the commit, by one workgroup walking the ops in tiles of 1,024.
__global__ __launch_bounds__(1024) void uio_afix_kernel(const h3c_update_io *__restrict__ ios, uint32_t n,
                                                        const h3c_chunk_state *__restrict__ chunks,
                                                        h3c_chunk_state *__restrict__ chunks_out, uint32_t nchunks,
                                                        uint8_t poly_type, uint32_t std_domain,
                                                        const PolyConsts *__restrict__ pc, AlignedArgs aa,
                                                        uint32_t *misc, h3c_update_result *__restrict__ res,
                                                        unsigned long long *__restrict__ ctr,
                                                        h3c_chunk_state *commit) {
  __shared__ uint32_t wagg[16][kFastCols], run[kFastCols], t0s[kFastCols], szs[kFastCols];
  __shared__ unsigned int cnt_ok, cnt_bad, app[kFastCols], stale;
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6, poly = pc->poly;
  // 1. deferred blocks, one wave each: walk back from the block's last op to the last one that passed
  const uint32_t nd = aa.ctl[kADefer];
  const uint32_t E = (aa.ctl[kAEpoch] + 0xFFu) & 0xFFu;  // the pass's epoch (its last workgroup advanced it)
  for (uint32_t d = wave; d < nd; d += 16) {
    const uint2 e = aa.defer[d];
    // the block's last op: the largest listed op of its key (every tile's last op of the block is listed)
    const unsigned long long key = aa.key[e.x];
    uint32_t j = e.x;
    for (uint32_t x = aa.head[fast_bucket(key, aa.hmask)]; aentry_valid(x, E); x = aa.link[(x & 0xFFFFFFu) - 1].y) {
      const uint32_t i = (x & 0xFFFFFFu) - 1;
      if (i >= n) break;
      if (aa.key[i] == key) j = max(j, i);
    }
    while (j != kNil && (uint32_t)(aa.dv[j] >> 32) != 1u) j = aa.pv[j].y;
    if (j == kNil) continue;  // every op of the block failed: it keeps its bytes
    const h3c_update_io f = ios[e.x];
    const uint64_t dst = chunks[f.chunk].base + f.offset, src = ios[j].payload;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<uint4 *>(dst + u * kRowBytes + 16u * lane) =
          *reinterpret_cast<const uint4 *>(src + u * kRowBytes + 16u * lane);
  }
  if (t < kFastCols) {
    run[t] = 0;
    app[t] = 0;
    t0s[t] = t < nchunks ? at0(chunks[t], t, aa, std_domain, pc) : 0u;
    szs[t] = t < nchunks ? chunks[t].size : 0u;
  }
  if (t == 0) cnt_ok = cnt_bad = stale = 0;
  __syncthreads();
  // 2. every op's shifted delta, the per-chunk XORs in sequence order, the results
  for (uint32_t b = 0; b < n; b += 1024) {
    const uint32_t j = b + t;
    uint32_t c = kNil, v = 0;
    bool pass = false;
    if (j < n) {
      const h3c_update_io io = ios[j];
      c = io.chunk;
      pass = (uint32_t)(aa.dv[j] >> 32) == 1u;
      if (pass) {
        uint32_t p = aa.pv[j].y, f = j, lastpass = kNil;
        while (p != kNil) {  // the last passing op before j on the block, else the block's first op
          f = p;
          if ((uint32_t)(aa.dv[p] >> 32) == 1u) {
            lastpass = p;
            break;
          }
          p = aa.pv[p].y;
        }
        const uint32_t old = lastpass != kNil ? aa.pv[lastpass].x : ((uint32_t)aa.dv[f] ^ aa.pv[f].x);
        const uint32_t sh = dxpow8_fast((int64_t)szs[c] - (int64_t)io.offset - (int64_t)kBlk, pc, poly);
        v = dgf_mul(aa.pv[j].x ^ old, sh, poly);
        atomicAdd(&cnt_ok, 1u);
        if (c < kFastCols) atomicOr(&app[c], 1u);
      } else {
        atomicAdd(&cnt_bad, 1u);
      }
    }
    uint32_t acc0 = 0, acc1 = 0, ip = 0;
    for (uint32_t u = 0; u < 64; ++u) {
      const uint32_t cu = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)u);
      const uint32_t vu = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)u);
      if (lane >= u && c == cu) ip ^= vu;
      if (cu == lane) acc0 ^= vu;
      if (cu == lane + 64) acc1 ^= vu;
    }
    wagg[wave][lane] = acc0;
    wagg[wave][64 + lane] = acc1;
    __syncthreads();
    if (j < n && c < kFastCols) {
      uint32_t e = run[c];
      for (uint32_t w = 0; w < wave; ++w) e ^= wagg[w][c];
      const uint32_t sv = t0s[c] ^ e ^ ip;
      h3c_update_result o{};
      o.status = pass ? H3C_OK : H3C_ERR_CHECKSUM_MISMATCH;
      o.size = szs[c];
      o.type = poly_type;
      o.value = pass ? (std_domain ? ~sv : sv) : (std_domain ? 0u : sv);
      res[j] = o;
    }
    __syncthreads();
    if (t < kFastCols) {
      uint32_t x = 0;
      for (uint32_t w = 0; w < 16; ++w) x ^= wagg[w][t];
      run[t] ^= x;
    }
    __syncthreads();
  }
  if (t < nchunks) {  // (exact mode: a chunk with no applied op keeps its stored value)
    h3c_chunk_state f = chunks[t];
    if (aa.crc0 && f.size && f.type == poly_type && t0s[t] != (std_domain ? ~f.value : f.value)) atomicAdd(&stale, 1u);
    if (!aa.crc0 || app[t]) {
      f.value = std_domain ? ~(t0s[t] ^ run[t]) : (t0s[t] ^ run[t]);
      f.type = poly_type;
    }
    chunks_out[t] = f;
    if (commit) commit[t] = f;
  }
  __syncthreads();
  if (t == 0) {
    for (int k = 0; k < kCtrN; ++k) ctr[k] = 0;
    ctr[std_domain ? kCtrRecalc : kCtrRead] = cnt_ok;
    ctr[kCtrMismatch] = cnt_bad;
    if (aa.crc0) ctr[kCtrStale] = stale;
    aa.ctl[kADefer] = 0;
    misc[kMiscFast] = kFastDone;
  }
}

// A second stream per calling thread and device: the payload CRCs run on it while the main
// stream sorts the ops (the sort does not depend on the A6 verdicts).
struct AuxStream {
  int dev = -1;
  hipStream_t st = nullptr;
  hipEvent_t ready = nullptr, done = nullptr;
};
template <class T>
T *carve(char *&p, size_t count) {
  T *r = reinterpret_cast<T *>(p);
  p += (count * sizeof(T) + 255) & ~size_t(255);
  return r;
}

uint32_t bits_for(uint64_t v) {  // bits to represent values < v
  uint32_t b = 0;
  while (b < 64 && (1ull << b) < v) ++b;
  return b;
}

using SortMerge = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                             rocprim::default_config, 1024 * 1024>;

// ---- stable counting sort of (chunk, op) by 8-bit digits, for batches of <= 256 tiles ----
// A pass is two launches with no initialised state: per-tile digit histograms, then a scatter
// in which every tile sums the histograms of the tiles before it (and all of them, for the
// digit bases) and ranks its items stably -- wave ranks from 8 ballots (lanes with the same
// digit), wave offsets from a per-digit prefix over the 16 waves.  Keys of <= 8 bits take one
// pass, <= 16 bits two (least significant digit first).  rocPRIM's onesweep pass measured
// 33 us for 100k keys of 7 bits, its merge path ~50 us for wider keys (r02_prim_probe.txt).
constexpr uint32_t kSortTile = 1024, kSortDigits = 256, kSortMaxTiles = 256;

__global__ __launch_bounds__(kSortTile) void csort_count_kernel(const uint32_t *__restrict__ keys, uint32_t n,
                                                                 uint32_t shift, uint32_t *__restrict__ counts) {
  __shared__ uint32_t h[kSortDigits];
  const uint32_t t = threadIdx.x, i = blockIdx.x * kSortTile + t;
  if (t < kSortDigits) h[t] = 0;
  __syncthreads();
  if (i < n) atomicAdd(&h[(keys[i] >> shift) & (kSortDigits - 1)], 1u);
  __syncthreads();
  if (t < kSortDigits) counts[blockIdx.x * kSortDigits + t] = h[t];
}

__global__ __launch_bounds__(kSortTile) void csort_scatter_kernel(const uint32_t *__restrict__ keys,
                                                                   const uint32_t *__restrict__ vals, uint32_t n,
                                                                   uint32_t shift, uint32_t ntiles,
                                                                   const uint32_t *__restrict__ counts,
                                                                   uint32_t *__restrict__ okeys,
                                                                   uint32_t *__restrict__ ovals) {
  constexpr uint32_t kW = kSortTile / 64, kQ = kSortTile / kSortDigits, kU = 8;
  // 17 KiB of LDS, so a scatter tile fits beside the payload-CRC kernel (140 KiB) on a CU
  __shared__ uint32_t off[kSortDigits];  // where this tile's items of digit b start
  __shared__ uint32_t wsum[kSortDigits / 64];
  __shared__ uint32_t wc[kW][kSortDigits];  // per-wave digit counts, then their prefix over waves
  uint32_t(*part)[kQ][kSortDigits] = reinterpret_cast<uint32_t(*)[kQ][kSortDigits]>(&wc[0][0]);  // first 8 KiB
  const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6, tile = blockIdx.x;
  {  // every tile's histogram, summed by 4 threads per digit with 8 loads in flight each
    const uint32_t dg = t % kSortDigits, q = t / kSortDigits;
    uint32_t pre = 0, tot = 0;
    for (uint32_t u0 = q; u0 < ntiles; u0 += kQ * kU) {
      uint32_t c[kU];
#pragma unroll
      for (uint32_t j = 0; j < kU; ++j) {
        const uint32_t u = u0 + j * kQ;
        c[j] = u < ntiles ? counts[u * kSortDigits + dg] : 0u;
      }
#pragma unroll
      for (uint32_t j = 0; j < kU; ++j) {
        tot += c[j];
        pre += u0 + j * kQ < tile ? c[j] : 0u;
      }
    }
    part[0][q][dg] = pre;
    part[1][q][dg] = tot;
  }
  // this item's digit, and its rank among the wave's lanes with the same digit
  const uint32_t i = tile * kSortTile + t;
  const bool valid = i < n;
  const uint32_t key = valid ? keys[i] : 0u, d = (key >> shift) & (kSortDigits - 1);
  uint64_t m = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
  for (uint32_t b = 0; b < 8; ++b) {
    const uint64_t s = __builtin_amdgcn_ballot_w64((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? s : ~s;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint32_t rank = (uint32_t)__popcll(m & below);
  __syncthreads();
  if (t < kSortDigits) {
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      pre += part[0][q][t];
      tot += part[1][q][t];
    }
    uint32_t inc = tot;  // inclusive scan of the digit totals: in the wave, then across 4 waves
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)inc, o, 64);
      if (lane >= o) inc += x;
    }
    if (lane == 63) wsum[wave] = inc;
    off[t] = inc - tot + pre;
  }
  __syncthreads();  // part is consumed: its LDS becomes the per-wave counts
  for (uint32_t e = t; e < kW * kSortDigits; e += kSortTile) wc[e / kSortDigits][e % kSortDigits] = 0;
  if (t < kSortDigits) {
    uint32_t add = 0;
    for (uint32_t w = 0; w < wave; ++w) add += wsum[w];
    off[t] += add;
  }
  __syncthreads();
  if (valid && rank == 0) wc[wave][d] = (uint32_t)__popcll(m);
  __syncthreads();
  if (t < kSortDigits) {
    uint32_t run = 0;
    for (uint32_t w = 0; w < kW; ++w) {
      const uint32_t x = wc[w][t];
      wc[w][t] = run;
      run += x;
    }
  }
  __syncthreads();
  if (valid) {
    const uint32_t dst = off[d] + wc[wave][d] + rank;
    okeys[dst] = key;
    ovals[dst] = vals[i];
  }
}

size_t csort_tmp_bytes(uint32_t n) {  // counts, and the keys / values between two passes
  const size_t ntiles = (n + kSortTile - 1) / kSortTile;
  return 4 * ntiles * kSortDigits + 256 + 8ull * n + 512;
}
bool csort_fits(uint32_t n, uint32_t bits) { return bits <= 16 && (n + kSortTile - 1) / kSortTile <= kSortMaxTiles; }

// Sort of (chunk, op), stable: the counting sort when it fits, else rocPRIM's merge-sort path
// (faster below 1M items than its onesweep passes for wide keys, profiles/r02_prim_probe.txt).
hipError_t sort_pairs(void *tmp, size_t &tmp_bytes, const uint32_t *k, uint32_t *k2, const uint32_t *v, uint32_t *v2,
                      uint32_t n, uint32_t bits, hipStream_t st) {
  if (!csort_fits(n, bits))
    return rocprim::radix_sort_pairs<SortMerge>(tmp, tmp_bytes, k, k2, v, v2, n, 0, bits, st);
  if (!tmp) {
    tmp_bytes = csort_tmp_bytes(n);
    return hipSuccess;
  }
  if (tmp_bytes < csort_tmp_bytes(n)) return hipErrorInvalidValue;
  const uint32_t ntiles = std::max(1u, (n + kSortTile - 1) / kSortTile);
  char *p = static_cast<char *>(tmp);
  uint32_t *counts = reinterpret_cast<uint32_t *>(p);
  p += (4ull * ntiles * kSortDigits + 255) & ~size_t(255);
  uint32_t *mk = reinterpret_cast<uint32_t *>(p), *mv = mk + n;
  const bool two = bits > 8;
  const uint32_t *ik = k, *iv = v;
  for (uint32_t pass = 0; pass < (two ? 2u : 1u); ++pass) {
    uint32_t *ok = two && pass == 0 ? mk : k2, *ov = two && pass == 0 ? mv : v2;
    hipLaunchKernelGGL(csort_count_kernel, dim3(ntiles), dim3(kSortTile), 0, st, ik, n, 8 * pass, counts);
    hipLaunchKernelGGL(csort_scatter_kernel, dim3(ntiles), dim3(kSortTile), 0, st, ik, iv, n, 8 * pass, ntiles,
                       counts, ok, ov);
    ik = ok;
    iv = ov;
  }
  return hipGetLastError();
}



// ---- per-thread cache of captured pipeline graphs (update_core) ----
// h3c_diag_counter: 0 graph replays, 1 captures, 2 capture failures, 3 front-void redos, 4 phase-B
// reruns, 5 failed-A6 redos, 6 short fragment guesses, 7 fast-branch batches, 8 fast-branch attempts
// abandoned (an op did not qualify), 9 fast-branch recoveries, 10 graphs refused by the topology check,
// 11 graphs refused by the pointer audit (graph_pointers_in_key), 12 aligned sub-branch batches (counted in 7
// too), 13 aligned attempts abandoned (an op not a full aligned block write), 14 aligned passes recomputed by
// uio_afix_kernel (an A6 failure, a deferred block, a look-back that gave up)
enum { kDiagReplay, kDiagCapture, kDiagCaptureFail, kDiagFrontVoid, kDiagPBVoid, kDiagA6Redo, kDiagShortF,
       kDiagFast, kDiagFastAbort, kDiagFastVoid, kDiagTopology, kDiagPtrAudit, kDiagAligned, kDiagAlignedAbort,
       kDiagAlignedFix, kDiagN };
std::atomic<uint64_t> g_graph_stats[kDiagN];
struct UpdGraphKey {
  int dev;
  uint8_t poly;
  uint32_t flags, n, nchunks, cap, hcap;
  const void *chunks, *chunks_out, *ios, *res, *ctr, *lease1, *lease2, *hout;
  hipStream_t aux;
  bool operator==(const UpdGraphKey &o) const { return std::memcmp(this, &o, sizeof(*this)) == 0; }
};
struct UpdGraphs {
  UpdGraphKey key{};
  hipGraphExec_t g = nullptr;
  bool failed = false;
  uint64_t used = 0;
};
// The graphs of `key`, or nullptr when this call should launch plainly: the first sight of a
// shape launches plainly (a caller whose buffers move every call never pays a capture); a
// shape seen among the last four plain calls returns an empty entry to capture into; later
// sights replay.  Graphs are not
// used while `st` itself is being captured, or with h3c_test_hook(H3C_HOOK_UPD_GRAPHS, 1).
// Per-thread HIP resources -- the aux stream sets, the capture streams, the graph cache.  When a
// thread ends they go back to process-wide pools (no HIP call in a thread-exit destructor) and the
// next thread that needs one on the same device takes it from there; graph execs of ended threads
// are destroyed by the next update call.  A caller that spawns short-lived threads therefore
// reuses a bounded set of streams instead of leaking them.
// The fast branch's per-thread scratch: the slow word and the bucket heads, zero between batches (the
// batch's tail kernels clear what it set), so no launch zeroes them per batch.  `dirty`: not known to be
// zero (new, or a batch that did not reach its outcome) -- zeroed before the next use.
struct FastScratch {
  int dev = -1;
  uint32_t *p = nullptr;
  size_t words = 0;
  bool dirty = true;
  uint32_t hcap = 0;      // the bucket count the heads were laid out for (another one: zeroed first)
  uint32_t abatches = 0;  // aligned batches since the last zeroing (the 8-bit epoch must not wrap onto live entries)
  bool fresh = true;      // newly allocated: its aligned range weights are not learnt yet (zeroed with the rest)
};
struct ResPool {
  std::mutex mu;
  std::vector<AuxStream> aux;
  std::vector<std::pair<int, hipStream_t>> cap;
  std::vector<hipGraphExec_t> dead;
  std::vector<FastScratch> scratch;
};
ResPool g_res;

struct ThreadRes {
  AuxStream aux[4];
  int aux_next = 0;
  hipStream_t cs[8] = {};
  int cs_dev[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  UpdGraphs cache[4];
  UpdGraphKey recent[4] = {};  // keys of the last plain calls (lease pools may alternate buffers)
  uint32_t recent_next = 0;
  // the fast branch's last outcome per batch shape and tables: a shape whose last batch did not
  // qualify goes straight to the general pipeline (an abandoned attempt costs a prep launch and a
  // synchronisation); it is tried again after kFastRetry general batches
  struct FastPred {
    int dev = -1;
    uint32_t flags = 0, n = 0, nchunks = 0, general_runs = 0;
    uint32_t last_us = 0;  // the last fast batch's time from its first launch to the outcome word (host clock)
    uint8_t aslow = 0;     // the aligned sub-branch: the shape's last attempt found an op it does not take
    uint32_t a_runs = 0;   // ... and the batches of the shape run without trying it since
    const void *chunks = nullptr, *ios = nullptr;
    uint8_t poly = 0, slow = 0;
    uint64_t used = 0;
  } pred[8];
  uint64_t tick = 0;
  std::vector<FastScratch> fscratch;  // one per device
  ~ThreadRes() {
    std::lock_guard<std::mutex> lk(g_res.mu);
    for (FastScratch &f : fscratch)
      if (f.p) {
        f.dirty = true;  // (the next owner zeroes it)
        g_res.scratch.push_back(f);
      }
    for (AuxStream &a : aux)
      if (a.st) g_res.aux.push_back(a);
    for (int i = 0; i < 8; ++i)
      if (cs[i]) g_res.cap.emplace_back(cs_dev[i], cs[i]);
    for (UpdGraphs &g : cache)
      if (g.g) g_res.dead.push_back(g.g);
  }
};
ThreadRes &tres() {
  thread_local ThreadRes r;
  return r;
}

// This thread's fast scratch on `dev` with at least `words` words (nullptr: allocation failed).
FastScratch *fast_scratch(int dev, size_t words) {
  ThreadRes &r = tres();
  FastScratch *f = nullptr;
  for (FastScratch &x : r.fscratch)
    if (x.dev == dev) f = &x;
  if (f && f->words >= words) return f;
  if (f) {  // too small: freed (this thread's earlier batches have completed)
    (void)hipFree(f->p);
    f->p = nullptr;
    f->words = 0;
  } else {
    r.fscratch.emplace_back();
    f = &r.fscratch.back();
    f->dev = dev;
  }
  {  // an ended thread's scratch, if one is large enough
    std::lock_guard<std::mutex> lk(g_res.mu);
    for (size_t i = 0; i < g_res.scratch.size(); ++i)
      if (g_res.scratch[i].dev == dev && g_res.scratch[i].words >= words) {
        *f = g_res.scratch[i];
        g_res.scratch.erase(g_res.scratch.begin() + (long)i);
        f->dirty = true;
        return f;
      }
  }
  const size_t w = std::max<size_t>(words, 1 + 4096);
  if (hipMalloc(reinterpret_cast<void **>(&f->p), w * 4) != hipSuccess) {
    f->p = nullptr;
    f->words = 0;
    return nullptr;
  }
  f->words = w;
  f->dirty = true;
  f->fresh = true;
  return f;
}
struct ScratchGuard {  // marks the scratch suspect unless the batch's outcome was read (disarm)
  FastScratch *f;
  ~ScratchGuard() {
    if (f) f->dirty = true;
  }
};

void drain_dead_graphs() {
  std::vector<hipGraphExec_t> dead;
  {
    std::lock_guard<std::mutex> lk(g_res.mu);
    dead.swap(g_res.dead);
  }
  for (hipGraphExec_t g : dead) (void)hipGraphExecDestroy(g);
}

// A second stream per calling thread and device (and its fork / join events).
int aux_stream(int dev, AuxStream *&out) {
  ThreadRes &tr = tres();
  for (AuxStream &a : tr.aux)
    if (a.dev == dev && a.st) {
      out = &a;
      return H3C_OK;
    }
  AuxStream &a = tr.aux[tr.aux_next++ & 3];
  {
    std::lock_guard<std::mutex> lk(g_res.mu);
    if (a.st) g_res.aux.push_back(a);  // a thread using more than 4 devices hands the oldest back
    a = AuxStream{};
    for (size_t i = 0; i < g_res.aux.size(); ++i)
      if (g_res.aux[i].dev == dev) {
        a = g_res.aux[i];
        g_res.aux.erase(g_res.aux.begin() + (long)i);
        break;
      }
  }
  if (!a.st) {
    HIP_TRY(hipStreamCreateWithFlags(&a.st, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&a.ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&a.done, hipEventDisableTiming));
    a.dev = dev;
  }
  out = &a;
  return H3C_OK;
}

constexpr uint32_t kFastRetry = 64;
ThreadRes::FastPred &fast_pred(int dev, uint8_t poly, uint32_t flags, uint32_t n, uint32_t nchunks, const void *chunks,
                               const void *ios) {
  ThreadRes &tr = tres();
  ThreadRes::FastPred *victim = &tr.pred[0];
  for (ThreadRes::FastPred &p : tr.pred) {
    if (p.dev == dev && p.poly == poly && p.flags == flags && p.n == n && p.nchunks == nchunks && p.chunks == chunks &&
        p.ios == ios) {
      p.used = ++tr.tick;
      return p;
    }
    if (p.used < victim->used) victim = &p;
  }
  *victim = ThreadRes::FastPred{};
  victim->dev = dev;
  victim->poly = poly;
  victim->flags = flags;
  victim->n = n;
  victim->nchunks = nchunks;
  victim->chunks = chunks;
  victim->ios = ios;
  victim->used = ++tr.tick;
  return *victim;
}

UpdGraphs *upd_graphs(const UpdGraphKey &key_in, hipStream_t st, bool asked) {
  ThreadRes &tr = tres();
  UpdGraphs(&cache)[4] = tr.cache;
  UpdGraphKey(&recent)[4] = tr.recent;
  uint32_t &recent_next = tr.recent_next;
  uint64_t &tick = tr.tick;
  // Only when the caller asks (H3C_UPD_GRAPHS): a launch into the legacy default stream made by
  // ANY thread of the process while a stream is capturing fails in HIP ("operation not permitted
  // when stream is capturing") and invalidates the capture, whatever the capture mode or the
  // capture stream's flags -- a 16-thread stress with captures in flight saw hundreds of such
  // failures (profiles/r02b_tsan.txt).  The engine cannot see other users of the GPU (PyTorch,
  // the caller's own threads), so only the caller can promise that none launches meanwhile.
  // Test hook: 1 never captures, 2 captures without the flag.
  const uint64_t hk = h3c_rt::hook(H3C_HOOK_UPD_GRAPHS);
  if (hk == 1 || (!asked && hk != 2 && hk != 3)) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return nullptr;
  }
  UpdGraphKey key;
  std::memset(&key, 0, sizeof(key));  // padding compared by memcmp
  key.dev = key_in.dev;
  key.poly = key_in.poly;
  key.flags = key_in.flags;
  key.n = key_in.n;
  key.nchunks = key_in.nchunks;
  key.cap = key_in.cap;
  key.hcap = key_in.hcap;
  key.chunks = key_in.chunks;
  key.chunks_out = key_in.chunks_out;
  key.ios = key_in.ios;
  key.res = key_in.res;
  key.ctr = key_in.ctr;
  key.lease1 = key_in.lease1;
  key.lease2 = key_in.lease2;
  key.hout = key_in.hout;  // (phase B writes the outcome words there)
  key.aux = key_in.aux;
  ++tick;
  for (UpdGraphs &g : cache)
    if (g.used && g.key == key) {
      g.used = tick;
      return g.failed ? nullptr : &g;
    }
  bool seen = false;
  for (const UpdGraphKey &r : recent) seen = seen || r == key;
  if (!seen) {
    recent[recent_next++ & 3] = key;
    return nullptr;
  }
  UpdGraphs *victim = &cache[0];
  for (UpdGraphs &g : cache)
    if (g.used < victim->used) victim = &g;
  if (victim->g) (void)hipGraphExecDestroy(victim->g);
  *victim = UpdGraphs{};
  victim->key = key;
  victim->used = tick;
  return victim;
}

// A per-thread, per-device stream to capture on: the caller's stream may be the legacy
// default stream, which cannot be captured (a graph then launches on it all the same).
hipStream_t capture_stream(int dev) {
  ThreadRes &tr = tres();
  for (int i = 0; i < 8; ++i)
    if (tr.cs_dev[i] == dev && tr.cs[i]) return tr.cs[i];
  for (int i = 0; i < 8; ++i)
    if (!tr.cs[i]) {
      {
        std::lock_guard<std::mutex> lk(g_res.mu);
        for (size_t k = 0; k < g_res.cap.size(); ++k)
          if (g_res.cap[k].first == dev) {
            tr.cs[i] = g_res.cap[k].second;
            g_res.cap.erase(g_res.cap.begin() + (long)k);
            break;
          }
      }
      if (!tr.cs[i] && hipStreamCreateWithFlags(&tr.cs[i], hipStreamNonBlocking) != hipSuccess) {
        tr.cs[i] = nullptr;
        return nullptr;
      }
      tr.cs_dev[i] = dev;
      return tr.cs[i];
    }
  return nullptr;
}

// Captures what `body` enqueues on `st` (and the streams it forks) into an executable graph.
// One capture at a time in the process: under concurrent captures from several threads the
// runtime failed captures and then other threads' launches ("operation failed due to a previous
// error during capture", profiles/r02b_tsan.txt).  Captures are rare (once per batch shape
// and thread), so the lock costs nothing in steady state.
std::mutex g_capture_mu;

// The shape of a captured graph (h3c_diag_last_graph): node count, root count, memset + memcpy nodes,
// kernel nodes, nodes reachable from the first root through edges, edges, the largest out-degree.
struct GraphShape {
  uint64_t nodes = 0, roots = 0, copies = 0, kernels = 0, reachable = 0, edges = 0, max_out = 0;
};
thread_local GraphShape t_last_graph;

// The engine's pipelines are chains of kernel nodes on one stream.  A captured graph is instantiated
// only if it is one: a single root, every node reachable from it, and no memset / memcpy node (round 3:
// a hipMemsetAsync at the head of the captured UpdateIO pipeline became a memset node that replays did
// not order before the prep kernel -- stale tickets, an illegal access; profiles/r04_graph_probe.txt
// records what HIP captures for that form).  Anything else runs as plain launches (h3c_diag_counter 10).
bool graph_is_a_chain(hipGraph_t g, GraphShape &sh) {
  sh = GraphShape{};
  size_t nn = 0, nr = 0, ne = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess || hipGraphGetRootNodes(g, nullptr, &nr) != hipSuccess ||
      hipGraphGetEdges(g, nullptr, nullptr, &ne) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  std::vector<hipGraphNode_t> nodes(nn), roots(nr), from(ne), to(ne);
  if ((nn && hipGraphGetNodes(g, nodes.data(), &nn) != hipSuccess) ||
      (nr && hipGraphGetRootNodes(g, roots.data(), &nr) != hipSuccess) ||
      (ne && hipGraphGetEdges(g, from.data(), to.data(), &ne) != hipSuccess)) {
    (void)hipGetLastError();
    return false;
  }
  sh.nodes = nn;
  sh.roots = nr;
  sh.edges = ne;
  for (hipGraphNode_t x : nodes) {
    hipGraphNodeType ty = hipGraphNodeTypeCount;
    if (hipGraphNodeGetType(x, &ty) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    sh.copies += ty == hipGraphNodeTypeMemset || ty == hipGraphNodeTypeMemcpy;
    sh.kernels += ty == hipGraphNodeTypeKernel;
  }
  std::vector<hipGraphNode_t> seen, todo;
  if (nr) todo.push_back(roots[0]);
  while (!todo.empty()) {
    const hipGraphNode_t x = todo.back();
    todo.pop_back();
    if (std::find(seen.begin(), seen.end(), x) != seen.end()) continue;
    seen.push_back(x);
    uint64_t out = 0;
    for (size_t e = 0; e < ne; ++e)
      if (from[e] == x) {
        todo.push_back(to[e]);
        ++out;
      }
    sh.max_out = std::max(sh.max_out, out);
  }
  sh.reachable = seen.size();
  return nr == 1 && sh.copies == 0 && sh.reachable == nn;
}

}  // namespace
// The struct arguments of capturable kernels: their pointer members (h3c_rt::ArgLayout).
namespace h3c_rt {
template <>
struct ArgLayout<FastArgs, void> {
  static void fill(ArgSpec &a) {
    struct_arg<FastArgs>(a, {offsetof(FastArgs, frag), offsetof(FastArgs, key), offsetof(FastArgs, link),
                             offsetof(FastArgs, head), offsetof(FastArgs, dv), offsetof(FastArgs, slow),
                             offsetof(FastArgs, pc), offsetof(FastArgs, chain)});
  }
};
template <>
struct ArgLayout<AlignedArgs, void> {
  static void fill(ArgSpec &a) {
    struct_arg<AlignedArgs>(a, {offsetof(AlignedArgs, ctl), offsetof(AlignedArgs, head), offsetof(AlignedArgs, gran),
                                offsetof(AlignedArgs, key), offsetof(AlignedArgs, link), offsetof(AlignedArgs, dv),
                                offsetof(AlignedArgs, pv), offsetof(AlignedArgs, inp), offsetof(AlignedArgs, defer),
                                offsetof(AlignedArgs, rec), offsetof(AlignedArgs, pr),
                                offsetof(AlignedArgs, stat), offsetof(AlignedArgs, hand),
                                offsetof(AlignedArgs, crc0)});
  }
};
template <>
struct ArgLayout<TMapFn, void> {
  static void fill(ArgSpec &a) {
    struct_arg<TMapFn>(a, {offsetof(TMapFn, pos), offsetof(TMapFn, eacc), offsetof(TMapFn, payraw),
                           offsetof(TMapFn, pc), offsetof(TMapFn, a6)});
  }
};
template <>
struct ArgLayout<SMapFn, void> {
  static void fill(ArgSpec &a) {
    struct_arg<SMapFn>(a, {offsetof(SMapFn, pos), offsetof(SMapFn, skey), offsetof(SMapFn, tscan),
                           offsetof(SMapFn, t0v), offsetof(SMapFn, eacc), offsetof(SMapFn, payraw),
                           offsetof(SMapFn, pc), offsetof(SMapFn, a6)});
  }
};
}  // namespace h3c_rt
namespace {

// Every kernel update_core may enqueue while capturing, with its argument layout.  A captured graph
// holding a kernel not listed here (rocPRIM's, on the paths that call it) is not instantiated.
const std::vector<h3c_rt::KernelSig> &capturable_kernels() {
  using h3c_rt::kernel_sig;
  static const std::vector<h3c_rt::KernelSig> sigs = {
#define H3C_SIG(k) kernel_sig(k, #k)
      H3C_SIG(uio_zero_kernel), H3C_SIG(uio_prep_kernel), H3C_SIG(csort_count_kernel),
      H3C_SIG(csort_scatter_kernel), H3C_SIG(uio_verify_t0_kernel), H3C_SIG(uio_sz_elem_kernel),
      H3C_SIG(uio_classify_kernel), H3C_SIG(uio_late_verify_kernel), H3C_SIG(uio_front_kernel),
      H3C_SIG(uio_frag_kernel), H3C_SIG(uio_tlink_kernel), H3C_SIG(uio_resolve_kernel), H3C_SIG(uio_heads_kernel),
      H3C_SIG(uio_block_kernel), H3C_SIG(uio_phaseb_kernel), H3C_SIG(uio_elem_kernel<TMapFn>),
      H3C_SIG(uio_elem_kernel<SMapFn>), H3C_SIG(uio_result_kernel), H3C_SIG(uio_stale_kernel),
      H3C_SIG(uio_commit_kernel), H3C_SIG(uio_fast_link_kernel), H3C_SIG(uio_fast_kernel),
      H3C_SIG(uio_fast_sum_kernel), H3C_SIG(uio_fast_res_kernel), H3C_SIG(uio_aprep_kernel),
      H3C_SIG(uio_afused_kernel), H3C_SIG(uio_apiece_kernel), h3c_rt::uio_piece_kernel_sig(),
#undef H3C_SIG
  };
  return sigs;
}

// What the last capture's pointer audit saw (h3c_diag_last_graph_audit): kernel nodes audited, pointer
// arguments checked, pointers outside every named buffer, kernel nodes with no registered layout.
struct GraphAudit {
  uint64_t kernels = 0, pointers = 0, outside = 0, unknown = 0;
};
thread_local GraphAudit t_last_audit;
struct AddrRange {
  uint64_t lo, hi;  // [lo, hi)
};

// Every pointer argument of every kernel node of `g` is null or lies inside one of `allow` (the
// buffers named by the batch's UpdGraphKey and the library's constant tables).  A kernel node whose
// function has no registered layout fails the audit (its arguments cannot be read).
bool graph_pointers_in_key(hipGraph_t g, const std::vector<AddrRange> &allow, GraphAudit &au) {
  au = GraphAudit{};
  size_t nn = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  std::vector<hipGraphNode_t> nodes(nn);
  if (nn && hipGraphGetNodes(g, nodes.data(), &nn) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const std::vector<h3c_rt::KernelSig> &sigs = capturable_kernels();
  bool ok = true;
  for (hipGraphNode_t x : nodes) {
    hipGraphNodeType ty = hipGraphNodeTypeCount;
    if (hipGraphNodeGetType(x, &ty) != hipSuccess || ty != hipGraphNodeTypeKernel) {
      (void)hipGetLastError();
      continue;  // (graph_is_a_chain refuses every other node type)
    }
    hipKernelNodeParams p{};
    if (hipGraphKernelNodeGetParams(x, &p) != hipSuccess) {
      (void)hipGetLastError();
      ++au.unknown;
      ok = false;
      continue;
    }
    ++au.kernels;
    const h3c_rt::KernelSig *sig = nullptr;
    for (const h3c_rt::KernelSig &s : sigs)
      if (s.fn == p.func) sig = &s;
    // the argument values: one pointer per argument (kernelParams), or one packed buffer (`extra`)
    const char *packed = nullptr;
    size_t packed_size = 0;
    if (!p.kernelParams && p.extra) {
      for (void **e = p.extra; *e != HIP_LAUNCH_PARAM_END; e += 2) {
        if (*e == HIP_LAUNCH_PARAM_BUFFER_POINTER) packed = static_cast<const char *>(e[1]);
        if (*e == HIP_LAUNCH_PARAM_BUFFER_SIZE) packed_size = *static_cast<const size_t *>(e[1]);
      }
    }
    if (!sig || (!p.kernelParams && !packed)) {
      ++au.unknown;
      ok = false;
      continue;
    }
    size_t off = 0;
    for (uint32_t i = 0; i < sig->nargs; ++i) {
      const h3c_rt::ArgSpec &a = sig->args[i];
      off = (off + a.align - 1) / a.align * a.align;
      const char *v = p.kernelParams ? static_cast<const char *>(p.kernelParams[i]) : packed + off;
      off += a.size;
      if (!p.kernelParams && off > packed_size) {
        ++au.unknown;
        ok = false;
        break;
      }
      for (uint32_t q = 0; q < a.nptr; ++q) {
        uint64_t ptr = 0;
        std::memcpy(&ptr, v + a.ptr_off[q], sizeof(ptr));
        ++au.pointers;
        if (!ptr) continue;
        bool in = false;
        for (const AddrRange &r : allow) in = in || (ptr >= r.lo && ptr < r.hi);
        if (!in) {
          ++au.outside;
          ok = false;
        }
      }
    }
  }
  return ok && au.kernels;
}

template <class Body>
int capture_graph(hipStream_t st, Body body, hipGraphExec_t &out, const std::vector<AddrRange> &allow) {
  std::lock_guard<std::mutex> lk(g_capture_mu);
  std::unique_lock<std::shared_mutex> gate(h3c_rt::capture_gate());  // (legacy-stream entries wait it out)
  // Relaxed: the capture makes no synchronous or allocating call itself, and it should not make
  // other threads' calls fail (under the thread-local mode a 16-thread stress saw another
  // thread's hipMemcpy fail; see upd_graphs for the legacy-stream limit that remains).
  const hipError_t be = hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed);
  if (be != hipSuccess) {
    h3c_rt::set_error("graph capture: hipStreamBeginCapture", be);
    return H3C_ERR_HIP;
  }
  const int r = body();
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(st, &g);
  if (r || e != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    if (!r) h3c_rt::set_error("graph capture: hipStreamEndCapture", e);  // (else the body's error stays)
    return r ? r : H3C_ERR_HIP;
  }
  if (!graph_is_a_chain(g, t_last_graph)) {  // not instantiated: plain launches for this shape
    (void)hipGraphDestroy(g);
    g_graph_stats[kDiagTopology].fetch_add(1);
    h3c_rt::set_error_text("graph capture: the captured pipeline is not one chain of kernel nodes");
    out = nullptr;
    return H3C_ERR_HIP;
  }
  if (!graph_pointers_in_key(g, allow, t_last_audit)) {  // a baked-in pointer the key does not name
    (void)hipGraphDestroy(g);
    g_graph_stats[kDiagPtrAudit].fetch_add(1);
    h3c_rt::set_error_text("graph capture: a kernel argument points outside the buffers of the graph key");
    out = nullptr;
    return H3C_ERR_HIP;
  }
  const hipError_t ie = hipGraphInstantiate(&out, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (ie != hipSuccess) {
    h3c_rt::set_error("graph capture: hipGraphInstantiate", ie);
    out = nullptr;
    return H3C_ERR_HIP;
  }
  return H3C_OK;
}

// Host-time trace of this thread's h3c_update_ios_dev calls on the fast branches (h3c_diag_host_trace):
// summed nanoseconds of [0] the previous call's return to this call's entry (the caller's own time),
// [1] entry to the first launch, [2] the launches, [3] the last launch to the outcome word seen, [4] the
// outcome to the return; [5] the number of calls.
struct HostTrace {
  std::chrono::steady_clock::time_point entry, last_return, launch0, launched, seen;
  bool have_return = false;
  uint64_t sum[6] = {0, 0, 0, 0, 0, 0};
};
thread_local HostTrace t_host;
inline uint64_t ns_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return (uint64_t)std::max<int64_t>(0, std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count());
}

// Spin (bounded) until the device sets a pinned host word; a blocking stream wait follows either way.
// The bound: h3c_test_hook(H3C_HOOK_FAST_POLL_US) / H3C_FAST_POLL_US when set, else twice the time this
// thread's last fast batch of the same shape took to reach its outcome (+ 50 us), within
// [kFastPollMinUs, kFastPollUs] -- a caller's core is not burnt for milliseconds on a batch known to take
// 0.3 ms, and a batch that runs long (a contended GPU) falls back to the blocking wait.
constexpr uint32_t kFastPollUs = 2000, kFastPollMinUs = 100;
uint32_t fast_poll_budget_us(uint32_t last_us) {
  const uint64_t hk = h3c_rt::hook(H3C_HOOK_FAST_POLL_US);
  if (hk) return (uint32_t)std::min<uint64_t>(hk, 1000000u);
  if (!last_us) return kFastPollUs;
  return std::min(kFastPollUs, std::max(kFastPollMinUs, 2 * last_us + 50));
}
bool poll_host_word(const uint32_t *w, uint32_t max_us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0; !__atomic_load_n(w, __ATOMIC_ACQUIRE); ++i) {
    __builtin_ia32_pause();
    if ((i & 255) == 255 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(max_us))
      return false;
  }
  return true;
}

// The stream's work done: hipStreamQuery polled for up to max_us (once the outcome word is set, the
// last kernel is ending; hipStreamSynchronize took 8-14 us more to return, profiles/r04_updio_host_timeline.txt),
// then the blocking wait.
hipError_t stream_wait(hipStream_t st, uint32_t max_us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    const hipError_t q = hipStreamQuery(st);
    if (q != hipErrorNotReady) return q;
    __builtin_ia32_pause();
    if ((i & 15) == 15 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(max_us)) break;
  }
  return hipStreamSynchronize(st);
}

// The pipeline on device arrays: chunks_in (read), chunks_out (final states; may not alias
// chunks_in), ios, results, ctr (h3c_update_counters layout, 8 x u64).  `epilogue` enqueues the
// caller's copies of the outputs before the final synchronisation; with `epi_graph` (its work is
// device-only and its arguments are part of the graph key) it is captured into the batch's graph.
// `commit_dev` (the device-table entry: the epilogue is its commit): the fast branch's tail commits the
// final states there itself and the epilogue runs only if the batch leaves the fast branch.
// Synchronous.
template <class Epilogue>
int update_core(uint8_t poly_type, const h3c_chunk_state *d_chunks, h3c_chunk_state *d_chunks_out, uint32_t nchunks,
                const h3c_update_io *d_ios, uint32_t n, h3c_update_result *d_res, uint32_t flags,
                unsigned long long *d_ctr, hipStream_t st, int dev, Epilogue epilogue, bool epi_graph = false,
                h3c_chunk_state *commit_dev = nullptr) {
  const bool std_domain = (flags & H3C_UPD_STD_DOMAIN) != 0;
  const bool exact = (flags & H3C_UPD_EXACT) != 0;
  flags &= H3C_UPD_STD_DOMAIN | H3C_UPD_EXACT | H3C_UPD_GRAPHS;
  drain_dead_graphs();
  const PolyConsts *pc = static_cast<const PolyConsts *>(h3c_rt::device_consts(dev, poly_type));
  const uint32_t poly = poly_type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;
  const uint32_t stdf = std_domain ? 1u : 0u, exactf = exact ? 1u : 0u;
  const uint32_t C = std::max(nchunks, 1u);

  // ---- device scratch: per op, per chunk, and per fragment for a guessed fragment count ----
  // (a fragment per 4 KiB block an op touches: one per block-aligned write of <= 4 KiB; the
  // guess is the larger of 2n + 1024 and the calling thread's last batch, and a batch that
  // needs more redoes its fragment stage once with the count known)
  const uint32_t ntiles_front = (uint32_t)((n + kFrontTile - 1) / kFrontTile);
  const uint32_t ntiles_pb = (uint32_t)((n + kPhaseBTile - 1) / kPhaseBTile);
  const uint32_t pbz_words = ntiles_pb * (uint32_t)(sizeof(PhaseBSlot) / 4) + 1;
  thread_local uint32_t last_frags = 0;
  // the one-pass front (uio_front_kernel) on the first attempt; test hook H3C_HOOK_UPD_FRONT = 1: the
  // scan-based stage (redone attempts always take that one)
  const bool front_path = (h3c_rt::hook(H3C_HOOK_UPD_FRONT) & 1) == 0;
  uint32_t cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(2ull * n + 1024, last_frags), 0x7FFFFFF0u);
  // the prep kernel's grid on the first attempt (its threads cover the piece items and the front
  // kernel's initialisations) and, on the serial front path, its scan states
  uint32_t hcap0 = 256;
  while (hcap0 < cap) hcap0 <<= 1;
  const uint32_t fz_words0 = front_path ? ntiles_front * (uint32_t)(sizeof(FrontSlot) / 4) : 0u;
  const uint32_t prep_tiles = (uint32_t)((std::max<size_t>(std::max<size_t>((size_t)n + C + 1, nchunks),
                                                           std::max<size_t>(fz_words0, front_path ? hcap0 : 0u)) +
                                          kPrepTile - 1) / kPrepTile);
  size_t sort_tmp = 0, scan_tmp = 0, pscan_tmp = 0, szscan_tmp = 0, ascan_tmp = 0;
  const uint32_t bits = bits_for((uint64_t)nchunks + 1);
  // rocPRIM's scratch sizes: each query makes ~6 device-property calls (~14 us per batch in all,
  // profiles/r04_updio_host_timeline.txt), so they are kept per thread for the last shapes seen
  struct TmpSizes {
    int dev = -1;
    uint32_t n = 0, C = 0, bits = 0;
    size_t v[5] = {};
  };
  thread_local TmpSizes tmp_cache[4];
  thread_local uint32_t tmp_next = 0;
  TmpSizes *ts_hit = nullptr;
  for (TmpSizes &x : tmp_cache)
    if (x.dev == dev && x.n == n && x.C == C && x.bits == bits) ts_hit = &x;
  if (ts_hit) {
    sort_tmp = ts_hit->v[0], scan_tmp = ts_hit->v[1], pscan_tmp = ts_hit->v[2], szscan_tmp = ts_hit->v[3];
    ascan_tmp = ts_hit->v[4];
  } else {
    HIP_TRY(sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, nullptr, n, bits, st));
    HIP_TRY(rocprim::exclusive_scan(nullptr, scan_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)n + 1,
                                    rocprim::plus<uint32_t>(), st));
    HIP_TRY(rocprim::exclusive_scan(nullptr, pscan_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u,
                                    (size_t)n + C + 1, rocprim::plus<uint32_t>(), st));
    HIP_TRY(rocprim::inclusive_scan_by_key(nullptr, szscan_tmp, (uint32_t *)nullptr, (SzTy *)nullptr, (SzTy *)nullptr,
                                           (size_t)n, SzTyOp(), rocprim::equal_to<uint32_t>(), st));
    HIP_TRY(rocprim::inclusive_scan_by_key(nullptr, ascan_tmp, (uint32_t *)nullptr, (Aff *)nullptr, (Aff *)nullptr,
                                           (size_t)n, AffOp{poly}, rocprim::equal_to<uint32_t>(), st));
    TmpSizes &e = tmp_cache[tmp_next++ % 4];
    e.dev = dev, e.n = n, e.C = C, e.bits = bits;
    e.v[0] = sort_tmp, e.v[1] = scan_tmp, e.v[2] = pscan_tmp, e.v[3] = szscan_tmp, e.v[4] = ascan_tmp;
  }
  const size_t tmp_bytes =
      std::max(std::max(std::max(sort_tmp, scan_tmp), std::max(szscan_tmp, ascan_tmp)), pscan_tmp);
  const size_t N1 = (size_t)n + 1, NP = (size_t)n + C;  // NP: piece-pass items (ops, then chunks)
  uint32_t *d_status, *d_key, *d_idx, *d_skey, *d_order, *d_np, *d_pbase, *d_paycrc0, *d_payraw, *d_nfrag, *d_fbase,
      *d_eacc, *d_t0, *d_misc, *d_a6, *d_late, *d_lbase;
  SzTy *d_sz, *d_szscan;
  FrontSlot *d_fslot;
  uint32_t *d_pbz;  // uio_phaseb_kernel: tile states, then its ticket
  OpPos *d_pos;
  Aff *d_tel, *d_tscan, *d_sel, *d_sscan;
  void *d_tmp, *d_ptmp;
  uint32_t *d_sstate;  // the prep kernel's scan states (serial front path)
  // the fast branch (uio_fast_kernel): tried first when the batch names <= 128 chunks, unless this
  // thread's last batch of the same shape and tables did not qualify (or the test hook says otherwise)
  const uint64_t fast_hook = h3c_rt::hook(H3C_HOOK_UPD_FAST);
  const uint32_t giveup = (uint32_t)h3c_rt::hook(H3C_HOOK_UPD_GIVEUP);
  const bool fast_able = fast_hook != 1 && nchunks >= 1 && nchunks <= kFastCols;
  ThreadRes::FastPred *fpred = fast_able ? &fast_pred(dev, poly_type, flags & ~H3C_UPD_GRAPHS, n, nchunks, d_chunks, d_ios)
                                         : nullptr;
  const bool try_fast = fast_able && (fast_hook == 2 || !fpred->slow || fpred->general_runs >= kFastRetry);
  // the aligned sub-branch (uio_aprep_kernel + uio_afused_kernel): tried before the chain-based branch when
  // every op may be a full aligned 4 KiB WRITE (trusted stored checksums), unless this thread's last batch of
  // the shape had an op it does not take (test hook H3C_HOOK_UPD_ALIGNED: 1 never, 2 always tried)
  const uint64_t aligned_hook = h3c_rt::hook(H3C_HOOK_UPD_ALIGNED);
  const bool try_aligned = fast_able && n <= kAMaxOps && aligned_hook != 1 &&
                           (aligned_hook == 2 || !fpred->aslow || fpred->a_runs >= kFastRetry);
  AlignedArgs aa{};
  const uint32_t nwg_fast = (uint32_t)std::max(1, h3c_rt::device_num_cu(dev)) * H3C_FAST_WG_MULT;
  const uint32_t ntiles_tail = (uint32_t)std::max<size_t>(1, ((size_t)n + 1023) / 1024);  // the tail kernels
  uint32_t hcap_fast = 256;
  while (hcap_fast < 2 * n) hcap_fast <<= 1;
  FastArgs fa{};
  unsigned long long *d_gran = nullptr;
  uint2 *d_part = nullptr;  // uio_fast_sum_kernel -> uio_fast_res_kernel: each op's XOR in its tile, chunk, state
  uint32_t *d_heavy = nullptr;  // uio_fast_link_kernel -> uio_fast_kernel: the starts of chains with later ops
  auto layout = [&](char *base) -> size_t {  // one layout, run with base 0 to size the lease
    char *cur = base;
    d_status = carve<uint32_t>(cur, n);
    d_key = carve<uint32_t>(cur, n);
    d_idx = carve<uint32_t>(cur, n);
    d_skey = carve<uint32_t>(cur, n);
    d_order = carve<uint32_t>(cur, n);
    d_np = carve<uint32_t>(cur, NP + 1);
    d_pbase = carve<uint32_t>(cur, NP + 1);
    d_paycrc0 = carve<uint32_t>(cur, NP);
    d_payraw = carve<uint32_t>(cur, n);
    d_a6 = carve<uint32_t>(cur, n);
    d_nfrag = carve<uint32_t>(cur, N1);
    d_fbase = carve<uint32_t>(cur, N1);
    d_late = carve<uint32_t>(cur, N1);
    d_lbase = carve<uint32_t>(cur, N1);
    d_eacc = carve<uint32_t>(cur, 2 * (size_t)n);
    d_t0 = carve<uint32_t>(cur, C);
    d_misc = carve<uint32_t>(cur, kMiscN);
    d_fslot = carve<FrontSlot>(cur, std::max(ntiles_front, 1u));
    d_pbz = carve<uint32_t>(cur, pbz_words);
    d_sz = carve<SzTy>(cur, n);
    d_szscan = carve<SzTy>(cur, n);
    d_pos = carve<OpPos>(cur, n);
    d_tel = carve<Aff>(cur, n);
    d_tscan = carve<Aff>(cur, n);
    d_sel = carve<Aff>(cur, n);
    d_sscan = carve<Aff>(cur, n);
    d_tmp = carve<char>(cur, tmp_bytes);
    d_ptmp = carve<char>(cur, pscan_tmp);
    d_sstate = carve<uint32_t>(cur, 3 + (size_t)prep_tiles);
    if (fast_able) {
      fa.frag = carve<FragDesc>(cur, n);
      fa.key = carve<unsigned long long>(cur, n);
      fa.link = carve<uint4>(cur, n);
      fa.hmask = hcap_fast - 1;  // (fa.head, fa.slow: the thread's FastScratch)
      fa.dv = carve<unsigned long long>(cur, n);
      fa.chain = carve<uint4>(cur, n);
      d_gran = carve<unsigned long long>(cur, (size_t)ntiles_tail * kFastCols);
      d_part = carve<uint2>(cur, n);
      d_heavy = carve<uint32_t>(cur, 64 * (((size_t)n + 63) / 64) + ((size_t)n + 63) / 64);
      aa.pv = carve<uint2>(cur, n);
      aa.inp = carve<uint32_t>(cur, n);
      aa.defer = carve<uint2>(cur, n);
      aa.rec = carve<uint4>(cur, 2 * (size_t)n);
      aa.pr = carve<uint2>(cur, n);
    }
    return (size_t)(cur - base);
  };
  const size_t lease1_bytes = layout(nullptr);
  h3c_rt::DeviceLease lease1(dev, lease1_bytes);
  if (!lease1.ok()) return H3C_ERR_HIP;
  layout(lease1.data());
  fa.pc = pc;
  h3c_rt::PinnedLease pin(4096);
  if (!pin.ok()) return H3C_ERR_HIP;
  uint32_t *h_F = reinterpret_cast<uint32_t *>(pin.data());
  uint32_t *d_hF = nullptr;  // the same words as the device addresses them (uio_phaseb_kernel writes them)
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_hF), h_F, 0));
  AuxStream *aux = nullptr;
  int rc = aux_stream(dev, aux);
  if (rc) return rc;
  // The buffers a captured graph of this batch may point into: those its UpdGraphKey names (the
  // caller's tables, the leases, the pinned outcome words, the thread's fast scratch) and the library's
  // constant tables.  Test hook H3C_HOOK_UPD_GRAPHS = 3 leaves lease1 out, so that the audit's refusal
  // path is exercised (every pipeline kernel points into lease1).
  auto allow_of = [&](const void *lease2, size_t lease2_bytes, const void *scratch, size_t scratch_bytes) {
    std::vector<AddrRange> a;
    auto add = [&](const void *p, size_t bytes) {
      if (p && bytes) a.push_back(AddrRange{(uint64_t)(uintptr_t)p, (uint64_t)(uintptr_t)p + bytes});
    };
    add(d_chunks, sizeof(h3c_chunk_state) * (size_t)nchunks);
    add(d_chunks_out, sizeof(h3c_chunk_state) * (size_t)C);
    add(d_ios, sizeof(h3c_update_io) * (size_t)n);
    add(d_res, sizeof(h3c_update_result) * (size_t)n);
    add(d_ctr, 8 * (size_t)kCtrN);
    if (h3c_rt::hook(H3C_HOOK_UPD_GRAPHS) != 3) add(lease1.data(), lease1_bytes);
    add(lease2, lease2_bytes);
    add(d_hF, 4096);
    add(scratch, scratch_bytes);
    add(h3c_rt::device_consts(dev, H3C_TYPE_CRC32C), sizeof(PolyConsts));
    add(h3c_rt::device_consts(dev, H3C_TYPE_CRC32), sizeof(PolyConsts));
    return a;
  };

  StreamDrain drain{st, true};  // every return below waits for both streams before the leases go back
  StreamDrain drain_aux{aux->st, true};
  const uint32_t tb = 256, gb = (uint32_t)((n + tb) / tb);  // n + 1 threads (the scans' extra entry)
  const uint32_t vb = (uint32_t)((std::max<size_t>(n, C) + tb - 1) / tb);
  auto scan_excl = [&](const uint32_t *in, uint32_t *out, hipStream_t q) -> hipError_t {
    size_t t = tmp_bytes;
    return rocprim::exclusive_scan(d_tmp, t, in, out, 0u, (size_t)n + 1, rocprim::plus<uint32_t>(), q);
  };
  uint32_t nofold = 0;  // a redo after a failed A6 knows every verdict: no check moves into the block kernel
  const bool front = front_path;
  const bool pb1 = (h3c_rt::hook(H3C_HOOK_UPD_FRONT) & 2) == 0;  // phase B in one launch (uio_phaseb_kernel)
  // per attempt (fragment arrays for a guessed count, see below)
  uint32_t hcap = 256;
  FragDesc *d_frag = nullptr;
  uint64_t *d_fkey = nullptr;
  uint32_t *d_prev = nullptr, *d_gnext = nullptr, *d_hhead = nullptr, *d_fnext = nullptr;
  // sizes and types per op (a segmented scan), the reference's cases, fragment counts
  auto phase_sizes = [&](hipStream_t q) -> int {
    hipLaunchKernelGGL(uio_sz_elem_kernel, dim3(gb), dim3(tb), 0, q, d_ios, d_order, n, d_status, poly_type, stdf,
                       d_sz);
    HIP_TRY(hipGetLastError());
    {
      size_t t = tmp_bytes;
      HIP_TRY(rocprim::inclusive_scan_by_key(d_tmp, t, d_skey, d_sz, d_szscan, (size_t)n, SzTyOp(),
                                             rocprim::equal_to<uint32_t>(), q));
    }
    hipLaunchKernelGGL(uio_classify_kernel, dim3(gb), dim3(tb), 0, q, d_ios, d_order, d_skey, n, d_chunks, nchunks,
                       d_szscan, d_status, poly_type, stdf, nofold, d_pos, d_nfrag, d_late);
    HIP_TRY(hipGetLastError());
    HIP_TRY(scan_excl(d_nfrag, d_fbase, q));
    return H3C_OK;
  };
  // phase A: validation, payload CRCs + A6 and the INIT CRCs (second stream), sort, and the
  // speculative sizes / cases / fragment counts
  auto phase_a = [&](hipStream_t q) -> int {
    const uint32_t fz_words = front ? ntiles_front * (uint32_t)(sizeof(FrontSlot) / 4) : 0u;
    // one stream on the front path: the prep kernel scans the piece counts itself, the piece pass
    // follows the sort, and the A6 verdicts and t0 come with the front kernel -- no fork and join
    // between streams (each cost ~7-10 us in graph replay: profiles/r03l_*)
    const bool serial = front;
    // (a kernel, not hipMemsetAsync: a memset node at the head of the captured graph was not
    // ordered before the prep kernel in replays -- stale tickets, r03m-r03p)
    if (serial) {
      hipLaunchKernelGGL(uio_zero_kernel, dim3(1), dim3(256), 0, q, d_sstate, 3u + prep_tiles, nullptr, 0u, nullptr,
                         0u, nullptr, 0u);
      HIP_TRY(hipGetLastError());
    }
    // serial: one tile per kPrepTile items (the initialisations beyond them grid-stride), so only
    // the tiles that count toward the last-tile test run
    const uint32_t ptiles = serial ? (uint32_t)(((size_t)n + C + 1 + kPrepTile - 1) / kPrepTile) : prep_tiles;
    hipLaunchKernelGGL(uio_prep_kernel, dim3(ptiles), dim3(kPrepTile), 0, q, d_ios, n, d_chunks, nchunks,
                       poly_type, stdf, exactf, d_status, d_key, d_idx, d_np, d_paycrc0, d_eacc, d_ctr, d_misc, d_a6,
                       reinterpret_cast<uint32_t *>(d_fslot), fz_words, d_hhead, front ? hcap : 0u, d_gnext, d_fnext,
                       front ? cap : 0u, serial ? d_pbase : nullptr, serial ? d_sstate : nullptr, FastArgs{});
    HIP_TRY(hipGetLastError());
    if (serial) {
      size_t t = tmp_bytes;
      HIP_TRY(sort_pairs(d_tmp, t, d_key, d_skey, d_idx, d_order, n, bits, q));
      return h3c_rt::launch_uio_piece_crc(q, dev, poly_type, d_ios, n, d_chunks, nchunks, d_pbase, d_sstate + 2,
                                          d_paycrc0, d_sstate + 3, kPrepTile, d_misc + kMiscErr);
    }
    // second stream, forked here: the piece counts' scan (its own scratch), one piece-CRC pass over
    // the payloads that are not fold candidates and the chunks CRC'd from their bytes (before the
    // block kernel overwrites them), then A6 and t0; this stream sorts the ops and runs the sizes
    // and fragment stages meanwhile.  (With the fold checks in the block kernel the piece pass is
    // short; in round 2, when it carried every payload, the scan ran before the fork.)
    HIP_TRY(hipEventRecord(aux->ready, q));
    HIP_TRY(hipStreamWaitEvent(aux->st, aux->ready, 0));
    {
      size_t t = pscan_tmp;
      HIP_TRY(rocprim::exclusive_scan(d_ptmp, t, d_np, d_pbase, 0u, NP + 1, rocprim::plus<uint32_t>(), aux->st));
    }
    // The ops' sort alone on this stream: its latency-bound passes took ~70 us beside the
    // bandwidth-bound payload-CRC kernel and ~12 us before it (profiles/r02_updio_sort_first_ab.txt)
    {
      size_t t = tmp_bytes;
      HIP_TRY(sort_pairs(d_tmp, t, d_key, d_skey, d_idx, d_order, n, bits, q));
    }
    int r = h3c_rt::launch_uio_piece_crc(aux->st, dev, poly_type, d_ios, n, d_chunks, nchunks, d_pbase, d_pbase + NP,
                                         d_paycrc0, nullptr, 0u, d_misc + kMiscErr);
    if (r) return r;
    hipLaunchKernelGGL(uio_verify_t0_kernel, dim3(vb), dim3(tb), 0, aux->st, d_ios, n, d_chunks, nchunks, poly_type,
                       exactf, stdf, d_paycrc0, pc, d_status, d_payraw, d_a6, d_misc, d_t0, d_chunks_out, 1u);
    HIP_TRY(hipGetLastError());
    if (front) {  // the sizes, cases, late A6 checks and fragments come in one launch (phase_frag)
      HIP_TRY(hipEventRecord(aux->done, aux->st));
      return H3C_OK;
    }
    r = phase_sizes(q);  // speculative: every A6 check passes (joined before the block kernel)
    if (r) return r;
    // second stream, after the cases are known: the late pass over the fold candidates that
    // were not folded (each one piece), beside the fragment stage
    HIP_TRY(hipEventRecord(aux->ready, q));
    HIP_TRY(hipStreamWaitEvent(aux->st, aux->ready, 0));
    {
      size_t t = tmp_bytes;
      HIP_TRY(rocprim::exclusive_scan(d_tmp, t, d_late, d_lbase, 0u, (size_t)n + 1, rocprim::plus<uint32_t>(),
                                      aux->st));
    }
    r = h3c_rt::launch_uio_piece_crc(aux->st, dev, poly_type, d_ios, n, d_chunks, 0, d_lbase, d_lbase + n,
                                     d_paycrc0, nullptr, 0u, d_misc + kMiscErr);
    if (r) return r;
    hipLaunchKernelGGL(uio_late_verify_kernel, dim3(gb), dim3(tb), 0, aux->st, d_ios, n, d_late, d_paycrc0, pc, stdf,
                       d_status, d_payraw, d_a6, d_misc);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(aux->done, aux->st));
    return H3C_OK;
  };

  // ---- the fast branch: zero, prep (with the fast tables), [piece pass: exact mode's chunk CRCs],
  // uio_fast_kernel -- four launches at most, one graph on request.  An op that does not qualify makes
  // uio_fast_kernel return at once (nothing written); the general pipeline below then runs the batch.
  // the thread's fast scratch (the slow word, the control words, granules and bucket heads): zero between
  // batches where the branches need it so; a new, suspect or re-laid-out scratch, or one whose aligned epochs
  // are about to wrap, is zeroed here, before the batch and outside any capture
  FastScratch *fsc = nullptr;
  if (try_aligned || try_fast) {
    fsc = fast_scratch(dev, kScratchHeads + 3 * (size_t)hcap_fast);
    if (!fsc) return H3C_ERR_HIP;
    if (fsc->hcap != hcap_fast || fsc->abatches >= kAEpochBatches) fsc->dirty = true;
    fa.slow = fsc->p;
    fa.head = fsc->p + kScratchHeads;
    aa.ctl = fsc->p + kScratchACtl;
    aa.gran = reinterpret_cast<unsigned long long *>(fsc->p + kScratchAGran);
    aa.stat = fsc->p + kScratchAStat;
    aa.head = fsc->p + kScratchHeads + hcap_fast;
    aa.hand = fsc->p + kScratchHeads + 2 * (size_t)hcap_fast;  // (hcap_fast >= 2n)
    aa.hmask = hcap_fast - 1;
    aa.key = fa.key;
    aa.link = fa.link;
    aa.dv = fa.dv;
    if (fsc->dirty) {
      const uint32_t zw = kScratchHeads + 3 * hcap_fast, zg = std::min(1024u, (zw + 1023) / 1024);
      // (the aligned range weights are kept across a re-zeroing: they describe the device, not the batches)
      const uint32_t w0 = fsc->fresh ? zw : kScratchACtl + kAW, w1 = fsc->fresh ? zw : kScratchACtl + kAW + kAClasses;
      hipLaunchKernelGGL(uio_zero_kernel, dim3(zg), dim3(256), 0, st, fsc->p, w0, fsc->p + w1, zw - w1, nullptr, 0u,
                         nullptr, 0u);
      HIP_TRY(hipGetLastError());
      fsc->dirty = false;
      fsc->fresh = false;
      fsc->hcap = hcap_fast;
      fsc->abatches = 0;
    }
  }
  uint32_t *h_fs = &h_F[kMiscFast - kMiscOutF];  // the outcome word, set last by the branches' last kernel

  // ---- the aligned sub-branch: uio_aprep_kernel + uio_afused_kernel, one graph on request ----
  if (try_aligned) {
    ScratchGuard sguard{fsc};  // (any return before the batch's outcome is read marks it suspect)
    const uint32_t num_cu = (uint32_t)std::max(1, h3c_rt::device_num_cu(dev));
    // the fewest workgroups that keep the most ops per wave (as upd_fused_kernel's grid)
    uint32_t nwg_a = std::min<uint32_t>(std::min(num_cu, kAGranRows), std::max<uint32_t>(1, (n + kBlkWaves - 1) / kBlkWaves));
    {
      const uint64_t per = ((uint64_t)n + (uint64_t)nwg_a * kBlkWaves - 1) / ((uint64_t)nwg_a * kBlkWaves);
      nwg_a = (uint32_t)std::max<uint64_t>(1, ((uint64_t)n + per * kBlkWaves - 1) / (per * kBlkWaves));
    }
    // (test hook H3C_HOOK_UPD_GIVEUP bit 3: ticket 1 gives up its look-back; bit 4: the pass reports itself void)
    const uint32_t force_void = ((giveup & 8) ? 1u : 0u) | ((giveup & 16) ? 2u : 0u);
    aa.crc0 = exact ? d_paycrc0 + n : nullptr;
    auto a_launch = [&](hipStream_t q) -> int {
      if (exact) {  // t0 from the bytes: the chunks' CRCs before uio_afused_kernel writes them
        hipLaunchKernelGGL(uio_apiece_kernel, dim3(1), dim3(64), 0, q, d_chunks, nchunks, poly_type, d_pbase,
                           d_sstate + 2, d_paycrc0 + n);
        HIP_TRY(hipGetLastError());
        const int r = h3c_rt::launch_uio_piece_crc(q, dev, poly_type, d_ios, 0u, d_chunks, nchunks, d_pbase, d_sstate + 2,
                                                   d_paycrc0 + n, nullptr, kPrepTile, d_misc + kMiscErr);
        if (r) return r;
      }
      hipLaunchKernelGGL(uio_aprep_kernel, dim3((n + kATile - 1) / kATile + 1), dim3(kATile), 0, q, d_ios, n, d_chunks,
                         nchunks, poly_type, stdf, d_misc, d_ctr, aa);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_afused_kernel, dim3(nwg_a), dim3(kBlkThreads), 0, q, d_ios, n, d_chunks, d_chunks_out,
                         nchunks, poly_type, stdf, pc, aa, d_misc, d_res, d_ctr, d_hF, commit_dev, force_void);
      HIP_TRY(hipGetLastError());
      return H3C_OK;
    };
    const UpdGraphKey akey{dev, poly_type, flags | 0x40000000u, n, nchunks, 0u, hcap_fast, d_chunks, d_chunks_out,
                           d_ios, d_res, d_ctr, lease1.data(), fsc->p, d_hF, nullptr};
    UpdGraphs *gr = upd_graphs(akey, st, (flags & H3C_UPD_GRAPHS) != 0);
    if (gr && !gr->g && !gr->failed) {
      hipStream_t cst = capture_stream(dev);
      rc = cst ? capture_graph(cst, [&] {
        int r = a_launch(cst);
        if (!r && epi_graph && !commit_dev) r = epilogue(cst, d_misc + kMiscOutF, cap);
        return r;
      }, gr->g, allow_of(nullptr, 0, fsc->p, 4 * fsc->words)) : H3C_ERR_HIP;
      g_graph_stats[rc ? kDiagCaptureFail : kDiagCapture].fetch_add(1);
      if (rc) {
        gr->failed = true;
        (void)hipGetLastError();
      }
      rc = H3C_OK;
    }
    const bool use_graph = gr && gr->g && !gr->failed;
    __atomic_store_n(h_fs, 0u, __ATOMIC_RELAXED);
    const auto t_launch = std::chrono::steady_clock::now();
    t_host.launch0 = t_launch;
    if (use_graph) {
      HIP_TRY(hipGraphLaunch(gr->g, st));
      g_graph_stats[kDiagReplay].fetch_add(1);
    } else {
      rc = a_launch(st);
      if (rc) return rc;
    }
    t_host.launched = std::chrono::steady_clock::now();
    if (!(use_graph && epi_graph) && !commit_dev) {
      rc = epilogue(st, d_misc + kMiscOutF, cap);
      if (rc) return rc;
    }
    const uint32_t poll_us = fast_poll_budget_us(fpred->last_us);
    const bool seen = poll_host_word(h_fs, poll_us);
    t_host.seen = std::chrono::steady_clock::now();
    if (seen)
      fpred->last_us = (uint32_t)std::max<int64_t>(
          1, std::chrono::duration_cast<std::chrono::microseconds>(t_host.seen - t_launch).count());
    else
      fpred->last_us = 0;
    auto prof_aligned = [&]() {  // the fused kernel's own wall-clock span (first workgroup start, last end)
      if (!h3c_rt::prof_enabled()) return;
      uint64_t t0, t1;
      std::memcpy(&t0, h_F + (kMiscT0 - kMiscOutF), 8);
      std::memcpy(&t1, h_F + (kMiscT1 - kMiscOutF), 8);
      const int khz = h3c_rt::device_wall_clock_khz(dev);
      if (t1 > t0 && khz > 0) h3c_rt::prof_add(H3C_PROF_UPDIO, (float)((double)(t1 - t0) / khz), 3ull * kBlk * n);
    };
    if (seen && commit_dev && *h_fs == kFastDone && !h_F[kMiscErr - kMiscOutF]) {
      // done on the device-table entry: the last workgroup committed the states and wrote every output before
      // the outcome word (see the fast branch below for why the call need not wait for the stream)
      prof_aligned();
      g_graph_stats[kDiagFast].fetch_add(1);
      g_graph_stats[kDiagAligned].fetch_add(1);
      fpred->aslow = 0;
      ++fsc->abatches;
      sguard.f = nullptr;
      drain.armed = drain_aux.armed = false;
      return H3C_OK;
    }
    const hipError_t se = stream_wait(st, seen ? std::min(poll_us, 200u) : 0u);
    if (se != hipSuccess) {
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error("h3c_update_ios (aligned branch)", se);
      return H3C_ERR_HIP;
    }
    const uint32_t fs = h_F[kMiscFast - kMiscOutF];
    if (fs != kFastDone && fs != kFastVoid && fs != kFastAbort) {
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error_text("h3c_update_ios: the aligned branch ended without an outcome");
      return H3C_ERR_HIP;
    }
    sguard.f = nullptr;  // (the last workgroup reset the control words and advanced the epoch)
    ++fsc->abatches;
    if (fs == kFastDone || fs == kFastVoid) {
      prof_aligned();
      g_graph_stats[kDiagFast].fetch_add(1);
      g_graph_stats[kDiagAligned].fetch_add(1);
      fpred->aslow = 0;
      if (fs == kFastVoid) {  // an A6 failure, a deferred block or a look-back that gave up: results from the records
        g_graph_stats[kDiagAlignedFix].fetch_add(1);
        hipLaunchKernelGGL(uio_afix_kernel, dim3(1), dim3(1024), 0, st, d_ios, n, d_chunks, d_chunks_out, nchunks,
                           poly_type, stdf, pc, aa, d_misc, d_res, d_ctr, commit_dev);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(h_F, d_misc + kMiscOutF, 4 * (kMiscN - kMiscOutF), hipMemcpyDeviceToHost, st));
        if (!commit_dev) {
          rc = epilogue(st, d_misc + kMiscOutF, cap);
          if (rc) return rc;
        }
        const hipError_t se2 = hipStreamSynchronize(st);
        if (se2 != hipSuccess) {
          drain.armed = drain_aux.armed = false;
          h3c_rt::set_error("h3c_update_ios (aligned-branch recovery)", se2);
          return H3C_ERR_HIP;
        }
      }
      drain.armed = drain_aux.armed = false;
      return H3C_OK;
    }
    // kFastAbort: some op is not a full aligned block write -- the chain-based fast branch (or the general
    // pipeline) runs the batch from the original tables
    g_graph_stats[kDiagAlignedAbort].fetch_add(1);
    fpred->aslow = 1;
    fpred->a_runs = 0;
  } else if (fpred) {
    ++fpred->a_runs;
  }

  if (try_fast) {
    const uint32_t ptiles_f = (uint32_t)(((size_t)n + C + 1 + kPrepTile - 1) / kPrepTile);
    ScratchGuard sguard{fsc};  // (any return before the batch's outcome is read marks it suspect)
    unsigned long long *d_ts = reinterpret_cast<unsigned long long *>(d_misc + kMiscT0);
    auto fast_kernel = [&](hipStream_t q, bool timed) -> int {
      hipLaunchKernelGGL(uio_fast_kernel, dim3(nwg_fast), dim3(kBlkThreads), 0, q, n, stdf, pc, fa.frag, fa.chain,
                         fa.dv, fa.slow, timed ? d_ts : nullptr, fa.key, fa.head, fa.hmask,
                         d_heavy, d_heavy + 64 * (((size_t)n + 63) / 64));
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_fast_sum_kernel, dim3(ntiles_tail), dim3(kTailTile), 0, q, n, pc, fa.frag, fa.key, fa.dv,
                         fa.slow, fa.head, fa.hmask, d_gran, d_part, d_misc + kMiscErr);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_fast_res_kernel, dim3(ntiles_tail), dim3(kTailTile), 0, q, d_chunks, d_chunks_out,
                         nchunks, n, poly_type, stdf, exactf, d_paycrc0 + n, pc, d_gran, d_part, d_misc, fa.slow,
                         d_res, d_ctr, d_hF, (giveup & 4) ? 1u : 0u, commit_dev);
      HIP_TRY(hipGetLastError());
      return H3C_OK;
    };
    auto fast_front = [&](hipStream_t q) -> int {  // [zero: exact mode's scan states], prep, [piece pass], link
      if (exact) {
        hipLaunchKernelGGL(uio_zero_kernel, dim3(1), dim3(256), 0, q, d_sstate, 3u + prep_tiles, nullptr, 0u, nullptr,
                           0u, nullptr, 0u);
        HIP_TRY(hipGetLastError());
      }
      hipLaunchKernelGGL(uio_prep_kernel, dim3(ptiles_f), dim3(kPrepTile), 0, q, d_ios, n, d_chunks, nchunks, poly_type,
                         stdf, exactf, d_status, d_key, d_idx, d_np, d_paycrc0, d_eacc, d_ctr, d_misc, d_a6, nullptr, 0u,
                         nullptr, 0u, nullptr, nullptr, 0u, exact ? d_pbase : nullptr, exact ? d_sstate : nullptr, fa);
      HIP_TRY(hipGetLastError());
      if (exact) {  // the chunks' CRCs before uio_fast_kernel writes them (t0 from the bytes)
        const int r = h3c_rt::launch_uio_piece_crc(q, dev, poly_type, d_ios, n, d_chunks, nchunks, d_pbase,
                                                   d_sstate + 2, d_paycrc0, d_sstate + 3, kPrepTile, d_misc + kMiscErr);
        if (r) return r;
      }
      hipLaunchKernelGGL(uio_fast_link_kernel, dim3((n + 255) / 256), dim3(256), 0, q, fa.link, fa.key, fa.head,
                         fa.hmask, n, fa.slow, fa.chain, d_ios, d_chunks, nchunks, poly_type, stdf, pc, fa.frag,
                         d_heavy, d_heavy + 64 * (((size_t)n + 63) / 64));
      HIP_TRY(hipGetLastError());
      return H3C_OK;
    };
    const UpdGraphKey fkey{dev, poly_type, flags | 0x80000000u, n, nchunks, 0u, hcap_fast, d_chunks, d_chunks_out,
                           d_ios, d_res, d_ctr, lease1.data(), fsc->p, d_hF, nullptr};
    UpdGraphs *gr = upd_graphs(fkey, st, (flags & H3C_UPD_GRAPHS) != 0);
    if (gr && !gr->g && !gr->failed) {
      hipStream_t cst = capture_stream(dev);
      rc = cst ? capture_graph(cst, [&] {
        int r = fast_front(cst);
        if (!r) r = fast_kernel(cst, true);
        if (!r && epi_graph && !commit_dev) r = epilogue(cst, d_misc + kMiscOutF, cap);
        return r;
      }, gr->g, allow_of(nullptr, 0, fsc->p, 4 * fsc->words)) : H3C_ERR_HIP;
      g_graph_stats[rc ? kDiagCaptureFail : kDiagCapture].fetch_add(1);
      if (rc) {
        gr->failed = true;
        (void)hipGetLastError();
      }
      rc = H3C_OK;
    }
    const bool use_graph = gr && gr->g && !gr->failed;
    __atomic_store_n(h_fs, 0u, __ATOMIC_RELAXED);
    const auto t_launch = std::chrono::steady_clock::now();
    if (use_graph) {
      HIP_TRY(hipGraphLaunch(gr->g, st));
      g_graph_stats[kDiagReplay].fetch_add(1);
    } else {
      rc = fast_front(st);
      if (rc) return rc;
      rc = fast_kernel(st, true);  // (timed by its own wall-clock stamps: an abandoned attempt counts nothing)
      if (rc) return rc;
    }
    if (!(use_graph && epi_graph) && !commit_dev) {
      rc = epilogue(st, d_misc + kMiscOutF, cap);
      if (rc) return rc;
    }
    // the outcome word polled for up to kFastPollUs before the blocking synchronisation: a blocking wait
    // that starts while the batch runs wakes ~10-20 us after it ends
    const uint32_t poll_us = fast_poll_budget_us(fpred->last_us);
    const bool seen = poll_host_word(h_fs, poll_us);
    if (seen)
      fpred->last_us = (uint32_t)std::max<int64_t>(
          1, std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t_launch).count());
    else
      fpred->last_us = 0;  // (unknown: the next batch of the shape spins up to the default bound)
    if (seen && commit_dev && *h_fs == kFastDone && !h_F[kMiscErr - kMiscOutF]) {
      // The device-table entry, done on the fast branch: the tail has committed the states and written
      // every output before the outcome word, and no further work of this call follows, so the call
      // returns without waiting for the stream's completion signal (~13 us after the last kernel ends,
      // profiles/r04_updio_host_timeline.txt).  Later work on `stream` is ordered after the batch; other
      // streams order themselves on an event recorded on `stream`, as for any enqueued work (h3c_crc.h).
      // (No hipStreamQuery here: one call took ~7 us; a fault would have kept the outcome word unset.)
      if (h3c_rt::prof_enabled()) {
        uint64_t t0, t1;
        std::memcpy(&t0, h_F + (kMiscT0 - kMiscOutF), 8);
        std::memcpy(&t1, h_F + (kMiscT1 - kMiscOutF), 8);
        const int khz = h3c_rt::device_wall_clock_khz(dev);
        if (t1 > t0 && khz > 0) h3c_rt::prof_add(H3C_PROF_UPDIO, (float)((double)(t1 - t0) / khz), 3ull * kBlk * n);
      }
      g_graph_stats[kDiagFast].fetch_add(1);
      fpred->slow = 0;
      sguard.f = nullptr;
      drain.armed = drain_aux.armed = false;
      return H3C_OK;
    }
    const hipError_t se = stream_wait(st, seen ? std::min(poll_us, 200u) : 0u);  // (unseen: spun long enough)
    if (se != hipSuccess) {
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error("h3c_update_ios (fast branch)", se);
      return H3C_ERR_HIP;
    }
    const uint32_t fs = h_F[kMiscFast - kMiscOutF];
    if (h_F[kMiscErr - kMiscOutF]) {
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error_text("h3c_update_ios: a piece table disagrees with its items (corrupt scratch)");
      return H3C_ERR_HIP;
    }
    sguard.f = nullptr;  // the tail ran to its outcome: the scratch is clean again
    if (fs == kFastDone || fs == kFastVoid) {
      if (h3c_rt::prof_enabled()) {  // the kernel's own wall-clock span (hipEvents carry no time in a graph)
        uint64_t t0, t1;
        std::memcpy(&t0, h_F + (kMiscT0 - kMiscOutF), 8);
        std::memcpy(&t1, h_F + (kMiscT1 - kMiscOutF), 8);
        const int khz = h3c_rt::device_wall_clock_khz(dev);
        if (t1 > t0 && khz > 0) h3c_rt::prof_add(H3C_PROF_UPDIO, (float)((double)(t1 - t0) / khz), 3ull * kBlk * n);
      }
      g_graph_stats[kDiagFast].fetch_add(1);
      fpred->slow = 0;
      if (fs == kFastVoid) {  // a workgroup gave up waiting: the bytes and deltas are complete, the results not
        g_graph_stats[kDiagFastVoid].fetch_add(1);
        hipLaunchKernelGGL(uio_fast_recover_kernel, dim3(1), dim3(1024), 0, st, d_chunks, d_chunks_out, nchunks, n,
                           poly_type, stdf, exactf, d_paycrc0 + n, pc, fa, d_misc, d_res, d_ctr);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(h_F, d_misc + kMiscOutF, 4 * (kMiscN - kMiscOutF), hipMemcpyDeviceToHost, st));
        rc = epilogue(st, d_misc + kMiscOutF, cap);
        if (rc) return rc;
        const hipError_t se2 = hipStreamSynchronize(st);
        if (se2 != hipSuccess || h_F[kMiscErr - kMiscOutF]) {
          drain.armed = drain_aux.armed = false;
          if (se2 != hipSuccess) h3c_rt::set_error("h3c_update_ios (fast-branch recovery)", se2);
          else h3c_rt::set_error_text("h3c_update_ios: fast-branch recovery found an op with no delta");
          return H3C_ERR_HIP;
        }
      }
      drain.armed = drain_aux.armed = false;
      return H3C_OK;
    }
    // kFastAbort: some op does not qualify -- the general pipeline runs the batch
    g_graph_stats[kDiagFastAbort].fetch_add(1);
    fpred->slow = 1;
    fpred->general_runs = 0;
  }
  if (fpred) ++fpred->general_runs;

  // ---- fragments, blocks, scans, results (redone once if the fragment guess was short) ----
  for (int attempt = 0;; ++attempt) {
    hcap = 256;
    while (hcap < cap) hcap <<= 1;
    auto layout2 = [&](char *base) -> size_t {
      char *c2 = base;
      d_frag = carve<FragDesc>(c2, cap);
      d_fkey = carve<uint64_t>(c2, cap);
      d_prev = carve<uint32_t>(c2, cap);
      d_gnext = carve<uint32_t>(c2, cap);
      d_fnext = carve<uint32_t>(c2, cap);
      d_hhead = carve<uint32_t>(c2, hcap);
      return (size_t)(c2 - base);
    };
    const size_t lease2_bytes = layout2(nullptr);
    h3c_rt::DeviceLease lease2(dev, lease2_bytes);
    if (!lease2.ok()) return H3C_ERR_HIP;
    StreamDrain drain2{st, true};
    layout2(lease2.data());
    const uint32_t *d_F = d_fbase + n;
    const uint32_t fb = (cap + tb - 1) / tb;
    auto phase_frag = [&](hipStream_t q) -> int {  // fragments and their chains
      if (front && attempt == 0) {
        hipLaunchKernelGGL(uio_front_kernel, dim3(std::max(ntiles_front, 1u)), dim3(kFrontTile), 0, q, d_ios, d_order,
                           d_skey, n, d_chunks, nchunks, d_status, poly_type, stdf, pc, d_pos, d_nfrag, d_fbase,
                           d_late, d_payraw, d_a6, d_misc, d_frag, d_fkey, cap, d_hhead, hcap - 1, d_gnext, d_prev,
                           d_fnext, d_fslot, d_paycrc0, exactf, d_t0, d_chunks_out,
                           d_sstate, giveup & 1u);
        HIP_TRY(hipGetLastError());
        return H3C_OK;
      }
      if (attempt) HIP_TRY(hipMemsetAsync(d_ctr, 0, 8 * kCtrN, q));  // the first attempt's counters
      hipLaunchKernelGGL(uio_frag_kernel, dim3((std::max(cap, hcap) + tb - 1) / tb), dim3(tb), 0, q, d_pos, d_fbase,
                         n, cap, d_ios, d_skey, d_chunks, d_frag, d_fkey, pc, d_hhead, hcap, stdf, d_payraw, d_fnext);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_tlink_kernel, dim3((cap + kLinkTile - 1) / kLinkTile), dim3(kLinkTile), 0, q, d_fkey,
                         d_F, cap, d_hhead, hcap - 1, d_gnext, d_prev);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_resolve_kernel, dim3(fb), dim3(tb), 0, q, d_fkey, d_F, cap, d_hhead, hcap - 1, d_gnext,
                         d_prev);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_heads_kernel, dim3(fb), dim3(tb), 0, q, d_prev, d_F, cap, d_frag, d_fnext);
      HIP_TRY(hipGetLastError());
      if (attempt == 0) {  // the A6 verdicts (the block kernel reads the flag) and t0
        HIP_TRY(hipStreamWaitEvent(q, aux->done, 0));
      }
      return H3C_OK;
    };
    auto phase_b_scans = [&](hipStream_t q) -> int {  // t' per op, then s' per op (two affine scans by chunk), results
      hipLaunchKernelGGL(uio_elem_kernel<TMapFn>, dim3(gb), dim3(tb), 0, q, TMapFn{d_pos, d_eacc, d_payraw, pc, d_a6},
                         n, d_tel);
      HIP_TRY(hipGetLastError());
      {
        size_t t = tmp_bytes;
        HIP_TRY(rocprim::inclusive_scan_by_key(d_tmp, t, d_skey, d_tel, d_tscan, (size_t)n, AffOp{poly},
                                               rocprim::equal_to<uint32_t>(), q));
      }
      hipLaunchKernelGGL(uio_elem_kernel<SMapFn>, dim3(gb), dim3(tb), 0, q,
                         SMapFn{d_pos, d_skey, nchunks, d_tscan, d_t0, d_eacc, d_payraw, pc, d_a6}, n, d_sel);
      HIP_TRY(hipGetLastError());
      {
        size_t t = tmp_bytes;
        HIP_TRY(rocprim::inclusive_scan_by_key(d_tmp, t, d_skey, d_sel, d_sscan, (size_t)n, AffOp{poly},
                                               rocprim::equal_to<uint32_t>(), q));
      }
      hipLaunchKernelGGL(uio_result_kernel, dim3(gb), dim3(tb), 0, q, d_pos, d_skey, n, d_sscan, d_chunks,
                         d_chunks_out, nchunks, d_t0, poly_type, stdf, poly, d_res, d_ctr, d_F, d_misc, d_a6);
      HIP_TRY(hipGetLastError());
      return H3C_OK;
    };
    auto phase_b = [&](hipStream_t q) -> int {
      if (pb1) {
        hipLaunchKernelGGL(uio_phaseb_kernel, dim3(std::max(ntiles_pb, 1u)), dim3(kPhaseBTile), 0, q, d_pos, d_skey, n,
                           d_eacc, d_payraw, pc, d_a6, d_t0, d_chunks, d_chunks_out, nchunks, poly_type, stdf, d_res,
                           d_ctr, d_F, d_misc, reinterpret_cast<PhaseBSlot *>(d_pbz), d_pbz + pbz_words - 1,
                           d_hF, (giveup >> 1) & 1u);
        HIP_TRY(hipGetLastError());
      } else {
        const int r = phase_b_scans(q);
        if (r) return r;
      }
      if (exact && nchunks) {
        hipLaunchKernelGGL(uio_stale_kernel, dim3((nchunks + tb - 1) / tb), dim3(tb), 0, q, d_chunks, nchunks, d_t0,
                           poly_type, stdf, d_ctr);
        HIP_TRY(hipGetLastError());
      }
      return H3C_OK;
    };
    // The first attempt runs as one HIP graph when this thread has seen the same batch shape and
    // buffers before (the lease pools hand a steady caller the same ones): ~30 launches and the
    // block kernel become one launch, and the short kernels run back to back instead of at the
    // host's launch rate.  The block kernel times itself there (wall clock).  (Two
    // graphs with the block kernel launched between them cost ~30 us more per config-3 batch:
    // the kernel after a multi-stream graph started ~24 us after the graph's last node,
    // profiles/r02_updio_one_graph_ab.txt.)
    const uint32_t blocks = (uint32_t)std::max(1, h3c_rt::device_num_cu(dev));
    auto block_kernel = [&](hipStream_t q, bool timed) -> int {
      hipLaunchKernelGGL(uio_block_kernel, dim3(blocks), dim3(kBlkThreads), 0, q, d_frag, d_fnext, d_F, cap, pc, d_eacc, d_misc,
                         timed ? reinterpret_cast<unsigned long long *>(d_misc + kMiscT0) : nullptr, stdf, d_payraw,
                         d_a6, d_pbz, pbz_words, d_misc);
      HIP_TRY(hipGetLastError());
      return H3C_OK;
    };
    // algorithmic bytes, per op: a 4 KiB block read and written once plus 4 KiB of new bytes
    // (exact for BASELINE config 3's block-aligned 4 KiB writes; bench.py states the unit)
    const uint64_t alg_bytes = 3ull * kBlk * n;
    UpdGraphs *gr = nullptr;
    if (attempt == 0) {
      const UpdGraphKey key{dev, poly_type, flags, n, nchunks, cap, hcap, d_chunks, d_chunks_out, d_ios, d_res,
                            d_ctr, lease1.data(), lease2.data(), d_hF, aux->st};
      gr = upd_graphs(key, st, (flags & H3C_UPD_GRAPHS) != 0);
    }
    if (gr && !gr->g && !gr->failed) {  // capture the attempt once, on a capture stream of this thread
      hipStream_t cst = capture_stream(dev);
      rc = cst ? capture_graph(cst, [&] {
        int r = phase_a(cst);
        if (!r) r = phase_frag(cst);
        if (!r) r = block_kernel(cst, true);
        if (!r) r = phase_b(cst);
        if (!r && epi_graph) r = epilogue(cst, d_misc + kMiscOutF, cap);
        return r;
      }, gr->g, allow_of(lease2.data(), lease2_bytes, nullptr, 0)) : H3C_ERR_HIP;
      if (rc) {  // not capturable here: plain launches from now on for this shape
        gr->failed = true;
        (void)hipGetLastError();
        g_graph_stats[kDiagCaptureFail].fetch_add(1);
      } else {
        g_graph_stats[kDiagCapture].fetch_add(1);
      }
      rc = H3C_OK;
    }
    const bool use_graph = gr && gr->g && !gr->failed;
    if (use_graph) {
      HIP_TRY(hipGraphLaunch(gr->g, st));
      g_graph_stats[kDiagReplay].fetch_add(1);
    } else {
      if (attempt == 0) {
        rc = phase_a(st);
        if (rc) return rc;
      }
      rc = phase_frag(st);
      if (rc) return rc;
      h3c_rt::ProfToken tok;
      HIP_TRY(h3c_rt::prof_begin(st, tok));
      rc = block_kernel(st, false);
      if (rc) return rc;
      HIP_TRY(h3c_rt::prof_end(st, tok, H3C_PROF_UPDIO, alg_bytes));
      rc = phase_b(st);
      if (rc) return rc;
    }
    const bool prof_graph = use_graph && h3c_rt::prof_enabled();
    if (!pb1)  // (uio_phaseb_kernel's last tile writes the outcome words to h_F itself)
      HIP_TRY(hipMemcpyAsync(h_F, d_misc + kMiscOutF, 4 * (kMiscN - kMiscOutF), hipMemcpyDeviceToHost, st));
    if (!(use_graph && epi_graph)) {
      rc = epilogue(st, d_misc + kMiscOutF, cap);  // (a redone attempt's outputs are replaced)
      if (rc) return rc;
    }
    const hipError_t se = hipStreamSynchronize(st);
    drain2.armed = false;
    if (se != hipSuccess) {
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error("h3c_update_ios", se);
      return H3C_ERR_HIP;
    }
    if (prof_graph) {  // the in-graph block kernel's own wall-clock span (hipEvents are not timed in a graph)
      uint64_t t0, t1;
      std::memcpy(&t0, h_F + (kMiscT0 - kMiscOutF), 8);
      std::memcpy(&t1, h_F + (kMiscT1 - kMiscOutF), 8);
      const int khz = h3c_rt::device_wall_clock_khz(dev);
      if (t1 > t0 && khz > 0) h3c_rt::prof_add(H3C_PROF_UPDIO, (float)((double)(t1 - t0) / khz), alg_bytes);
    }
    if (h_F[kMiscPBVoid - kMiscOutF] && h_F[0] <= cap && !h_F[1]) {
      g_graph_stats[kDiagPBVoid].fetch_add(1);
      // a phase-B tile gave up waiting (its CU starved by other work): the chunk bytes are
      // written and right; redo phase B the scan-based way over the same state, then the epilogue
      HIP_TRY(hipMemsetAsync(d_ctr, 0, 8 * kCtrN, st));
      HIP_TRY(hipMemsetAsync(d_misc + kMiscPBVoid, 0, 4, st));  // (the epilogue below commits)
      rc = phase_b_scans(st);
      if (rc) return rc;
      if (exact && nchunks) {
        hipLaunchKernelGGL(uio_stale_kernel, dim3((nchunks + tb - 1) / tb), dim3(tb), 0, st, d_chunks, nchunks, d_t0,
                           poly_type, stdf, d_ctr);
        HIP_TRY(hipGetLastError());
      }
      HIP_TRY(hipMemcpyAsync(h_F, d_misc + kMiscOutF, 4 * (kMiscN - kMiscOutF), hipMemcpyDeviceToHost, st));
      rc = epilogue(st, d_misc + kMiscOutF, cap);
      if (rc) return rc;
      const hipError_t se2 = hipStreamSynchronize(st);
      if (se2 != hipSuccess) {
        drain.armed = drain_aux.armed = false;
        h3c_rt::set_error("h3c_update_ios", se2);
        return H3C_ERR_HIP;
      }
    }
    if (h_F[kMiscErr - kMiscOutF]) {
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error_text("h3c_update_ios: a piece table disagrees with its items (corrupt scratch)");
      return H3C_ERR_HIP;
    }
    const uint32_t F = h_F[0], a6_failed = h_F[1];
    const bool void_pass = (a6_failed & kMiscVoid) != 0;  // a front tile gave up waiting: F means nothing
    if (!void_pass) last_frags = F;
    if (F <= cap && !a6_failed) break;
    // a redo: counted by its cause (h3c_diag_counter 3, 5, 6)
    g_graph_stats[void_pass ? kDiagFrontVoid : (a6_failed & 1u) ? kDiagA6Redo : kDiagShortF].fetch_add(1);
    if (attempt >= 2) {  // cannot happen: a redo knows the verdicts, and the count after the first redo
      drain.armed = drain_aux.armed = false;
      h3c_rt::set_error_text("h3c_update_ios: fragment count changed between attempts");
      return H3C_ERR_HIP;
    }
    // nothing was written (no chain ran): redo on the scan-based stage, with the count known and,
    // after a failed A6 (or a void front pass), the sizes / cases / fragment counts recomputed from
    // the real verdicts (F can only shrink).  A failed A6 came from the piece passes or the late
    // checks; the fold candidates' own checks never ran, so every typed WRITE is checked again
    // first and the redo moves no check into the block kernel.
    if (!void_pass) cap = std::max(cap, F);
    if (a6_failed) {
      hipLaunchKernelGGL(uio_redo_pieces_kernel, dim3((uint32_t)((NP + 1 + tb - 1) / tb)), dim3(tb), 0, st, d_ios, n,
                         (uint32_t)NP, d_status, d_np, d_paycrc0);
      HIP_TRY(hipGetLastError());
      {
        size_t t = tmp_bytes;
        HIP_TRY(rocprim::exclusive_scan(d_tmp, t, d_np, d_pbase, 0u, NP + 1, rocprim::plus<uint32_t>(), st));
      }
      rc = h3c_rt::launch_uio_piece_crc(st, dev, poly_type, d_ios, n, d_chunks, nchunks, d_pbase, d_pbase + NP,
                                        d_paycrc0, nullptr, 0u, d_misc + kMiscErr);
      if (rc) return rc;
      hipLaunchKernelGGL(uio_verify_t0_kernel, dim3(vb), dim3(tb), 0, st, d_ios, n, d_chunks, nchunks, poly_type,
                         exactf, stdf, d_paycrc0, pc, d_status, d_payraw, d_a6, d_misc, d_t0, d_chunks_out, 0u);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(uio_merge_a6_kernel, dim3(gb), dim3(tb), 0, st, d_a6, n, d_status, d_misc);
      HIP_TRY(hipGetLastError());
      nofold = 1;
      rc = phase_sizes(st);
      if (rc) return rc;
    }
  }
  drain.armed = drain_aux.armed = false;
  return H3C_OK;
}

bool valid_update_args(uint8_t poly_type, const void *chunks, uint32_t nchunks, const void *ios, uint32_t n,
                       const void *results) {
  if (poly_type != H3C_TYPE_CRC32C && poly_type != H3C_TYPE_CRC32) return false;
  return !((n && (!ios || !results)) || (nchunks && !chunks) || n >= 0x7FFFFFFFu || nchunks >= (1u << 28));
}

void counters_from(const unsigned long long *h, h3c_update_counters *c) {
  c->none = h[kCtrNone];
  c->reuse = h[kCtrReuse];
  c->combine = h[kCtrCombine];
  c->read_chunk = h[kCtrRead];
  c->recalculate = h[kCtrRecalc];
  c->checksum_mismatch = h[kCtrMismatch];
  c->invalid = h[kCtrInvalid];
  c->stale_chunks = h[kCtrStale];
}

}  // namespace

extern "C" int h3c_diag_last_graph(uint64_t *out7) {
  if (!out7) return H3C_ERR_INVALID_ARG;
  const GraphShape &g = t_last_graph;
  const uint64_t v[7] = {g.nodes, g.roots, g.copies, g.kernels, g.reachable, g.edges, g.max_out};
  std::memcpy(out7, v, sizeof(v));
  return H3C_OK;
}

extern "C" int h3c_diag_last_graph_audit(uint64_t *out4) {
  if (!out4) return H3C_ERR_INVALID_ARG;
  const GraphAudit &a = t_last_audit;
  const uint64_t v[4] = {a.kernels, a.pointers, a.outside, a.unknown};
  std::memcpy(out4, v, sizeof(v));
  return H3C_OK;
}

extern "C" int h3c_diag_host_trace(uint64_t *out6, int reset) {
  if (!out6) return H3C_ERR_INVALID_ARG;
  std::memcpy(out6, t_host.sum, sizeof(t_host.sum));
  if (reset) {
    std::memset(t_host.sum, 0, sizeof(t_host.sum));
    t_host.have_return = false;
  }
  return H3C_OK;
}

extern "C" uint64_t h3c_diag_counter(int which) {
  return which >= 0 && which < kDiagN ? g_graph_stats[which].load() : 0;
}

extern "C" int h3c_update_ios_ex(uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                                 uint32_t n, h3c_update_result *results, uint32_t flags, h3c_update_counters *counters,
                                 void *stream) {
  if (counters) std::memset(counters, 0, sizeof(*counters));
  if (!valid_update_args(poly_type, chunks, nchunks, ios, n, results)) return H3C_ERR_INVALID_ARG;
  for (uint32_t c = 0; c < nchunks; ++c)  // a chunk longer than its capacity is a caller bug
    if (chunks[c].size > chunks[c].chunk_size) {
      h3c_rt::set_error_text("h3c_update_ios: a chunk's size exceeds its chunk_size");
      return H3C_ERR_INVALID_ARG;
    }
  if (n == 0) return H3C_OK;
  int dev = 0;
  int rc = h3c_rt::current_device(&dev);
  if (rc) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t C = std::max(nchunks, 1u);
  // device copies of the caller's arrays; the chunk table and counters through pinned staging
  const size_t cb = ((sizeof(h3c_chunk_state) * C + 255) & ~size_t(255));
  h3c_rt::DeviceLease lease(dev, 3 * cb + 256 + ((sizeof(h3c_update_io) * n + 255) & ~size_t(255)) +
                                     sizeof(h3c_update_result) * n + 256);
  h3c_rt::PinnedLease pin(2 * cb + 256);
  if (!lease.ok() || !pin.ok()) return H3C_ERR_HIP;
  char *cur = lease.data();
  h3c_chunk_state *d_in = carve<h3c_chunk_state>(cur, C);
  char *d_outblk = carve<char>(cur, cb + 64);  // [final chunks | counters]
  h3c_chunk_state *d_out = reinterpret_cast<h3c_chunk_state *>(d_outblk);
  unsigned long long *d_ctr = reinterpret_cast<unsigned long long *>(d_outblk + cb);
  h3c_update_io *d_ios = carve<h3c_update_io>(cur, n);
  h3c_update_result *d_res = carve<h3c_update_result>(cur, n);
  char *hin = pin.data(), *hout = pin.data() + cb + 256;
  std::memcpy(hin, chunks, sizeof(h3c_chunk_state) * nchunks);
  {
    StreamDrain drain{st, true};
    HIP_TRY(hipMemcpyAsync(d_in, hin, sizeof(h3c_chunk_state) * nchunks, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_ios, ios, sizeof(h3c_update_io) * n, hipMemcpyHostToDevice, st));
    rc = update_core(poly_type, d_in, d_out, nchunks, d_ios, n, d_res, flags, d_ctr, st, dev,
                     [&](hipStream_t s, const uint32_t *, uint32_t) -> int {
      HIP_TRY(hipMemcpyAsync(results, d_res, sizeof(h3c_update_result) * n, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipMemcpyAsync(hout, d_outblk, cb + 64, hipMemcpyDeviceToHost, s));
      return H3C_OK;
    });
    if (rc) return rc;
    drain.armed = false;
  }
  std::memcpy(chunks, hout, sizeof(h3c_chunk_state) * nchunks);
  if (counters) counters_from(reinterpret_cast<const unsigned long long *>(hout + cb), counters);
  return H3C_OK;
}

extern "C" int h3c_update_ios_dev(uint8_t poly_type, h3c_chunk_state *chunks_dev, uint32_t nchunks,
                                  const h3c_update_io *ios_dev, uint32_t n, h3c_update_result *results_dev,
                                  uint32_t flags, h3c_update_counters *counters_dev, void *stream) {
  t_host.entry = std::chrono::steady_clock::now();
  t_host.launch0 = t_host.launched = t_host.seen = t_host.entry;
  struct TraceOut {
    ~TraceOut() {
      HostTrace &h = t_host;
      const auto now = std::chrono::steady_clock::now();
      if (h.have_return) h.sum[0] += ns_between(h.last_return, h.entry);
      h.sum[1] += ns_between(h.entry, h.launch0);
      h.sum[2] += ns_between(h.launch0, h.launched);
      h.sum[3] += ns_between(h.launched, h.seen);
      h.sum[4] += ns_between(h.seen, now);
      h.sum[5] += 1;
      h.last_return = now;
      h.have_return = true;
    }
  } trace_out;
  if (!valid_update_args(poly_type, chunks_dev, nchunks, ios_dev, n, results_dev)) return H3C_ERR_INVALID_ARG;
  int dev = 0;
  int rc = h3c_rt::current_device(&dev);
  if (rc) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) {
    if (counters_dev) HIP_TRY(hipMemsetAsync(counters_dev, 0, sizeof(h3c_update_counters), st));
    return H3C_OK;
  }
  const uint32_t C = std::max(nchunks, 1u);
  h3c_rt::DeviceLease lease(dev, sizeof(h3c_chunk_state) * C + 256 + sizeof(h3c_update_counters) + 256);
  if (!lease.ok()) return H3C_ERR_HIP;
  char *cur = lease.data();
  h3c_chunk_state *d_out = carve<h3c_chunk_state>(cur, C);
  unsigned long long *d_ctr = counters_dev ? reinterpret_cast<unsigned long long *>(counters_dev)
                                           : carve<unsigned long long>(cur, kCtrN);
  StreamDrain drain{st, true};
  rc = update_core(poly_type, chunks_dev, d_out, nchunks, ios_dev, n, results_dev, flags, d_ctr, st, dev,
                   [&](hipStream_t s, const uint32_t *outcome, uint32_t cap) -> int {
                     // the final states replace the input table only if this pass is not
                     // redone: a redo must start from the batch's original states
                     if (nchunks) {
                       hipLaunchKernelGGL(uio_commit_kernel, dim3((nchunks + 255) / 256), dim3(256), 0, s, d_out,
                                          chunks_dev, nchunks, outcome, cap);
                       HIP_TRY(hipGetLastError());
                     }
                     return H3C_OK;
                   }, true, nchunks ? chunks_dev : nullptr);
  if (rc) return rc;
  drain.armed = false;
  return H3C_OK;
}

extern "C" int h3c_update_ios(uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                              uint32_t n, h3c_update_result *results, uint32_t flags, void *stream) {
  return h3c_update_ios_ex(poly_type, chunks, nchunks, ios, n, results, flags, nullptr, stream);
}

#if H3C_AF_TRACE
extern "C" int h3c_diag_af_trace(unsigned long long *out, int n) {  // (trace builds only)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_af_wg), 40ull * (unsigned)n) == hipSuccess ? 0 : -1;
}
extern "C" int h3c_diag_af_entry(unsigned long long *out, int n) {  // (trace builds only)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_af_entry), 16ull * (unsigned)n) == hipSuccess ? 0 : -1;
}
extern "C" int h3c_diag_af_waves(unsigned long long *out, uint32_t *blk, uint32_t *fin, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_af_wave), 128ull * (unsigned)n) == hipSuccess &&
                 hipMemcpyFromSymbol(blk, HIP_SYMBOL(g_af_blk), 16ull * (unsigned)n) == hipSuccess &&
                 hipMemcpyFromSymbol(fin, HIP_SYMBOL(g_af_fin), 64ull * (unsigned)n) == hipSuccess
             ? 0
             : -1;
}
#endif
#if H3C_FAST_TRACE == 3
extern "C" int h3c_diag_fast_wg(unsigned long long *out, int n) {  // (trace builds only)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_wg), 16ull * (unsigned)n) == hipSuccess ? 0 : -1;
}
extern "C" int h3c_diag_fast_rot(uint32_t rot) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fast_rot), &rot, 4) == hipSuccess ? 0 : -1;
}
#endif
