// h3c_common.hpp -- device/host building blocks shared by the engine's translation
// units (h3c_engine.hip: create/verify/combine; h3c_update.hip: partial updates).
// Everything here has internal linkage (anonymous namespace); the shared runtime
// state lives behind the h3c_rt:: functions defined in h3c_engine.hip.
#pragma once
#include <cstddef>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <initializer_list>
#include <shared_mutex>
#include <string>
#include <type_traits>

#include "h3c_crc.h"

namespace h3c_rt {
// HIP fails a launch into the legacy default stream made while any stream of the process is capturing.
// The engine's own captures (h3c_update_ios with H3C_UPD_GRAPHS) hold this gate exclusively; its
// synchronous entries that launch onto the legacy stream (stream == NULL: h3c_batch_create / verify,
// h3c_crc32c, the folly-signature entries) hold it shared, so they wait out an engine capture instead of
// failing (and the folly entries aborting).  Captures by other libraries remain the caller's concern.
std::shared_mutex &capture_gate();
// Per-device constant block for `type` (H3C_TYPE_CRC32C / H3C_TYPE_CRC32), built on first use.
const void *device_consts(int dev, int type);
int device_num_cu(int dev);
int device_wall_clock_khz(int dev);  // the rate of the device's wall_clock64() counter
// hipGetDevice + lazy init; returns H3C_OK or an h3c_status.
int current_device(int *dev);
void set_error(const char *what, hipError_t e);
void set_error_text(const char *text);
// Profiling hooks (h3c_profile_enable), per kind.  prof_stamp: the kernel stamps its own first
// workgroup start and last workgroup end on the device wall clock into a slot (`ts`, passed to
// the kernel; stamp_begin / stamp_end) -- nothing is added to the stream.  prof_begin: an event
// pair around the launch (for pipelines of copies and kernels; an event record costs the stream
// ~6 us, profiles/r04_*_rocprof_kernel_stats.csv timelines).
struct ProfToken;
// Gives back what a token holds when no prof_end took it over (an early error return between the two):
// the stamp slot's pending record is dropped, so h3c_profile_read neither waits on it nor counts it, and
// the pool rewinds past it; an event pair is destroyed.
void prof_cancel(const ProfToken &t);
struct ProfToken {
  bool on = false;
  hipEvent_t a = nullptr, b = nullptr;
  unsigned long long *ts = nullptr;  // prof_stamp's slot (device), or nullptr
  int dev = -1;
  int slot = -1;
  mutable bool closed = false;  // prof_end took over the slot or the events
  ProfToken() = default;
  ProfToken(const ProfToken &) = delete;
  ProfToken &operator=(const ProfToken &) = delete;
  ~ProfToken() {
    if (!closed && (ts || a || b)) prof_cancel(*this);
  }
};
hipError_t prof_begin(hipStream_t st, ProfToken &t);
hipError_t prof_stamp(int dev, ProfToken &t);
hipError_t prof_end(hipStream_t st, const ProfToken &t, int kind, uint64_t bytes);
// For launches timed by hipEvents recorded inside a replayed graph: whether profiling is on, and
// one launch's measured time added to the totals.
bool prof_enabled();
void prof_add(int kind, float ms, uint64_t bytes);

// Pinned host staging for the synchronous entry points.  Every host<->device transfer
// of host-side metadata or pageable payloads goes through one of these: a pageable
// hipMemcpyAsync into stream-ordered (hipMallocAsync) memory was measured to deliver
// stale bytes to the next kernel under ROCm 7.2's runtime, a pinned source never.
// Buffers come from a process-wide pool (mutex-protected, grow-only; one lease per
// concurrent call) and go back to it when the lease ends, after the call's final
// stream synchronisation.
// Device scratch for the synchronous entry points, from a per-device pool of hipMalloc'd
// buffers (grow-only, reused; one lease per concurrent call, returned after the call's
// final stream synchronisation).  Stream-ordered hipMallocAsync pools were measured to
// hand kernels stale bytes under ROCm 7.2's runtime; a plain pooled hipMalloc never.
class DeviceLease {
 public:
  DeviceLease(int dev, size_t bytes);
  ~DeviceLease();
  DeviceLease(const DeviceLease &) = delete;
  DeviceLease &operator=(const DeviceLease &) = delete;
  char *data() const { return p_; }
  bool ok() const { return p_ != nullptr; }

 private:
  int dev_ = 0;
  char *p_ = nullptr;
  size_t cap_ = 0;
};

class PinnedLease {
 public:
  explicit PinnedLease(size_t bytes);
  ~PinnedLease();
  PinnedLease(const PinnedLease &) = delete;
  PinnedLease &operator=(const PinnedLease &) = delete;
  char *data() const { return p_; }
  bool ok() const { return p_ != nullptr; }

 private:
  char *p_ = nullptr;
  size_t cap_ = 0;
};

// Waits for `st` on scope exit while armed: device work that reads or writes leased
// buffers must finish before the leases go back to their pools, on every return path.
// Declare it after the leases it protects (destructors run in reverse order).
struct StreamDrain {
  hipStream_t st;
  bool armed = false;
  ~StreamDrain() {
    if (armed) (void)hipStreamSynchronize(st);
  }
};

// Restores the caller's current device on scope exit (entry points that switch to a
// plan's / pipeline's device must not leave the caller on it after an early error).
struct DeviceRestore {
  int prev = -1;
  ~DeviceRestore() {
    if (prev >= 0) {
      int cur = -1;
      if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
  }
};

// Device copy of a descriptor (32 B).
struct DevChunk {
  uint64_t ptr;
  uint64_t len;
  uint32_t start;
  uint32_t out_idx;
  uint32_t seg_begin;
  uint32_t flags;  // bit0: result is {NONE,0}
  uint32_t xstart; // start * x^(8*len): the init's share of the raw CRC (set_fold_consts)
  uint32_t xlast;  // x^(8*r), r = the last segment's length: folds the segments
};
constexpr uint32_t kFlagNone = 1u;

// Segment-CRC + finalize launches over `nchunks` device descriptors (one polynomial
// group); profiled as `prof_kind` when >= 0.  Defined in h3c_engine.hip.
// small_rows != 0: every chunk is exactly one segment of at most small_rows 1 KiB rows
// (see small_rows_for) and none is NONE-flagged -- the small-chunk kernel then computes
// and stores the results.
// A small-path batch whose chunks share one length (a multiple of the small kernel's row), one
// start and row-aligned addresses (uniform_for): seg_uni_kernel.  contiguous: chunk i at
// base + i * stride with result i, no descriptor reads.
struct UniformBatch {
  uint32_t lanes = 0;  // 4, 8 or 16 lanes per chunk; 0: not uniform
  uint32_t rows = 0;   // rows of 16 * lanes bytes per chunk
  uint32_t xs = 0;     // the shared start's share of the raw CRC
  bool contiguous = false;
  uint64_t base = 0, stride = 0;
};
int launch_crc(hipStream_t st, int dev, int type, const DevChunk *d_chunks, uint32_t nchunks, uint32_t total_segs,
               uint32_t max_chunk_segs, uint64_t payload_bytes, uint64_t seg_bytes, uint32_t dbg, uint32_t *d_segcrc,
               const uint32_t *expected, uint32_t *out_raw, uint8_t *ok, uint32_t *mismatch, int prof_kind,
               uint32_t small_rows = 0, const UniformBatch *uni = nullptr);
// Payload CRCs of UpdateIOs in 4 KiB pieces (op_piece_crc_kernel): crc0_out[i] ^= init-0 CRC
// of item i; pbase = exclusive scan of the per-item piece counts, *d_total their sum.  Items:
// the n op payloads followed by the contents [0, size) of nchunks chunks (item
// n + c; 0 pieces skips an item): one launch for both, pbase over n + nchunks items.
int launch_uio_piece_crc(hipStream_t st, int dev, int type, const h3c_update_io *ios, uint32_t n,
                         const h3c_chunk_state *chunks, uint32_t nchunks, const uint32_t *pbase,
                         const uint32_t *d_total, uint32_t *crc0_out, const uint32_t *tbase = nullptr,
                         uint32_t tile = 0, uint32_t *err = nullptr);  // err: set when a piece falls outside its item  // tbase: item i's offset is pbase[i] + tbase[i / tile]
// Rows (1 KiB, absolute alignment) a byte range touches.
inline uint32_t host_rows(uint64_t ptr, uint64_t len) {
  return len ? (uint32_t)((((ptr + len + 1023) & ~uint64_t(1023)) - (ptr & ~uint64_t(1023))) / 1024) : 0;
}
// launch_crc's small_rows for host descriptors `c` (laid out with max_segs segments per
// chunk at most): their largest row count when all qualify for the small-chunk kernel, else 0.
uint32_t small_rows_for(const DevChunk *c, size_t n, uint32_t max_segs);
// uniform_for: fills `u` when host descriptors `c` (with small_rows != 0) form a UniformBatch.
void uniform_for(const DevChunk *c, size_t n, uint32_t small_rows, UniformBatch &u);
// The same from bounds alone: chunks of at most max_len bytes in at most max_segs segments.
uint32_t small_rows_bound(uint64_t max_len, uint32_t max_segs);
// Segment size the engine picks for a batch of `total_bytes` on device `dev`.
uint64_t pick_seg(uint64_t total_bytes, int dev);
// h3c_test_hook values (0 = default; initialised once from the environment).
uint64_t hook(int key);

// ---- kernel argument layouts, for auditing the pointers baked into captured graphs ----
// A captured graph replays its kernels with the argument values of the capture.  update_core keys its
// graph cache by every buffer the pipeline touches (UpdGraphKey); before a graph is instantiated, every
// pointer argument of every kernel node is checked to lie inside one of those buffers or the library's
// constant tables (a pointer outside them would replay into memory the key does not name).  HIP gives a
// node's argument values but not their types, so each kernel that can be captured registers its layout:
// per argument its size, alignment and the offsets of the pointers inside it (a pointer argument: 0; a
// struct argument: its pointer members, by an ArgLayout<> specialisation).
struct ArgSpec {
  uint16_t size = 0, align = 1;
  uint8_t nptr = 0;
  uint16_t ptr_off[12] = {};
};
struct KernelSig {
  const void *fn = nullptr;
  const char *name = nullptr;
  uint32_t nargs = 0;
  ArgSpec args[40];
};
template <class T, class = void>
struct ArgLayout {
  static_assert(std::is_arithmetic<T>::value || std::is_enum<T>::value,
                "a struct kernel argument needs an ArgLayout<> specialisation naming its pointer members");
  static void fill(ArgSpec &a) {
    a.size = sizeof(T);
    a.align = alignof(T);
  }
};
template <class T>
struct ArgLayout<T *, void> {
  static void fill(ArgSpec &a) {
    a.size = sizeof(T *);
    a.align = alignof(T *);
    a.nptr = 1;
    a.ptr_off[0] = 0;
  }
};
// a struct argument whose pointer members sit at `offs` (offsetof each)
template <class S>
inline void struct_arg(ArgSpec &a, std::initializer_list<size_t> offs) {
  a.size = sizeof(S);
  a.align = alignof(S);
  for (size_t o : offs) a.ptr_off[a.nptr++] = (uint16_t)o;
}
template <class... A>
KernelSig kernel_sig(void (*f)(A...), const char *name) {
  static_assert(sizeof...(A) <= 40, "too many kernel arguments for KernelSig");
  KernelSig s;
  s.fn = reinterpret_cast<const void *>(f);
  s.name = name;
  s.nargs = sizeof...(A);
  uint32_t i = 0;
  (void)i;
  (ArgLayout<typename std::remove_cv<A>::type>::fill(s.args[i++]), ...);
  return s;
}
// op_piece_crc_kernel<UioPieceSrc>'s layout (its argument struct is h3c_engine.hip's own).
KernelSig uio_piece_kernel_sig();
}  // namespace h3c_rt

#define HIP_TRY(expr)               \
  do {                              \
    hipError_t e_ = (expr);         \
    if (e_ != hipSuccess) {         \
      h3c_rt::set_error(#expr, e_); \
      return H3C_ERR_HIP;           \
    }                               \
  } while (0)

namespace {

constexpr uint32_t kPolyCrc32c = 0x82F63B78u;
constexpr uint32_t kPolyCrc32 = 0xEDB88320u;
constexpr uint32_t kOne = 0x80000000u;  // x^0 in the reflected representation
constexpr int kRowBytes = 1024;         // 64 lanes x 16 B
constexpr int kQuadRowBytes = 256;      // small-chunk kernel: 16 lanes x 16 B per chunk, 4 chunks per wave
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

// x^(8n) with a small per-thread memo (batches repeat a few chunk lengths).
uint32_t hxpow8n_memo(uint64_t n, uint32_t poly) {
  struct Entry {
    uint64_t n;
    uint32_t poly, v;
  };
  thread_local Entry memo[64] = {};
  thread_local bool used[64] = {};
  const uint32_t h = (uint32_t)((n * 0x9E3779B97F4A7C15ull) >> 58) ^ (poly & 63u);
  Entry &e = memo[h & 63];
  if (used[h & 63] && e.n == n && e.poly == poly) return e.v;
  e = Entry{n, poly, hxpow8n(n, poly)};
  used[h & 63] = true;
  return e.v;
}

// x^-1: the y with y*x == 1.  Multiplying by x is y>>1 ^ (poly if y&1); the
// result is x^0 (bit 31) only when y&1 and (y>>1)^poly == 1<<31.
uint32_t hx_inverse(uint32_t poly) { return ((poly ^ kOne) << 1) | 1u; }

// Device-side constant block, one per polynomial per device.
struct PolyConsts {
  uint32_t tab[4][256];  // tab[k][b] = (b << 8k) * x^(8*kRowBytes)
  uint32_t fix[256];     // [4l+j] = x^-(8*(16l+4j))
  uint32_t fixz[16];     // [z]    = x^-(8z)
  uint32_t pow8[64];     // [k]    = x^(8*2^k)
  uint32_t ipow8[64];    // [k]    = x^-(8*2^k)  (x is invertible mod P: P has a constant term)
  uint32_t poly;
  uint32_t pad[3];
  // Byte tables for multiplying by the 7 constants of the wave fold (wave_fold_tab):
  // red[0] = x^-32 (one dword back), red[1+k] = x^-(8*16*2^k) (2^k lanes back), k = 0..5.
  // red[m][k][b] = (b << 8k) * C_m, so a*C_m = XOR_k red[m][k][byte k of a].
  uint32_t red[7][4][256];
  uint32_t tabq[4][256];  // tabq[k][b] = (b << 8k) * x^(8*kQuadRowBytes): the small-chunk kernel's rows
  uint32_t tabo[4][256];  // tabo[k][b] = (b << 8k) * x^(8*128): its 8-lane (128-byte row) variant
  uint32_t tabf[4][256];  // tabf[k][b] = (b << 8k) * x^(8*64): its 4-lane (64-byte row) variant
  uint32_t tab2[4][256];  // (b << 8k) * x^(8*32): the uniform kernel's 2-lane (32-byte row) variant
  uint32_t tab1[4][256];  // (b << 8k) * x^(8*16): its 1-lane (16-byte row) variant
  // Shift tables for x^(8e), 0 <= e < 2^26 (dxpow8_fast): x^(8*4096*k) and x^(8r), r < 4096.
  uint32_t x4k[16384];
  uint32_t xb[4096];
};
constexpr int kRedTables = 7;
constexpr int kRedWords = kRedTables * 4 * 256;  // 7168 dwords = 28 KiB of LDS

static_assert(offsetof(PolyConsts, red) % 16 == 0, "fill_tables copies the fold tables in 16-byte pieces");
inline void build_consts(PolyConsts &pc, uint32_t poly) {
  std::memset(&pc, 0, sizeof(pc));
  pc.poly = poly;
  const uint32_t row = hxpow8n(kRowBytes, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) pc.tab[k][b] = hgf_mul(b << (8 * k), row, poly);
  const uint32_t qrow = hxpow8n(kQuadRowBytes, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) pc.tabq[k][b] = hgf_mul(b << (8 * k), qrow, poly);
  const uint32_t orow = hxpow8n(128, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) pc.tabo[k][b] = hgf_mul(b << (8 * k), orow, poly);
  const uint32_t frow = hxpow8n(64, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) pc.tabf[k][b] = hgf_mul(b << (8 * k), frow, poly);
  const uint32_t row2 = hxpow8n(32, poly), row1 = hxpow8n(16, poly);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) {
      pc.tab2[k][b] = hgf_mul(b << (8 * k), row2, poly);
      pc.tab1[k][b] = hgf_mul(b << (8 * k), row1, poly);
    }
  const uint32_t xinv8 = hgf_pow(hx_inverse(poly), 8, poly);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 4; ++j) pc.fix[4 * l + j] = hgf_pow(xinv8, 16u * l + 4u * j, poly);
  for (int z = 0; z < 16; ++z) pc.fixz[z] = hgf_pow(xinv8, z, poly);
  uint32_t p = 0x00800000u, q = xinv8;
  for (int k = 0; k < 64; ++k) {
    pc.pow8[k] = p;
    pc.ipow8[k] = q;
    p = hgf_mul(p, p, poly);
    q = hgf_mul(q, q, poly);
  }
  for (int m = 0; m < kRedTables; ++m) {
    const uint32_t c = hgf_pow(xinv8, m == 0 ? 4u : 16u << (m - 1), poly);
    for (int k = 0; k < 4; ++k)
      for (uint32_t b = 0; b < 256; ++b) pc.red[m][k][b] = hgf_mul(b << (8 * k), c, poly);
  }
  const uint32_t x8 = 0x00800000u, x4096 = hxpow8n(4096, poly);
  pc.xb[0] = pc.x4k[0] = kOne;
  for (int r = 1; r < 4096; ++r) pc.xb[r] = hgf_mul(pc.xb[r - 1], x8, poly);
  for (int k = 1; k < 16384; ++k) pc.x4k[k] = hgf_mul(pc.x4k[k - 1], x4096, poly);
}

using h3c_rt::DevChunk;
using h3c_rt::kFlagNone;

// start * x^(8n) with a one-entry per-thread memo (batches repeat one start and length).
inline uint32_t hstart_shift(uint32_t start, uint64_t n, uint32_t poly) {
  if (!start) return 0;
  thread_local uint64_t m_n = ~0ull;
  thread_local uint32_t m_start = 0, m_poly = 0, m_v = 0;
  if (n == m_n && start == m_start && poly == m_poly) return m_v;
  m_v = hgf_mul(start, hxpow8n_memo(n, poly), poly);
  m_n = n;
  m_start = start;
  m_poly = poly;
  return m_v;
}

// The finalize kernels' per-chunk shift constants, computed on the host once per
// distinct (start, length) instead of ~26 bit-serial GF(2) multiplies per chunk on the device.
inline void set_fold_consts(DevChunk &c, uint64_t seg_bytes, uint32_t poly) {
  c.xstart = hstart_shift(c.start, c.len, poly);
  const uint64_t m = (c.len + seg_bytes - 1) / seg_bytes;
  c.xlast = m ? hxpow8n_memo(c.len - (m - 1) * seg_bytes, poly) : kOne;
}

// ---------------------------------------------------------------- device GF(2)
// h3c_rt::prof_stamp's kernel side: the first workgroup's start (atomicMin) and the last
// workgroup's end (atomicMax) on the device wall clock; one atomic each per workgroup.  The
// stamped kernels are wrappers around a body function, so every wave reaches stamp_end (a body's
// early return comes back to it); the bodies have no barrier after their early returns.
__device__ __forceinline__ void stamp_begin(unsigned long long *ts) {
  if (ts && threadIdx.x == 0) atomicMin(&ts[0], (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void stamp_end(unsigned long long *ts) {
  if (!ts) return;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&ts[1], (unsigned long long)wall_clock64());
}

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

// x^(8n) for a signed byte count n (negative: the inverse shift, used when a chunk shrinks).
__device__ inline uint32_t dxpow8s(int64_t n, const PolyConsts *__restrict__ pc, uint32_t poly) {
  if (n >= 0) return dxpow8n((uint64_t)n, pc, poly);
  uint64_t m = (uint64_t)(-n);
  uint32_t r = kOne;
  int k = 0;
  while (m) {
    if (m & 1u) r = (r == kOne) ? pc->ipow8[k] : dgf_mul(r, pc->ipow8[k], poly);
    m >>= 1;
    ++k;
  }
  return r;
}

// a * b with the common identities short-cut (0 and x^0 = kOne).
__device__ __forceinline__ uint32_t dgf_mul_fast(uint32_t a, uint32_t b, uint32_t poly) {
  if (a == 0 || b == 0) return 0;
  if (a == kOne) return b;
  if (b == kOne) return a;
  return dgf_mul(a, b, poly);
}

// x^(8e) for a signed byte count e: two table lookups and one multiply for 0 <= e < 2^26
// (chunk offsets: kMaxChunkSize is 64 MiB, src/storage/store/ChunkMetadata.h:22), the
// square-and-multiply chains otherwise.
__device__ __forceinline__ uint32_t dxpow8_fast(int64_t e, const PolyConsts *__restrict__ pc, uint32_t poly) {
  if (e >= 0 && e < (int64_t(1) << 26)) return dgf_mul_fast(pc->x4k[e >> 12], pc->xb[e & 4095], poly);
  return dxpow8s(e, pc, poly);
}


// Per-lane LDS addressing of the replicated tables (see kernel header comment): two registers;
// the tables' remaining offsets ride in the ds_read immediate.
struct LaneLut {
  uint32_t off[2];
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;  // gfx950 has no v_xor3_b32; v_bitop3_b32 with truth table 0x96 is a^b^c
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// Layout: table t (0..3), entry b, copy c at byte address
//   (t>>1)*64 KiB + b*256 + (t&1)*128 + c*4,
// i.e. each 256-byte LDS row holds entry b of two tables x 32 copies.  ds_read_b32
// banks on (addr/4)%32 = c, so lane l reading copy l%32 never conflicts.  The
// address is one v_perm_b32: byte1 <- byte k of r, bytes 0 and 2 <- the lane's
// lane offset (byte0 = c<<2, byte2 = t>>1: off[t>>1]), byte3 <- 0; the (t&1)<<7 of tables 1 and 3
// is the ds_read's immediate offset (two offset registers a lane instead of four).
__device__ __forceinline__ LaneLut make_lut(uint32_t lane) {
  LaneLut L;
  const uint32_t c4 = (lane & 31u) * 4u;
  L.off[0] = c4;
  L.off[1] = c4 | 0x10000u;
  return L;
}
__device__ __forceinline__ uint32_t row_step(uint32_t r, const char *lb, const LaneLut &L) {
  const uint32_t a0 = __builtin_amdgcn_perm(r, L.off[0], 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(r, L.off[0], 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(r, L.off[1], 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(r, L.off[1], 0x0C020700u);
  const uint32_t t0 = *reinterpret_cast<const uint32_t *>(lb + a0);
  const uint32_t t1 = *reinterpret_cast<const uint32_t *>(lb + a1 + 128);
  const uint32_t t2 = *reinterpret_cast<const uint32_t *>(lb + a2);
  const uint32_t t3 = *reinterpret_cast<const uint32_t *>(lb + a3 + 128);
  return xor3(t0, t1, t2) ^ t3;
}
// LDS dword i holds table ((i>>14)<<1 | (i>>5)&1), entry (i>>6)&255.
__device__ __forceinline__ uint32_t fill_value_of(const uint32_t (*tab)[256], int i) {
  return tab[((i >> 14) << 1) | ((i >> 5) & 1)][(i >> 6) & 255];
}
// A 16-copy image of the same tables (64 KiB), for a kernel that runs two workgroups per CU:
// table t, entry b, copy c at byte address b*256 + t*64 + c*4 (the v_perm address keeps b in
// byte 1; byte 0 = t<<6 | c<<2).  Lanes l and l+16 share a copy: ds_read_b32 banks on
// (addr/4)%32 = (t&1)*16 + c, a 2-way conflict inside each 32-lane half-wave.
constexpr int kLdsWords16 = 4 * 256 * 16;  // 16384 dwords = 64 KiB
__device__ __forceinline__ LaneLut make_lut16(uint32_t lane) {
  LaneLut L;
  L.off[0] = (lane & 15u) * 4u;  // (t << 6: the immediate offset)
  L.off[1] = 0;
  return L;
}
__device__ __forceinline__ uint32_t row_step16(uint32_t r, const char *lb, const LaneLut &L) {
  const uint32_t a0 = __builtin_amdgcn_perm(r, L.off[0], 0x0C0C0400u);
  const uint32_t a1 = __builtin_amdgcn_perm(r, L.off[0], 0x0C0C0500u);
  const uint32_t a2 = __builtin_amdgcn_perm(r, L.off[0], 0x0C0C0600u);
  const uint32_t a3 = __builtin_amdgcn_perm(r, L.off[0], 0x0C0C0700u);
  const uint32_t t0 = *reinterpret_cast<const uint32_t *>(lb + a0);
  const uint32_t t1 = *reinterpret_cast<const uint32_t *>(lb + a1 + 64);
  const uint32_t t2 = *reinterpret_cast<const uint32_t *>(lb + a2 + 128);
  const uint32_t t3 = *reinterpret_cast<const uint32_t *>(lb + a3 + 192);
  return xor3(t0, t1, t2) ^ t3;
}
// LDS dword i of the 16-copy image holds table (i>>4)&3, entry (i>>6)&255.
__device__ __forceinline__ uint32_t fill_value16_of(const uint32_t (*tab)[256], int i) {
  return tab[(i >> 4) & 3][(i >> 6) & 255];
}
// The replicated stride tables and the fold tables into LDS (no barrier: the caller's).  With
// the 32-copy layout each table entry is loaded from HBM / L2 once and its 32 copies -- 128
// contiguous bytes -- written with 8 ds_write_b128 (the dword-per-copy loop loaded every entry 32
// times: ~20 us at the start of every workgroup); the fold tables go over in 16-byte pieces.
// `lds` must be 16-byte aligned; `red_words` a multiple of 4.
__device__ __forceinline__ void fill_tables(uint32_t *lds, const uint32_t (*tab)[256], const uint32_t *red_g,
                                            uint32_t red_words, uint32_t tid, uint32_t nthreads) {
  for (uint32_t e = tid; e < 1024u; e += nthreads) {
    const uint32_t t = e >> 8, b = e & 255u;
    const uint32_t v = tab[t][b];
    uint4 *dst = reinterpret_cast<uint4 *>(lds + (t >> 1) * 16384u + b * 64u + (t & 1u) * 32u);
    const uint4 q = make_uint4(v, v, v, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = q;
  }
  const uint4 *rs = reinterpret_cast<const uint4 *>(red_g);
  uint4 *rd = reinterpret_cast<uint4 *>(lds + kLdsWords);
  for (uint32_t i = tid; i < red_words / 4u; i += nthreads) rd[i] = rs[i];
}
// The LDS image of the 1 KiB-stride tables (rows of 64 lanes x 16 B).
__device__ __forceinline__ uint32_t fill_value(const PolyConsts *__restrict__ pc, int i) {
  return fill_value_of(pc->tab, i);
}

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

// A row load of the partial-update kernels (random 4 KiB read-modify-write: the old block, the payload).
// Nontemporal by default, as for streamed reads; H3C_RMW_NT_LOADS=0 makes them plain (A/B).  Round 5 measured
// the policies per kernel on config 3 (profiles/r05s_rmw_policy_ab.txt): plain *stores* for the write-back
// take the aligned UpdateIO kernel from 265 to 244 us and the block path's from 265 to 234 us, while plain
// loads help alone but lose beside plain stores (258 / 251 us).  Nothing in a partial-update kernel reads a
// line another workgroup wrote in the same launch (a block is read by its first writer only, payloads are
// never written), so write-back lines held in one XCD's L2 need no coherence inside a launch.
#ifndef H3C_RMW_NT_LOADS
#define H3C_RMW_NT_LOADS 1
#endif
__device__ __forceinline__ uint4 load_row_rmw(uint64_t a) {
#if H3C_RMW_NT_LOADS
  return load_row(a);
#else
  const v4u v = *(gv4p)a;
  return make_uint4(v.x, v.y, v.z, v.w);
#endif
}

// The fused config-3 kernels' per-XCD range weights move this fraction of the way to the last batch's measured
// class rates each batch (w <- w + gain * (rate / mean - w)).
#ifndef H3C_W_GAIN
#define H3C_W_GAIN 0.5
#endif

// The old rows of a partial update: `blk` when they are the chunk's own block (the block's first writer, which
// writes the block back), else a previous writer's payload.  The block's rows load plainly (the same wave
// writes the block back: the lines are then in L2 for the plain stores), the payloads nontemporally:
// upd_fused_kernel 234.3 -> 222.8 us, uio_afused_kernel ~-2 us (profiles/r05s_rmw_policy_ab.txt, part 4);
// H3C_RMW_BLOCK_PLAIN=0 loads both nontemporally.
#ifndef H3C_RMW_BLOCK_PLAIN
#define H3C_RMW_BLOCK_PLAIN 1
#endif
__device__ __forceinline__ uint4 load_row_old(uint64_t a, bool blk) {
  if (H3C_RMW_BLOCK_PLAIN && blk) {
    const v4u v = *(gv4p)a;
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return load_row_rmw(a);
}

// A row load of a kernel whose rows per chunk are narrower than a 128-byte line (fewer than 8 lanes x
// 16 B: the small-chunk kernels' 4-lane groups, 64-byte rows).  Nontemporal loads skip the CU's L1, so
// the two 64-byte halves of a line reach L2 as separate requests, and 7-8 % of the lines were fetched
// from HBM twice (TCC_MISS 1.077x the lines of an 8 GiB probe; plain loads: 1.000x, at the same speed:
// scripts/fetchcal.hip, profiles/r04_fetchcal.txt).  Plain loads keep the line in L1 for its other half.
template <uint64_t kRowBytesPerChunk>
__device__ __forceinline__ uint4 load_row_w(uint64_t a) {
  if (kRowBytesPerChunk >= 128) return load_row(a);
#ifndef H3C_SUBLINE_NT
  const v4u v = *(gv4p)a;
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return load_row(a);  // (A/B: round 3's nontemporal sub-line rows)
#endif
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
__device__ __forceinline__ void consume16(Streams &st, uint4 v, const char *lb, const LaneLut &L) {
  st.s0 = row_step16(st.s0 ^ v.x, lb, L);
  st.s1 = row_step16(st.s1 ^ v.y, lb, L);
  st.s2 = row_step16(st.s2 ^ v.z, lb, L);
  st.s3 = row_step16(st.s3 ^ v.w, lb, L);
}

// a * C for the constant whose byte tables start at `t` (4 x 256 dwords in LDS).
__device__ __forceinline__ uint32_t tab_mul(uint32_t a, const uint32_t *t) {
  return xor3(t[a & 255u], t[256u + ((a >> 8) & 255u)], t[512u + ((a >> 16) & 255u)]) ^ t[768u + (a >> 24)];
}

// Fold a wave's 256 stream states into the init-0 CRC of the rows they walked:
//   acc = XOR_{l,j} s(l,j) * x^-(8*(16l+4j))
// (stream (l,j) ended 16l+4j bytes past the 16-byte-rounded end).  Instead of 4 general
// GF(2) multiplies by per-lane constants (~200 VALU ops each), every multiply here is by
// one of 7 wave-uniform constants via byte tables in LDS (`red` = the 7168 dwords laid out
// as PolyConsts::red): a Horner pass over the lane's 4 streams with x^-32, then a 6-level
// shuffle tree whose level k folds lane l+2^k into lane l with x^-(128*2^k).  Lanes that
// no longer carry a partial sum skip the lookups (fewer LDS bank conflicts).  The result
// is valid in lane 0 only.
__device__ __forceinline__ uint32_t wave_fold_tab(const Streams &st, uint32_t lane, const uint32_t *red) {
  uint32_t v = tab_mul(st.s3, red) ^ st.s2;
  v = tab_mul(v, red) ^ st.s1;
  v = tab_mul(v, red) ^ st.s0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t o = __shfl_down(v, 1u << k, 64);
    if ((lane & ((2u << k) - 1u)) == 0) v ^= tab_mul(o, red + 1024 * (k + 1));
  }
  return v;
}


// N independent wave folds interleaved (N chunks' stream sets): the same arithmetic as
// wave_fold_tab, but the LDS-latency-bound Horner / tree chains of N chunks overlap.
template <int N>
__device__ __forceinline__ void wave_fold_tab_n(const Streams (&st)[N], uint32_t lane, const uint32_t *red,
                                                uint32_t (&out)[N]) {
  uint32_t v[N];
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = tab_mul(st[j].s3, red) ^ st[j].s2;
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = tab_mul(v[j], red) ^ st[j].s1;
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = tab_mul(v[j], red) ^ st[j].s0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    uint32_t o[N];
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = __shfl_down(v[j], 1u << k, 64);
    if ((lane & ((2u << k) - 1u)) == 0) {
#pragma unroll
      for (int j = 0; j < N; ++j) v[j] ^= tab_mul(o[j], red + 1024 * (k + 1));
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) out[j] = v[j];
}

#ifndef H3C_UNROLL
#define H3C_UNROLL 4
#endif
constexpr uint32_t kSmallRows = 8;  // segments of at most this many rows load all rows at once
constexpr int kUnroll = H3C_UNROLL;  // rows in flight per batch (x2 with the prefetch)


// init-0 CRC of bytes [S, E) (E > S), computed by one wavefront; valid in lane 0.
// The rows are the 1 KiB blocks [A, B) of absolute addresses covering [S, E), so every
// row load is 8 whole 128-byte lines whatever the payload's alignment; the first and
// last rows are masked (bytes outside [S, E) read as zero and pieces with no payload
// byte are never dereferenced).  Leading zeros do not change an init-0 CRC; the
// B - E trailing zeros are removed at the end with one multiply by x^-(8(B-E)).
__device__ inline uint32_t segment_crc0(uint64_t S, uint64_t E, uint32_t lane, const char *lb, const LaneLut &L,
                                        const uint32_t fix[4], const uint32_t *red,
                                        const PolyConsts *__restrict__ pc, uint32_t poly, uint32_t dbg) {
  const uint64_t A = S & ~uint64_t(kRowBytes - 1);
  const uint64_t B = (E + kRowBytes - 1) & ~uint64_t(kRowBytes - 1);
  const uint32_t K = (uint32_t)((B - A) / kRowBytes);
  const uint64_t base = A + 16u * lane;

  Streams st{0, 0, 0, 0};
  uint32_t r = 1;
  const uint32_t plain_end = K >= 2 ? K - 1 : 1;
  bool tail_done = false;
  if (!(dbg & 1u) && K >= 2 && K <= kSmallRows) {
    // A short segment (<= kSmallRows rows, e.g. a 4 KiB read or write buffer): issue
    // every row load before the first is consumed -- one memory round trip per segment
    // instead of one per row.
    uint4 v[kSmallRows];
    v[0] = load_masked(base, S, E);
#pragma unroll
    for (uint32_t u = 1; u + 1 < kSmallRows; ++u)
      if (u < plain_end) v[u] = load_row(base + (uint64_t)u * kRowBytes);
    v[kSmallRows - 1] = load_masked(base + (uint64_t)(K - 1) * kRowBytes, S, E);
    consume(st, v[0], lb, L);
#pragma unroll
    for (uint32_t u = 1; u + 1 < kSmallRows; ++u)
      if (u < plain_end) consume(st, v[u], lb, L);
    consume(st, v[kSmallRows - 1], lb, L);
    r = plain_end;
    tail_done = true;
  } else {
    // row 0 (masked)
    consume(st, load_masked(base, S, E), lb, L);
  }
  // Rows 1 .. K-2 lie fully inside [S, E).  They are read with saddr-form global
  // loads: wave-uniform 64-bit row base in SGPRs + per-lane 32-bit offset 16*lane,
  // so no per-row VGPR address arithmetic.  Prefetch rows are clamped to the last
  // plain row (every load stays inside the segment; the few clamped re-reads at a
  // segment's end hit in cache).  One batch of kUnroll rows is in flight while the
  // previous batch is consumed.
  if (!tail_done && !(dbg & 1u) && r + kUnroll <= plain_end) {
    // readfirstlane returns int: widen through uint32_t so the low half is not sign-extended.
    const uint64_t row0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)A) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(A >> 32)) << 32);
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
    // NOTE: an explicit two-buffer ping-pong form of this loop (no copy) gave wrong CRCs
    // under ROCm 7.2 hipcc -O3 at kUnroll=4 in round 1 (correct at -O1 and kUnroll=2).
    // Rebuilt against the current source (H3C_PINGPONG=1 below) it is correct at -O3 and
    // -O1 but 4 % slower (profiles/r02_pingpong_repro.txt), so the copy form stays; the
    // copies are register renames.
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
  if (K >= 2 && !tail_done) consume(st, load_masked(base + (uint64_t)(K - 1) * kRowBytes, S, E), lb, L);

  // Move every stream back to B (stream (l, j) ends 16l + 4j bytes past it).
  (void)fix;
  uint32_t acc = wave_fold_tab(st, lane, red);
  // ... then drop the B - E trailing zeros: x^-(8*pad) = x^-(8*16*(pad>>4)) * x^-(8*(pad&15))
  const uint32_t pad = (uint32_t)(B - E);
  if (pad >> 4) acc = dgf_mul(acc, pc->fix[4 * (pad >> 4)], poly);
  if (pad & 15) acc = dgf_mul(acc, pc->fixz[pad & 15], poly);
  return acc;
}

}  // namespace
