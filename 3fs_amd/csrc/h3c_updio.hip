// h3c_updio.hip -- general batched chunk updates on MI355X: every UpdateIO case of
// ChunkReplica::update (src/storage/store/ChunkReplica.cc:131-317) and its
// updateChecksum (:319-394), or the Rust chunk engine's Chunk::safe_write /
// copy_on_write checksum (src/storage/chunk_engine/src/alloc/chunk.rs:89-281).
//
// The reference handles one UpdateIO at a time: verify the client checksum of the
// payload (:193-207), zero-fill a gap, write / truncate / extend, and then either
// reuse, combine (append), or re-read prefix + suffix of the chunk from disk and CRC
// them (case iv: O(chunk) per write).  Here a batch of ops is applied with O(op bytes)
// work by linearity of CRC over GF(2).  With r the raw CRC (init ~0) of the chunk's
// n bytes, every op is an affine map of r:
//   WRITE [o, o+len), n -> n' = max(n, o+len):
//       r' = r * x^(8(n'-n)) ^ D * x^(8(n'-o-len)),
//       D  = crc0(payload) ^ crc0(old[o, e)) * x^(8(o+len-e)),  e = min(o+len, n)
//       (bytes at or past n read as zero; a gap [n, o) is zero on both sides)
//   TRUNCATE to t < n:   r' = (r ^ crc0(old[t, n))) * x^(-8(n-t))
//   grow to t > n (TRUNCATE or EXTEND, zero fill): r' = r * x^(8(t-n))
//   INIT (the chunk's stored checksum is not of this polynomial): r' = crc of [0, n)
// Pipeline (one host <-> device round trip per batch):
//   A. payload CRC jobs of every WRITE (seg_crc_kernel via launch_crc), run on the device
//      ahead of the update in the same stream.
//   B. host pass in sequence order: sizes, the reference's case analysis, and byte
//      jobs (old-range / cut-tail CRCs, payload copies, zero fills).  Jobs that touch
//      the same 4 KiB block are put in successive epochs (conflict levels); within an
//      epoch no two ops share a block.  The pass is speculative: it assumes every client
//      checksum matches (a rejected op changes nothing); the device checks them after A
//      and, on a mismatch, the copy kernels write nothing and the batch is redone with
//      the payload CRCs known.
//   C. per epoch: one launch_crc over the epoch's CRC jobs (reads the chunk before
//      this epoch's writes), then one copy kernel.
//   D. per op an affine element (M, E); rocPRIM inclusive_scan_by_key over
//      (chunk, sequence) order composes them; r_after = r0 * M ^ E.
//   E. host: per-op results and final chunk states from the case analysis:
//      case (i) (write type NONE or empty chunk) stores 0; cases (ii)-(iv) store the
//      CRC of the chunk after the op (reuse and combine equal it given a consistent
//      stored checksum; the client checksum was verified in A).
#include <sched.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <unistd.h>

#include <rocprim/device/device_scan_by_key.hpp>

#include "h3c_common.hpp"

namespace {

constexpr uint32_t kNoJob = 0xFFFFFFFFu;
constexpr uint64_t kConflictBlock = 4096;  // ops touching a common block go to different epochs
constexpr uint64_t kCopyPiece = 256u << 10;

enum : uint32_t { kAffNop = 0, kAffInit = 1, kAffWrite = 2, kAffTrunc = 3, kAffGrow = 4 };

struct AffIn {  // every length is below the chunk size (32 bits)
  uint32_t nb, na; // chunk length before / after the op
  uint32_t len;    // WRITE: payload bytes; INIT: chunk bytes
  uint32_t pad;    // WRITE: zero bytes after the old range (o + len - e)
  uint32_t tail;   // WRITE: bytes after the write in the new chunk (n' - o - len)
  uint32_t job;    // CRC job (old range / cut tail / whole chunk) or kNoJob
  uint32_t op;     // WRITE: op index (payload CRC)
  uint32_t kind;
};

struct Aff {
  uint32_t m, e;  // r -> r * m ^ e
};

__host__ __device__ inline uint32_t gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

struct AffOp {  // apply a, then b
  uint32_t poly;
  __host__ __device__ Aff operator()(const Aff &a, const Aff &b) const {
    // most ops leave the chunk length unchanged (m = 1: overwrites inside the chunk), and
    // then composing them is a XOR, not two bit-serial GF(2) multiplies
    if (b.m == kOne) return Aff{a.m, a.e ^ b.e};
    if (a.m == kOne) return Aff{b.m, gf_mul(a.e, b.m, poly) ^ b.e};
    return Aff{gf_mul(a.m, b.m, poly), gf_mul(a.e, b.m, poly) ^ b.e};
  }
};

struct CopyPiece {
  uint64_t dst, src, len;  // src == 0: zero fill
};

// A client checksum to check against the payload's CRC on the device (speculative pass).
struct VerifyItem {
  uint32_t op, want;
};

// bad[1 + k] = item k's payload CRC differs from the client's; bad[0] = any did.
__global__ void updio_verify_kernel(const VerifyItem *__restrict__ items, uint32_t nver,
                                    const uint32_t *__restrict__ payraw, uint32_t std_domain,
                                    uint32_t *__restrict__ bad) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nver) return;
  const VerifyItem it = items[k];
  const uint32_t got = std_domain ? ~payraw[it.op] : payraw[it.op];
  if (got != it.want) {
    bad[1 + k] = 1;
    atomicOr(bad, 1u);
  }
}

// One workgroup per piece (<= kCopyPiece bytes).  16-byte vector body when source and
// destination share their alignment (or for zero fill), bytes otherwise.  Nothing is
// written when `gate` is set (a client checksum failed in the speculative pass).
__global__ __launch_bounds__(256) void updio_copy_kernel(const CopyPiece *__restrict__ pieces,
                                                         const uint32_t *__restrict__ gate) {
  if (gate && *gate) return;
  const CopyPiece pc = pieces[blockIdx.x];
  uint8_t *d = reinterpret_cast<uint8_t *>(pc.dst);
  const uint8_t *s = reinterpret_cast<const uint8_t *>(pc.src);
  const uint64_t len = pc.len;
  if (s == nullptr || ((pc.dst ^ pc.src) & 15u) == 0) {
    const uint64_t head = min<uint64_t>(len, (16u - (pc.dst & 15u)) & 15u);
    for (uint64_t k = threadIdx.x; k < head; k += blockDim.x) d[k] = s ? s[k] : 0;
    const uint64_t nvec = (len - head) / 16;
    uint4 *d4 = reinterpret_cast<uint4 *>(d + head);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(s ? s + head : nullptr);
    for (uint64_t k = threadIdx.x; k < nvec; k += blockDim.x) d4[k] = s ? s4[k] : make_uint4(0, 0, 0, 0);
    for (uint64_t k = head + 16 * nvec + threadIdx.x; k < len; k += blockDim.x) d[k] = s ? s[k] : 0;
  } else {
    for (uint64_t k = threadIdx.x; k < len; k += blockDim.x) d[k] = s[k];
  }
}

__global__ void updio_aff_kernel(const AffIn *__restrict__ in, uint32_t npos, const uint32_t *__restrict__ payraw,
                                 const uint32_t *__restrict__ jobcrc, const PolyConsts *__restrict__ pc,
                                 Aff *__restrict__ out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npos) return;
  const AffIn a = in[p];
  const uint32_t poly = pc->poly;
  Aff r{kOne, 0u};
  switch (a.kind) {
    case kAffInit:  // reset to the chunk's CRC: shift(~0, n) ^ crc0(bytes)
      r.m = 0;
      r.e = dgf_mul(0xFFFFFFFFu, dxpow8n(a.len, pc, poly), poly) ^ jobcrc[a.job];
      break;
    case kAffWrite: {
      uint32_t d = payraw[a.op] ^ dgf_mul(0xFFFFFFFFu, dxpow8n(a.len, pc, poly), poly);  // crc0(payload)
      if (a.job != kNoJob) d ^= dgf_mul(jobcrc[a.job], dxpow8n(a.pad, pc, poly), poly);
      r.m = dxpow8s((int64_t)a.na - (int64_t)a.nb, pc, poly);
      r.e = dgf_mul(d, dxpow8n(a.tail, pc, poly), poly);
      break;
    }
    case kAffTrunc:
      r.m = dxpow8s((int64_t)a.na - (int64_t)a.nb, pc, poly);
      r.e = dgf_mul(jobcrc[a.job], r.m, poly);
      break;
    case kAffGrow:
      r.m = dxpow8s((int64_t)a.na - (int64_t)a.nb, pc, poly);
      break;
    default:
      break;
  }
  out[p] = r;
}

__global__ void updio_true_kernel(const Aff *__restrict__ scan, const uint32_t *__restrict__ key, uint32_t npos,
                                  const uint32_t *__restrict__ raw0, uint32_t poly, uint32_t *__restrict__ out) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npos) return;
  const Aff a = scan[p];
  const uint32_t r0 = raw0[key[p]];
  out[p] = (a.m == kOne ? r0 : dgf_mul(r0, a.m, poly)) ^ a.e;
}

using h3c_rt::StreamDrain;

// Device arena for one call: every buffer is carved from one pooled device lease
// (h3c_rt::DeviceLease; hipMallocAsync pools gave kernels stale bytes under ROCm 7.2).
struct Arena {
  char *base = nullptr;
  size_t off = 0;
  template <class T>
  T *take(size_t count) {
    T *p = reinterpret_cast<T *>(base + off);
    off += (count * sizeof(T) + 255) & ~size_t(255);
    return p;
  }
};

// Segment layout of a list of CRC jobs for launch_crc.
struct CrcBatch {
  std::vector<DevChunk> chunks;
  uint32_t total_segs = 0, max_segs = 0;
  uint64_t bytes = 0, max_len = 0;
};

// set_fold_consts with a one-entry cache per constant: a batch's jobs mostly share one
// length, and the shared memo behind set_fold_consts is thread_local (a TLS lookup per call
// in a shared library).  One cache per thread and call (the polynomial is fixed).
struct FoldCache {
  uint64_t r = ~0ull, n = ~0ull;
  uint32_t vr = 0, start = 0, vs = 0;
  void set(DevChunk &c, uint64_t seg_bytes, uint32_t poly) {
    const uint64_t m = (c.len + seg_bytes - 1) / seg_bytes;
    if (!m) {
      c.xlast = kOne;
    } else {
      const uint64_t rem = c.len - (m - 1) * seg_bytes;
      if (rem != r) {
        r = rem;
        vr = hxpow8n_memo(rem, poly);
      }
      c.xlast = vr;
    }
    if (!c.start) {
      c.xstart = 0;
    } else {
      if (c.len != n || c.start != start) {
        n = c.len;
        start = c.start;
        vs = hstart_shift(c.start, c.len, poly);
      }
      c.xstart = vs;
    }
  }
};

void add_job(CrcBatch &b, FoldCache &fc, uint64_t ptr, uint64_t len, uint32_t start, uint32_t out_idx,
             uint64_t seg_bytes, uint32_t poly) {
  DevChunk c{};
  c.ptr = ptr;
  c.len = len;
  c.start = start;
  c.out_idx = out_idx;
  c.seg_begin = b.total_segs;
  fc.set(c, seg_bytes, poly);
  const uint32_t ns = (uint32_t)((len + seg_bytes - 1) / seg_bytes);
  b.total_segs += ns;
  b.max_segs = std::max(b.max_segs, ns);
  b.bytes += len;
  b.max_len = std::max(b.max_len, len);
  b.chunks.push_back(c);
}

enum class Src : uint8_t { kInitial, kZero, kTrue };

struct Track {
  uint32_t size = 0;
  uint8_t type = H3C_TYPE_NONE;
  Src src = Src::kInitial;
  uint32_t true_pos = 0;   // scan position whose CRC is the stored value (Src::kTrue)
  bool started = false;    // has a scan segment
};

// H3C_UPDIO_TIMING=1: per-phase wall times on stderr (tuning aid).
struct PhaseClock {
  bool on = std::getenv("H3C_UPDIO_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[updio] %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

struct OpOut {
  Src src = Src::kInitial;
  uint32_t pos = 0;
  uint32_t chunk = 0;
};

// Chunk- and op-indexed state of the host pass.  With T threads, thread t owns a
// contiguous range of chunks (and their ops), so every write here is to a disjoint entry.
struct PassShared {
  std::vector<Track> tr;
  std::vector<uint32_t> cur;  // next free scan position per chunk
  std::vector<OpOut> outs;
  std::vector<uint32_t> raw0;
};

// One thread's job lists.  Job ids are local until the merge adds the thread's base.
struct PassLocal {
  std::vector<CrcBatch> ep_crc;
  std::vector<std::vector<CopyPiece>> ep_copy;
  std::vector<VerifyItem> verify;  // speculative attempt: client checksums checked on the device
  uint32_t njobs = 0;
  size_t nep = 0;  // epochs in use (ep_crc / ep_copy keep their storage across calls)
  // last epoch + 1 per 4 KiB block of the chunk being processed, tagged with `gen` (one
  // generation per chunk, so nothing is cleared between chunks)
  std::vector<uint64_t> blk;
  uint32_t gen = 0;
  void next_chunk(uint64_t blocks) {
    if (blk.size() < blocks || gen == 0xFFFFFFFFu) {
      blk.assign(std::max<uint64_t>(blocks, blk.size()), 0);
      gen = 0;
    }
    ++gen;
  }
  void clear() {
    for (size_t e = 0; e < nep; ++e) {
      ep_crc[e].chunks.clear();
      ep_crc[e].total_segs = ep_crc[e].max_segs = 0;
      ep_crc[e].bytes = ep_crc[e].max_len = 0;
      ep_copy[e].clear();
    }
    nep = 0;
    verify.clear();
    njobs = 0;
  }
};

// A persistent worker pool for the host pass (one per calling thread, so concurrent
// callers never wait on each other).  run(n, fn) calls fn(0..n-1); the caller runs fn(0).
class HostPool {
 public:
  explicit HostPool(unsigned workers) {
    for (unsigned w = 0; w < workers; ++w) th_.emplace_back([this, w] { loop(w + 1); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (std::thread &t : th_) t.join();
  }
  unsigned size() const { return (unsigned)th_.size() + 1; }
  void run(unsigned n, const std::function<void(unsigned)> &fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void loop(unsigned id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned)> *fn;
      unsigned n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
        n = n_;
      }
      if (id < n) {
        (*fn)(id);
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)> *fn_ = nullptr;
  unsigned n_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Threads for the host pass: 1 below kParallelOps ops, else H3C_HOST_THREADS, by default
// 16 capped by the CPUs this process may run on (16 threads: 41 M writes/s against 31 M
// with 8 on the GPU box's 16-core share, profiles/r01d_updio_host_threads_ab.txt).  A
// service calling from many threads at once should lower it: each calling thread keeps
// its own pool.
constexpr uint32_t kParallelOps = 16384;
unsigned pass_threads(uint32_t n) {
  if (n < kParallelOps) return 1;
  static const unsigned t = [] {
    const char *e = std::getenv("H3C_HOST_THREADS");
    int v = 16;
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) v = std::min(v, std::max(CPU_COUNT(&cs), 1));
    if (e) v = std::atoi(e);
    return (unsigned)std::min(std::max(v, 1), 32);
  }();
  return t;
}

void run_threads(unsigned T, const std::function<void(unsigned)> &fn) {
  if (T <= 1) {
    fn(0);
    return;
  }
  thread_local std::unique_ptr<HostPool> pool;
  thread_local pid_t owner = 0;
  if (pool && owner != getpid()) (void)pool.release();  // forked child: the workers do not exist here
  if (!pool || pool->size() < T) {
    pool.reset(new HostPool(T - 1));
    owner = getpid();
  }
  pool->run(T, fn);
}

// fn(k) for k in [0, ntasks) on T pool threads that pull tasks from a shared counter: a
// thread the OS runs slowly (the GPU boxes share their cores) takes fewer tasks.
void run_tasks(unsigned T, unsigned ntasks, const std::function<void(unsigned)> &fn) {
  std::atomic<unsigned> next{0};
  run_threads(std::min(T, ntasks), [&](unsigned) {
    for (unsigned k; (k = next.fetch_add(1, std::memory_order_relaxed)) < ntasks;) fn(k);
  });
}

// Per-thread host scratch, reused across calls: the pass touches tens of MB of host
// vectors per 100k ops, and fresh allocations each call cost page faults of the same
// order as the pass itself.
struct UpdioScratch {
  PassShared S;
  std::vector<PassLocal> L;
  CrcBatch pay;
  std::vector<CrcBatch> pay_parts;  // payload CRC jobs per op range
  std::vector<uint32_t> status, payraw, truev, start, opstart, order, cut, hist;
};

// Scan positions in (chunk, sequence) order, laid out before the pass: chunk c owns
// [start[c], start[c+1]), one slot per op that passed validation plus one for an INIT
// reset when the chunk's stored checksum is not of this polynomial.  Slots the pass does
// not use (rejected ops) stay identity elements.  Returns the slot count.
uint32_t plan_positions(uint8_t poly_type, const h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                        uint32_t n, const std::vector<uint32_t> &status, std::vector<uint32_t> &start) {
  start.assign(nchunks + 1, 0);
  for (uint32_t i = 0; i < n; ++i)
    if (status[i] != H3C_ERR_INVALID_ARG) ++start[ios[i].chunk + 1];
  for (uint32_t c = 0; c < nchunks; ++c) {
    if (start[c + 1] && chunks[c].size != 0 && chunks[c].type != poly_type) ++start[c + 1];
    start[c + 1] += start[c];
  }
  return start[nchunks];
}

// Op indices grouped by chunk, each group in sequence order (a stable counting sort):
// the ops of chunk c are order[opstart[c] .. opstart[c+1]).  Ops naming no chunk of the
// batch are left out; other invalid ops stay (their result reports the chunk's size).
void group_ops(const h3c_update_io *ios, uint32_t n, uint32_t nchunks, std::vector<uint32_t> &opstart,
               std::vector<uint32_t> &order) {
  opstart.assign(nchunks + 1, 0);
  for (uint32_t i = 0; i < n; ++i)
    if (ios[i].chunk < nchunks) ++opstart[ios[i].chunk + 1];
  for (uint32_t c = 0; c < nchunks; ++c) opstart[c + 1] += opstart[c];
  order.resize(opstart[nchunks]);
  std::vector<uint32_t> fill(opstart.begin(), opstart.end() - 1);
  for (uint32_t i = 0; i < n; ++i)
    if (ios[i].chunk < nchunks) order[fill[ios[i].chunk]++] = i;
}

// plan_positions + group_ops in one parallel counting sort (per-op-range histograms,
// prefix, stable scatter) when the per-thread histograms are small against the batch.
void layout_ops(uint8_t poly_type, const h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                uint32_t n, const std::vector<uint32_t> &status, unsigned T, std::vector<uint32_t> &start,
                std::vector<uint32_t> &opstart, std::vector<uint32_t> &order, std::vector<uint32_t> &hist) {
  if (T <= 1 || (uint64_t)nchunks * 4 > n) {
    plan_positions(poly_type, chunks, nchunks, ios, n, status, start);
    group_ops(ios, n, nchunks, opstart, order);
    return;
  }
  // hist[t][c]: ops of range t naming chunk c; hist[T + t][c]: of those, the ones that passed validation
  hist.resize((size_t)2 * T * nchunks);
  auto range = [&](unsigned t, uint32_t &i0, uint32_t &i1) {
    i0 = (uint32_t)((uint64_t)n * t / T);
    i1 = (uint32_t)((uint64_t)n * (t + 1) / T);
  };
  run_threads(T, [&](unsigned t) {
    uint32_t *all = &hist[(size_t)t * nchunks], *ok = &hist[(size_t)(T + t) * nchunks];
    std::fill(all, all + nchunks, 0u);
    std::fill(ok, ok + nchunks, 0u);
    uint32_t i0, i1;
    range(t, i0, i1);
    for (uint32_t i = i0; i < i1; ++i) {
      const uint32_t c = ios[i].chunk;
      if (c >= nchunks) continue;
      ++all[c];
      ok[c] += status[i] != H3C_ERR_INVALID_ARG;
    }
  });
  start.resize(nchunks + 1);
  opstart.resize(nchunks + 1);
  uint32_t pos = 0, op = 0;
  for (uint32_t c = 0; c < nchunks; ++c) {
    start[c] = pos;
    opstart[c] = op;
    uint32_t nok = 0;
    for (unsigned t = 0; t < T; ++t) {
      uint32_t &a = hist[(size_t)t * nchunks + c];
      const uint32_t na = a;
      a = op;  // becomes range t's scatter base for chunk c
      op += na;
      nok += hist[(size_t)(T + t) * nchunks + c];
    }
    pos += nok + (nok && chunks[c].size != 0 && chunks[c].type != poly_type ? 1u : 0u);
  }
  start[nchunks] = pos;
  opstart[nchunks] = op;
  order.resize(op);
  run_threads(T, [&](unsigned t) {
    uint32_t *base = &hist[(size_t)t * nchunks];
    uint32_t i0, i1;
    range(t, i0, i1);
    for (uint32_t i = i0; i < i1; ++i)
      if (ios[i].chunk < nchunks) order[base[ios[i].chunk]++] = i;
  });
}

// Thread t's chunks [cut[t], cut[t+1]): contiguous ranges of about n/T ops each.
void cut_chunks(const std::vector<uint32_t> &opstart, uint32_t nchunks, unsigned T, std::vector<uint32_t> &cut) {
  cut.assign(T + 1, nchunks);
  cut[0] = 0;
  const uint64_t total = opstart[nchunks];
  uint32_t c = 0;
  for (unsigned t = 1; t < T; ++t) {
    const uint64_t want = total * t / T;
    while (c < nchunks && opstart[c] < want) ++c;
    cut[t] = std::max(c, cut[t - 1]);
  }
}

// B. the host pass over chunks [clo, chi), each chunk's ops in sequence order.
// `payraw` == nullptr: speculative (every WRITE's client checksum is assumed to match and
// queued for the device check); otherwise the payload CRCs are known and `status` already
// carries every mismatch.  S.outs (indexed like `order`, so each thread writes one
// contiguous range: no false sharing) must hold order.size() entries and S.tr / S.cur /
// S.raw0 nchunks;
// this thread fills its own.
void host_pass(uint8_t poly_type, uint32_t poly, bool std_domain, const h3c_chunk_state *chunks,
               const h3c_update_io *ios, uint32_t *status, const uint32_t *payraw, uint64_t seg_j,
               const uint32_t *start, const uint32_t *opstart, const uint32_t *order, AffIn *lay, uint32_t *keys,
               uint32_t clo, uint32_t chi, PassShared &S, PassLocal &L) {
  L.clear();
  // The current chunk's state lives in locals and is stored once per chunk: S.tr / S.cur /
  // S.raw0 entries of neighbouring chunks share cache lines across threads.
  Track tk;
  uint32_t cur = 0, raw0 = 0;
  FoldCache fc;

  auto epoch_for = [&](uint32_t c, uint64_t a, uint64_t b) -> uint32_t {  // touched [a, b) of chunk c
    (void)c;
    if (b <= a) return 0;
    uint32_t e = 0;
    const uint64_t b0 = a / kConflictBlock, b1 = (b - 1) / kConflictBlock;
    const uint64_t tag = (uint64_t)L.gen << 32;
    for (uint64_t k = b0; k <= b1; ++k)
      if ((L.blk[k] & ~0xFFFFFFFFull) == tag) e = std::max(e, (uint32_t)L.blk[k]);
    for (uint64_t k = b0; k <= b1; ++k) L.blk[k] = tag | (e + 1);
    if (L.nep <= e) {
      L.nep = e + 1;
      if (L.ep_crc.size() < L.nep) {
        L.ep_crc.resize(L.nep);
        L.ep_copy.resize(L.nep);
      }
    }
    return e;
  };
  auto add_copy = [&](uint32_t e, uint64_t dst, uint64_t src, uint64_t len) {
    for (uint64_t k = 0; k < len; k += kCopyPiece)
      L.ep_copy[e].push_back(CopyPiece{dst + k, src ? src + k : 0, std::min(kCopyPiece, len - k)});
  };
  auto new_elem = [&](const AffIn &a) -> uint32_t {
    const uint32_t p = cur++;
    lay[p] = a;
    return p;
  };

  const uint32_t kend = opstart[chi];
  for (uint32_t c = clo; c < chi; ++c) {
    tk = Track{};
    tk.size = chunks[c].size;
    tk.type = chunks[c].type;
    cur = start[c];
    raw0 = 0;
    L.next_chunk(((uint64_t)chunks[c].chunk_size + kConflictBlock - 1) / kConflictBlock);
    for (uint32_t k = opstart[c]; k < opstart[c + 1]; ++k) {
      if (k + 16 < kend) {  // ops are visited in chunk order: their records are scattered
        __builtin_prefetch(&ios[order[k + 16]]);
        __builtin_prefetch(&status[order[k + 16]]);
      }
      const uint32_t i = order[k];
      const h3c_update_io &io = ios[i];
      if (status[i] == H3C_ERR_INVALID_ARG) continue;  // (marked by an earlier attempt)
      const uint64_t base = chunks[c].base;
      // A6: the client's checksum of the payload (:193-207); TRUNCATE / EXTEND carry NONE.
      if (status[i] == H3C_OK && io.checksum_type != H3C_TYPE_NONE && io.length != 0) {
        if (io.kind != H3C_UPD_WRITE) {
          status[i] = H3C_ERR_CHECKSUM_MISMATCH;
        } else if (payraw) {
          const uint32_t got = std_domain ? ~payraw[i] : payraw[i];
          if (got != io.checksum_value) status[i] = H3C_ERR_CHECKSUM_MISMATCH;
        } else {
          L.verify.push_back(VerifyItem{i, io.checksum_value});
        }
      }
      if (status[i] == H3C_ERR_CHECKSUM_MISMATCH) {  // rejected: nothing changes
        S.outs[k] = OpOut{tk.src, tk.true_pos, c};
        continue;
      }
      // TRUNCATE / EXTEND store a checksum of the chunk's own type (:328-332); one of the
      // other polynomial cannot be derived from this batch's CRC state (documented limit).
      if (io.kind != H3C_UPD_WRITE && !std_domain && tk.type != H3C_TYPE_NONE && tk.type != poly_type) {
        status[i] = H3C_ERR_INVALID_ARG;
        continue;
      }
      if (!tk.started) {  // the chunk's scan segment starts from a known CRC or an INIT reset
        tk.started = true;
        const h3c_chunk_state &cs = chunks[c];
        if (cs.size == 0) {
          raw0 = 0xFFFFFFFFu;  // raw CRC of no bytes
        } else if (cs.type == poly_type) {
          raw0 = std_domain ? ~cs.value : cs.value;
        } else {
          const uint32_t e = epoch_for(c, 0, cs.size);
          add_job(L.ep_crc[e], fc, base, cs.size, 0u, L.njobs, seg_j, poly);
          AffIn a{};
          a.kind = kAffInit;
          a.len = cs.size;
          a.job = L.njobs++;
          new_elem(a);
        }
      }
      const uint64_t nb = tk.size;
      uint64_t na = nb;
      AffIn a{};
      a.job = kNoJob;
      uint8_t type_after = tk.type;
      if (io.kind == H3C_UPD_WRITE) {  // :281-291, doRealWrite :124
        const uint64_t o = io.offset, len = io.length;
        na = std::max<uint64_t>(nb, o + len);
        const uint32_t e = epoch_for(c, std::min(o, nb), (o > nb || len) ? o + len : 0);
        if (o < nb && len) {
          const uint64_t end = std::min(o + len, nb);
          add_job(L.ep_crc[e], fc, base + o, end - o, 0u, L.njobs, seg_j, poly);
          a.job = L.njobs++;
          a.pad = (uint32_t)(o + len - end);
        }
        if (o > nb) add_copy(e, base + nb, 0, o - nb);
        if (len) add_copy(e, base + o, io.payload, len);
        a.kind = kAffWrite;
        a.len = (uint32_t)len;
        a.tail = (uint32_t)(na - o - len);
        a.op = i;
        type_after = io.checksum_type;
      } else {  // TRUNCATE / EXTEND (:260-273)
        const uint64_t l = io.length;
        if (l < nb && io.kind == H3C_UPD_TRUNCATE) {
          na = l;
          const uint32_t e = epoch_for(c, l, nb);
          add_job(L.ep_crc[e], fc, base + l, nb - l, 0u, L.njobs, seg_j, poly);
          a.kind = kAffTrunc;
          a.job = L.njobs++;
        } else if (l > nb) {
          na = l;
          const uint32_t e = epoch_for(c, nb, l);
          add_copy(e, base + nb, 0, l - nb);
          a.kind = kAffGrow;
        } else {
          a.kind = kAffNop;
        }
      }
      a.nb = (uint32_t)nb;
      a.na = (uint32_t)na;
      const uint32_t id = new_elem(a);
      tk.size = (uint32_t)na;
      tk.type = type_after;
      // updateChecksum: case (i) stores 0 (:334-336); (ii)-(iv) the chunk's CRC.
      if (!std_domain && (type_after == H3C_TYPE_NONE || na == 0)) {
        tk.src = Src::kZero;
      } else {
        tk.src = Src::kTrue;
        tk.true_pos = id;  // scan position
      }
      S.outs[k] = OpOut{tk.src, tk.true_pos, c};
    }
    S.tr[c] = tk;
    S.cur[c] = cur;
    S.raw0[c] = raw0;
    for (uint32_t p = cur; p < start[c + 1]; ++p) lay[p] = AffIn{0, 0, 0, 0, 0, kNoJob, 0, kAffNop};
    for (uint32_t p = start[c]; p < start[c + 1]; ++p) keys[p] = c;
  }
}

// Where the threads' lists go in the flattened per-epoch arrays (epoch-major, then thread).
struct PassMerge {
  size_t nep = 0, crc_total = 0, copy_total = 0, ver_total = 0;
  uint32_t njobs = 0, max_segs = 0;
  std::vector<uint32_t> job_base;             // [t]
  std::vector<size_t> ver_off;                // [t]
  std::vector<size_t> crc_off, copy_off;      // [e * T + t]
  std::vector<uint32_t> seg_base;             // [e * T + t]: segments of earlier threads in epoch e
  std::vector<CrcBatch> ep;                   // per-epoch totals (chunks unused)
  std::vector<size_t> ep_crc_begin, ep_copy_begin, ep_copy_count;

  void build(const std::vector<PassLocal> &L, unsigned T) {
    nep = 0;
    for (unsigned t = 0; t < T; ++t) nep = std::max(nep, L[t].nep);
    job_base.assign(T, 0);
    ver_off.assign(T, 0);
    njobs = 0;
    ver_total = 0;
    for (unsigned t = 0; t < T; ++t) {
      job_base[t] = njobs;
      njobs += L[t].njobs;
      ver_off[t] = ver_total;
      ver_total += L[t].verify.size();
    }
    crc_off.assign(nep * T, 0);
    copy_off.assign(nep * T, 0);
    seg_base.assign(nep * T, 0);
    ep.assign(nep, CrcBatch{});
    ep_crc_begin.assign(nep, 0);
    ep_copy_begin.assign(nep, 0);
    ep_copy_count.assign(nep, 0);
    crc_total = copy_total = 0;
    max_segs = 0;
    for (size_t e = 0; e < nep; ++e) {
      ep_crc_begin[e] = crc_total;
      ep_copy_begin[e] = copy_total;
      for (unsigned t = 0; t < T; ++t) {
        crc_off[e * T + t] = crc_total;
        copy_off[e * T + t] = copy_total;
        seg_base[e * T + t] = ep[e].total_segs;
        if (e < L[t].nep) {
          const CrcBatch &b = L[t].ep_crc[e];
          crc_total += b.chunks.size();
          copy_total += L[t].ep_copy[e].size();
          ep[e].total_segs += b.total_segs;
          ep[e].max_segs = std::max(ep[e].max_segs, b.max_segs);
          ep[e].bytes += b.bytes;
          ep[e].max_len = std::max(ep[e].max_len, b.max_len);
        }
      }
      ep_copy_count[e] = copy_total - ep_copy_begin[e];
      max_segs = std::max(max_segs, ep[e].total_segs);
    }
  }
  size_t ep_crc_count(size_t e) const { return (e + 1 < nep ? ep_crc_begin[e + 1] : crc_total) - ep_crc_begin[e]; }
};

// Phase 2 of the pass, per thread: its lists into the pinned staging with global job ids
// and epoch-relative segment indices, and its scan elements' job ids made global.
void pass_publish(const PassLocal &L, const PassMerge &M, unsigned t, unsigned T, uint32_t clo, uint32_t chi,
                  const uint32_t *start, const PassShared &S, AffIn *lay, DevChunk *crc, CopyPiece *copy,
                  VerifyItem *ver) {
  const uint32_t jb = M.job_base[t];
  for (size_t e = 0; e < L.nep; ++e) {
    DevChunk *dst = crc + M.crc_off[e * T + t];
    const uint32_t sb = M.seg_base[e * T + t];
    for (const DevChunk &d : L.ep_crc[e].chunks) {
      *dst = d;
      dst->out_idx += jb;
      dst->seg_begin += sb;
      ++dst;
    }
    if (!L.ep_copy[e].empty())
      std::memcpy(copy + M.copy_off[e * T + t], L.ep_copy[e].data(), L.ep_copy[e].size() * sizeof(CopyPiece));
  }
  if (!L.verify.empty()) std::memcpy(ver + M.ver_off[t], L.verify.data(), L.verify.size() * sizeof(VerifyItem));
  if (jb)
    for (uint32_t c = clo; c < chi; ++c)
      for (uint32_t p = start[c]; p < S.cur[c]; ++p)
        if (lay[p].job != kNoJob) lay[p].job += jb;
}

}  // namespace

extern "C" int h3c_update_ios(uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                              uint32_t n, h3c_update_result *results, uint32_t flags, void *stream) {
  if (poly_type != H3C_TYPE_CRC32C && poly_type != H3C_TYPE_CRC32) return H3C_ERR_INVALID_ARG;
  if ((n && (!ios || !results)) || (nchunks && !chunks) || n >= 0x7FFFFFFFu) return H3C_ERR_INVALID_ARG;
  for (uint32_t c = 0; c < nchunks; ++c)  // a chunk longer than its capacity is a caller bug
    if (chunks[c].size > chunks[c].chunk_size) {
      h3c_rt::set_error_text("h3c_update_ios: a chunk's size exceeds its chunk_size");
      return H3C_ERR_INVALID_ARG;
    }
  if (n == 0) return H3C_OK;
  const bool std_domain = (flags & H3C_UPD_STD_DOMAIN) != 0;
  int dev = 0;
  int rc = h3c_rt::current_device(&dev);
  if (rc) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const PolyConsts *pc = static_cast<const PolyConsts *>(h3c_rt::device_consts(dev, poly_type));
  const uint32_t poly = poly_type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;

  PhaseClock clk;
  thread_local UpdioScratch tls_ws;
  UpdioScratch &ws = tls_ws;  // a local name: lambdas run on pool threads must not name the thread_local
  const unsigned T = std::max(1u, std::min<unsigned>(pass_threads(n), nchunks));
  // ---- per-op validation (range :140-145, kind, client checksum type), by op range ----
  std::vector<uint32_t> &status = ws.status;
  status.resize(n);
  std::vector<uint64_t> part_bytes(T, 0);
  run_threads(T, [&](unsigned t) {
    const uint32_t i0 = (uint32_t)((uint64_t)n * t / T), i1 = (uint32_t)((uint64_t)n * (t + 1) / T);
    uint64_t pb = 0;
    for (uint32_t i = i0; i < i1; ++i) {
      const h3c_update_io &io = ios[i];
      status[i] = H3C_OK;
      const bool kind_ok = io.kind == H3C_UPD_WRITE || io.kind == H3C_UPD_TRUNCATE || io.kind == H3C_UPD_EXTEND;
      if (io.chunk >= nchunks || !kind_ok) {
        status[i] = H3C_ERR_INVALID_ARG;
        continue;
      }
      const h3c_chunk_state &c = chunks[io.chunk];
      if (io.offset >= c.chunk_size || (uint64_t)io.offset + io.length > c.chunk_size || !c.base ||
          (io.checksum_type != H3C_TYPE_NONE && io.checksum_type != poly_type) ||
          (io.kind == H3C_UPD_WRITE && io.length && !io.payload)) {
        status[i] = H3C_ERR_INVALID_ARG;
        continue;
      }
      if (io.kind == H3C_UPD_WRITE) pb += io.length;
    }
    part_bytes[t] = pb;
  });
  uint64_t pay_bytes = 0;
  for (unsigned t = 0; t < T; ++t) pay_bytes += part_bytes[t];
  // A. payload CRC jobs (raw, init ~0) of every valid WRITE, built per op range: run on the
  // device in the same stream as the update itself; the old-range CRC jobs of B use the
  // same segment size.  `pay` holds the totals; the parts are published into staging.
  const uint64_t seg = h3c_rt::pick_seg(pay_bytes, dev);
  if (ws.pay_parts.size() < T) ws.pay_parts.resize(T);
  run_threads(T, [&](unsigned t) {
    CrcBatch &b = ws.pay_parts[t];
    b.chunks.clear();
    b.total_segs = b.max_segs = 0;
    b.bytes = b.max_len = 0;
    FoldCache fc;
    const uint32_t i0 = (uint32_t)((uint64_t)n * t / T), i1 = (uint32_t)((uint64_t)n * (t + 1) / T);
    for (uint32_t i = i0; i < i1; ++i)
      if (status[i] == H3C_OK && ios[i].kind == H3C_UPD_WRITE && ios[i].length)
        add_job(b, fc, ios[i].payload, ios[i].length, 0xFFFFFFFFu, i, seg, poly);
  });
  CrcBatch &pay = ws.pay;  // totals only (its chunk list stays empty)
  pay.chunks.clear();
  pay.total_segs = pay.max_segs = 0;
  pay.bytes = pay.max_len = 0;
  std::vector<size_t> pay_off(T + 1, 0);
  std::vector<uint32_t> pay_seg_base(T, 0);
  for (unsigned t = 0; t < T; ++t) {
    const CrcBatch &b = ws.pay_parts[t];
    pay_off[t + 1] = pay_off[t] + b.chunks.size();
    pay_seg_base[t] = pay.total_segs;
    pay.total_segs += b.total_segs;
    pay.max_segs = std::max(pay.max_segs, b.max_segs);
    pay.bytes += b.bytes;
    pay.max_len = std::max(pay.max_len, b.max_len);
  }
  // The speculative attempt's payload CRCs need nothing from the host pass: they are
  // uploaded and launched now, so the device works through them while B runs on the host.
  const size_t npay = pay_off[T];
  h3c_rt::DeviceLease pay_dev(dev, (npay * sizeof(DevChunk) + 4ull * std::max(pay.total_segs, 1u) + 4ull * n) +
                                       3 * 256);
  h3c_rt::PinnedLease pay_pin(npay * sizeof(DevChunk) + 256);
  if (!pay_dev.ok() || !pay_pin.ok()) return H3C_ERR_HIP;
  StreamDrain drain{st};  // declared after the leases: every return below waits for the stream first
  Arena pa;
  pa.base = pay_dev.data();
  DevChunk *d_pay = pa.take<DevChunk>(npay);
  uint32_t *d_payseg = pa.take<uint32_t>(std::max(pay.total_segs, 1u));
  uint32_t *d_payraw_spec = pa.take<uint32_t>(n);
  if (npay)
    run_threads(T, [&](unsigned t) {
      DevChunk *dst = reinterpret_cast<DevChunk *>(pay_pin.data()) + pay_off[t];
      for (const DevChunk &d : ws.pay_parts[t].chunks) {
        *dst = d;
        dst->seg_begin += pay_seg_base[t];
        ++dst;
      }
    });
  drain.armed = true;
  HIP_TRY(hipMemsetAsync(d_payraw_spec, 0xFF, 4ull * n, st));
  if (npay) {
    HIP_TRY(hipMemcpyAsync(d_pay, pay_pin.data(), npay * sizeof(DevChunk), hipMemcpyHostToDevice, st));
    const int r = h3c_rt::launch_crc(st, dev, poly_type, d_pay, (uint32_t)npay, pay.total_segs, pay.max_segs, pay.bytes,
                                     seg, 0, d_payseg, nullptr, d_payraw_spec, nullptr, nullptr, -1,
                                     h3c_rt::small_rows_bound(pay.max_len, pay.max_segs));
    if (r) return r;
  }
  clk.mark("A prepare");

  // B + C-D, speculatively first: the host pass assumes every client checksum matches and
  // the device checks them before any byte is written (the copy kernels are gated on the
  // check).  A mismatch (rare: a corrupted transfer) costs a second attempt with the
  // payload CRCs known.  One host <-> device round trip per batch in the common case.
  PassShared &S = ws.S;
  // the pass runs as NT chunk-range tasks (4 per thread) pulled by the T threads
  const unsigned NT = std::max(1u, std::min<unsigned>(T == 1 ? 1u : 4u * T, nchunks));
  if (ws.L.size() < NT) ws.L.resize(NT);
  std::vector<uint32_t> &payraw = ws.payraw;  // known payload CRCs (second attempt only)
  std::vector<uint32_t> &truev = ws.truev;
  // scan elements and keys are written by the pass straight into pinned staging
  layout_ops(poly_type, chunks, nchunks, ios, n, status, T, ws.start, ws.opstart, ws.order, ws.hist);
  const uint32_t npos = ws.start[nchunks];
  const size_t lay_bytes = ((size_t)npos * sizeof(AffIn) + 255) & ~size_t(255);
  h3c_rt::PinnedLease pin_el(lay_bytes + 4ull * npos + 256);
  if (!pin_el.ok()) return H3C_ERR_HIP;
  AffIn *lay = reinterpret_cast<AffIn *>(pin_el.data());
  uint32_t *keys = reinterpret_cast<uint32_t *>(pin_el.data() + lay_bytes);
  truev.resize(npos);  // every entry is filled from the device before it is read
  S.tr.resize(nchunks);
  S.cur.resize(nchunks);
  S.raw0.resize(nchunks);
  S.outs.resize(ws.order.size());  // written by the pass for every op it accepts, read only for those
  cut_chunks(ws.opstart, nchunks, NT, ws.cut);
  clk.mark("B layout");
  PassMerge M;
  for (int attempt = 0;; ++attempt) {
    const bool spec = attempt == 0;
    run_tasks(T, NT, [&](unsigned k) {
      host_pass(poly_type, poly, std_domain, chunks, ios, status.data(), spec ? nullptr : payraw.data(), seg,
                ws.start.data(), ws.opstart.data(), ws.order.data(), lay, keys, ws.cut[k], ws.cut[k + 1], S,
                ws.L[k]);
    });
    M.build(ws.L, NT);
    clk.mark("B pass");
    // ---- C-D. device: payload CRCs + check (speculative), epochs, affine scan ----
    const uint32_t nver = (uint32_t)M.ver_total;
    size_t scan_tmp = 0;
    if (npos)
      HIP_TRY(rocprim::inclusive_scan_by_key(nullptr, scan_tmp, (uint32_t *)nullptr, (Aff *)nullptr, (Aff *)nullptr,
                                             (size_t)npos, AffOp{poly}, rocprim::equal_to<uint32_t>(), st));
    const size_t crc_chunks = M.crc_total, copy_pieces = M.copy_total;
    const uint32_t max_segs = M.max_segs;
    Arena a;
    const size_t bytes = crc_chunks * sizeof(DevChunk) + copy_pieces * sizeof(CopyPiece) +
                         nver * sizeof(VerifyItem) + 4ull * max_segs + 4ull * std::max(M.njobs, 1u) + 4ull * n +
                         npos * (sizeof(AffIn) + 2 * sizeof(Aff) + 8) + 4ull * nchunks + 4ull * nver + scan_tmp +
                         16 * 256;
    h3c_rt::DeviceLease scratch(dev, bytes);
    if (!scratch.ok()) return H3C_ERR_HIP;
    a.base = scratch.data();
    DevChunk *d_crc = a.take<DevChunk>(crc_chunks);
    CopyPiece *d_copy = a.take<CopyPiece>(copy_pieces);
    VerifyItem *d_ver = a.take<VerifyItem>(nver);
    uint32_t *d_seg = a.take<uint32_t>(max_segs);
    uint32_t *d_jobcrc = a.take<uint32_t>(std::max(M.njobs, 1u));
    uint32_t *d_payraw = spec ? d_payraw_spec : a.take<uint32_t>(n);
    AffIn *d_in = a.take<AffIn>(npos);
    Aff *d_aff = a.take<Aff>(npos);
    Aff *d_scan = a.take<Aff>(npos);
    uint32_t *d_keys = a.take<uint32_t>(npos);
    uint32_t *d_true = a.take<uint32_t>(npos);
    uint32_t *d_raw0 = a.take<uint32_t>(nchunks);
    uint32_t *d_bad = a.take<uint32_t>(1 + nver);  // [0]: any mismatch (gates the copies); [1+k]: item k
    void *d_tmp = a.take<char>(scan_tmp);

    // pinned staging: uploads [crc jobs | copies | verify | payraw | raw0] (the scan
    // elements and keys are already in pin_el), downloads [true values | mismatch flags |
    // payload CRCs]
    enum { kCrc, kCopy, kVer, kPayraw, kRaw0, kUp, kTrue = kUp, kBad, kPayBack, kAll };
    size_t len[kAll] = {crc_chunks * sizeof(DevChunk), copy_pieces * sizeof(CopyPiece),
                        nver * sizeof(VerifyItem), spec ? 0 : 4ull * n, 4ull * nchunks, 4ull * npos,
                        spec ? 4ull * (1 + nver) : 0, spec ? 4ull * n : 0};
    void *dst[kUp] = {d_crc, d_copy, d_ver, d_payraw, d_raw0};
    size_t off[kAll + 1];
    off[0] = 0;
    for (int k = 0; k < kAll; ++k) off[k + 1] = off[k] + ((len[k] + 255) & ~size_t(255));
    h3c_rt::PinnedLease pin(off[kAll]);
    if (!pin.ok()) return H3C_ERR_HIP;
    char *hp = pin.data();
    run_tasks(T, NT, [&](unsigned k) {
      pass_publish(ws.L[k], M, k, NT, ws.cut[k], ws.cut[k + 1], ws.start.data(), S, lay,
                   reinterpret_cast<DevChunk *>(hp + off[kCrc]),
                   reinterpret_cast<CopyPiece *>(hp + off[kCopy]), reinterpret_cast<VerifyItem *>(hp + off[kVer]));
    });
    if (!spec) std::memcpy(hp + off[kPayraw], payraw.data(), len[kPayraw]);
    std::memcpy(hp + off[kRaw0], S.raw0.data(), len[kRaw0]);
    const VerifyItem *ver_host = reinterpret_cast<const VerifyItem *>(hp + off[kVer]);

    int err = H3C_OK;
    auto body = [&]() -> int {
      for (int k = 0; k < kUp; ++k)
        if (len[k]) HIP_TRY(hipMemcpyAsync(dst[k], hp + off[k], len[k], hipMemcpyHostToDevice, st));
      if (npos) {
        HIP_TRY(hipMemcpyAsync(d_in, lay, npos * sizeof(AffIn), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(d_keys, keys, 4ull * npos, hipMemcpyHostToDevice, st));
      }
      if (spec) {  // the payload CRCs were launched before the host pass
        HIP_TRY(hipMemsetAsync(d_bad, 0, 4ull * (1 + nver), st));
        if (nver) {
          hipLaunchKernelGGL(updio_verify_kernel, dim3((nver + 255) / 256), dim3(256), 0, st, d_ver, nver, d_payraw,
                             std_domain ? 1u : 0u, d_bad);
          HIP_TRY(hipGetLastError());
        }
      }
      const uint32_t *gate = spec ? d_bad : nullptr;
      for (size_t e = 0; e < M.nep; ++e) {
        const size_t nc = M.ep_crc_count(e);
        if (nc) {
          const CrcBatch &b = M.ep[e];
          const int r = h3c_rt::launch_crc(st, dev, poly_type, d_crc + M.ep_crc_begin[e], (uint32_t)nc, b.total_segs,
                                           b.max_segs, b.bytes, seg, 0, d_seg, nullptr, d_jobcrc, nullptr, nullptr,
                                           -1, h3c_rt::small_rows_bound(b.max_len, b.max_segs));
          if (r) return r;
        }
        if (M.ep_copy_count[e]) {
          hipLaunchKernelGGL(updio_copy_kernel, dim3((uint32_t)M.ep_copy_count[e]), dim3(256), 0, st,
                             d_copy + M.ep_copy_begin[e], gate);
          HIP_TRY(hipGetLastError());
        }
      }
      if (npos) {
        const uint32_t tb = 256, gb = (npos + tb - 1) / tb;
        hipLaunchKernelGGL(updio_aff_kernel, dim3(gb), dim3(tb), 0, st, d_in, npos, d_payraw, d_jobcrc, pc, d_aff);
        HIP_TRY(hipGetLastError());
        size_t tmp = scan_tmp;
        HIP_TRY(rocprim::inclusive_scan_by_key(d_tmp, tmp, d_keys, d_aff, d_scan, (size_t)npos, AffOp{poly},
                                               rocprim::equal_to<uint32_t>(), st));
        hipLaunchKernelGGL(updio_true_kernel, dim3(gb), dim3(tb), 0, st, d_scan, d_keys, npos, d_raw0, poly, d_true);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(hp + off[kTrue], d_true, len[kTrue], hipMemcpyDeviceToHost, st));
      }
      if (spec) {
        HIP_TRY(hipMemcpyAsync(hp + off[kBad], d_bad, len[kBad], hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(hp + off[kPayBack], d_payraw, len[kPayBack], hipMemcpyDeviceToHost, st));
      }
      return H3C_OK;
    };
    err = body();
    const hipError_t e = hipStreamSynchronize(st);  // the leases are reused only after this
    drain.armed = false;
    if (err) return err;
    if (e != hipSuccess) {
      h3c_rt::set_error("h3c_update_ios", e);
      return H3C_ERR_HIP;
    }
    clk.mark("C-D device");
    if (spec) {
      const uint32_t *bad = reinterpret_cast<const uint32_t *>(hp + off[kBad]);
      if (bad[0]) {  // a client checksum did not match: nothing was written; redo with them known
        payraw.assign(n, 0xFFFFFFFFu);
        std::memcpy(payraw.data(), hp + off[kPayBack], 4ull * n);
        for (uint32_t k = 0; k < nver; ++k)
          if (bad[1 + k]) status[ver_host[k].op] = H3C_ERR_CHECKSUM_MISMATCH;
        continue;
      }
    }
    if (npos) std::memcpy(truev.data(), hp + off[kTrue], 4ull * npos);
    break;
  }

  // ---- E. results and final chunk states, per chunk range on the pass's threads ----
  for (uint32_t i = 0; i < n; ++i)
    if (ios[i].chunk >= nchunks) {  // IOResult default {NONE, 0}
      std::memset(&results[i], 0, sizeof(h3c_update_result));
      results[i].status = status[i];
    }
  run_tasks(T, NT, [&](unsigned k) {
    for (uint32_t c = ws.cut[k]; c < ws.cut[k + 1]; ++c) {
      const uint32_t init_value = chunks[c].value;
      auto value_of = [&](Src src, uint32_t pos) -> uint32_t {
        if (src == Src::kZero) return 0u;
        if (src == Src::kInitial) return init_value;
        return std_domain ? ~truev[pos] : truev[pos];
      };
      // replay sizes and types in sequence order for per-op results
      uint32_t size_now = chunks[c].size;
      uint8_t type_now = chunks[c].type;
      for (uint32_t k = ws.opstart[c]; k < ws.opstart[c + 1]; ++k) {
        const uint32_t i = ws.order[k];
        const h3c_update_io &io = ios[i];
        h3c_update_result &r = results[i];
        std::memset(&r, 0, sizeof(r));
        r.status = status[i];
        if (status[i] == H3C_ERR_INVALID_ARG) {  // IOResult default {NONE, 0}
          r.size = size_now;
          continue;
        }
        if (status[i] == H3C_OK) {  // size after the op (as in the pass)
          uint64_t na = size_now;
          if (io.kind == H3C_UPD_WRITE) na = std::max<uint64_t>(size_now, (uint64_t)io.offset + io.length);
          else if (io.kind == H3C_UPD_TRUNCATE || io.length > size_now) na = io.length;
          size_now = (uint32_t)na;
          if (io.kind == H3C_UPD_WRITE) type_now = io.checksum_type;
        }
        r.size = size_now;
        r.type = (std_domain && status[i] == H3C_OK) ? poly_type : type_now;
        r.value = value_of(S.outs[k].src, S.outs[k].pos);
      }
      if (S.tr[c].started) {
        chunks[c].size = S.tr[c].size;
        chunks[c].type = std_domain ? poly_type : S.tr[c].type;
        chunks[c].value = value_of(S.tr[c].src, S.tr[c].true_pos);
      }
    }
  });
  clk.mark("E results");
  if (clk.on)
    std::fprintf(stderr, "[updio] threads %u, tasks %u, epochs %zu, crc jobs %u, elements %u\n", T, NT, M.nep,
                 M.njobs, npos);
  return H3C_OK;
}

// Diagnostic hook, no device work (the payload-job build here is single-threaded; the
// call itself builds it per op range on the pool): host time of one speculative h3c_update_ios pass over
// `ios` (payload-job build, position plan, op grouping, host pass B with its merge and
// publication into staging), the fastest of `reps`; the phase split goes to stderr with
// H3C_UPDIO_TIMING.  Used to tune the host pass without a GPU.
extern "C" double h3c_diag_updio_host_ms(uint8_t poly_type, const h3c_chunk_state *chunks, uint32_t nchunks,
                                         const h3c_update_io *ios, uint32_t n, int reps) {
  const uint32_t poly = poly_type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;
  thread_local UpdioScratch tls_ws;
  UpdioScratch &ws = tls_ws;
  double total = 0, t_a = 0, t_b = 0, t_c = 0;
  std::vector<AffIn> lay;
  std::vector<uint32_t> keys;
  std::vector<DevChunk> crc;
  std::vector<CopyPiece> copy;
  std::vector<VerifyItem> ver;
  const unsigned T = std::max(1u, std::min<unsigned>(pass_threads(n), nchunks));
  const unsigned NT = std::max(1u, std::min<unsigned>(T == 1 ? 1u : 4u * T, nchunks));
  if (ws.L.size() < NT) ws.L.resize(NT);
  PassMerge M;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    ws.status.assign(n, H3C_OK);
    for (uint32_t i = 0; i < n; ++i)
      if (ios[i].chunk >= nchunks) ws.status[i] = H3C_ERR_INVALID_ARG;
    const uint64_t seg = 1u << 20;
    CrcBatch &pay = ws.pay;
    pay.chunks.clear();
    pay.total_segs = pay.max_segs = 0;
    pay.bytes = pay.max_len = 0;
    FoldCache fc;
    for (uint32_t i = 0; i < n; ++i)
      if (ws.status[i] == H3C_OK && ios[i].kind == H3C_UPD_WRITE && ios[i].length)
        add_job(pay, fc, ios[i].payload, ios[i].length, 0xFFFFFFFFu, i, seg, poly);
    const uint32_t npos = plan_positions(poly_type, chunks, nchunks, ios, n, ws.status, ws.start);
    lay.resize(npos);
    keys.resize(npos);
    ws.S.tr.resize(nchunks);
    ws.S.cur.resize(nchunks);
    ws.S.raw0.resize(nchunks);
    group_ops(ios, n, nchunks, ws.opstart, ws.order);
    ws.S.outs.assign(ws.order.size(), OpOut{});
    cut_chunks(ws.opstart, nchunks, NT, ws.cut);
    const auto t1 = std::chrono::steady_clock::now();
    std::vector<double> busy(NT, 0.0);
    run_tasks(T, NT, [&](unsigned k) {
      const auto b0 = std::chrono::steady_clock::now();
      host_pass(poly_type, poly, false, chunks, ios, ws.status.data(), nullptr, seg, ws.start.data(),
                ws.opstart.data(), ws.order.data(), lay.data(), keys.data(), ws.cut[k], ws.cut[k + 1], ws.S, ws.L[k]);
      busy[k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - b0).count();
    });
    if (std::getenv("H3C_UPDIO_BUSY") && r == reps - 1)
      for (unsigned k = 0; k < NT; ++k) std::fprintf(stderr, "  task %u busy %.3f ms\n", k, busy[k]);
    M.build(ws.L, NT);
    const auto t2 = std::chrono::steady_clock::now();
    crc.resize(M.crc_total);
    copy.resize(M.copy_total);
    ver.resize(M.ver_total);
    run_tasks(T, NT, [&](unsigned k) {
      pass_publish(ws.L[k], M, k, NT, ws.cut[k], ws.cut[k + 1], ws.start.data(), ws.S, lay.data(), crc.data(),
                   copy.data(), ver.data());
    });
    const auto t3 = std::chrono::steady_clock::now();
    using ms = std::chrono::duration<double, std::milli>;
    if (r == 0 || ms(t3 - t0).count() < total) {  // the fastest repetition
      t_a = ms(t1 - t0).count();
      t_b = ms(t2 - t1).count();
      t_c = ms(t3 - t2).count();
      total = ms(t3 - t0).count();
    }
  }
  if (std::getenv("H3C_UPDIO_TIMING"))
    std::fprintf(stderr, "[updio host] threads %u: payload jobs + plan + grouping %.3f ms, pass %.3f ms, publish %.3f ms\n",
                 T, t_a, t_b, t_c);
  return total;
}
