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
// Pipeline:
//   A. payload CRCs of every WRITE (seg_crc_kernel via launch_crc) -> host: the
//      client-checksum verify decides which ops apply (a rejected op changes nothing).
//   B. host pass in sequence order: sizes, the reference's case analysis, and byte
//      jobs (old-range / cut-tail CRCs, payload copies, zero fills).  Jobs that touch
//      the same 4 KiB block are put in successive epochs (conflict levels); within an
//      epoch no two ops share a block.
//   C. per epoch: one launch_crc over the epoch's CRC jobs (reads the chunk before
//      this epoch's writes), then one copy kernel.
//   D. per op an affine element (M, E); rocPRIM inclusive_scan_by_key over
//      (chunk, sequence) order composes them; r_after = r0 * M ^ E.
//   E. host: per-op results and final chunk states from the case analysis:
//      case (i) (write type NONE or empty chunk) stores 0; cases (ii)-(iv) store the
//      CRC of the chunk after the op (reuse and combine equal it given a consistent
//      stored checksum; the client checksum was verified in A).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>

#include <rocprim/device/device_scan_by_key.hpp>

#include "h3c_common.hpp"

namespace {

constexpr uint32_t kNoJob = 0xFFFFFFFFu;
constexpr uint64_t kConflictBlock = 4096;  // ops touching a common block go to different epochs
constexpr uint64_t kCopyPiece = 256u << 10;

enum : uint32_t { kAffNop = 0, kAffInit = 1, kAffWrite = 2, kAffTrunc = 3, kAffGrow = 4 };

struct AffIn {
  int64_t delta;   // n' - n
  uint64_t len;    // WRITE: payload bytes; INIT: chunk bytes
  uint64_t pad;    // WRITE: zero bytes after the old range (o + len - e)
  uint64_t tail;   // WRITE: bytes after the write in the new chunk (n' - o - len)
  uint32_t job;    // CRC job (old range / cut tail / whole chunk) or kNoJob
  uint32_t op;     // WRITE: op index (payload CRC)
  uint32_t kind;
  uint32_t pad2;
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
    return Aff{gf_mul(a.m, b.m, poly), gf_mul(a.e, b.m, poly) ^ b.e};
  }
};

struct CopyPiece {
  uint64_t dst, src, len;  // src == 0: zero fill
};

// One workgroup per piece (<= kCopyPiece bytes).  16-byte vector body when source and
// destination share their alignment (or for zero fill), bytes otherwise.
__global__ __launch_bounds__(256) void updio_copy_kernel(const CopyPiece *__restrict__ pieces) {
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
      r.m = dxpow8s(a.delta, pc, poly);
      r.e = dgf_mul(d, dxpow8n(a.tail, pc, poly), poly);
      break;
    }
    case kAffTrunc:
      r.m = dxpow8s(a.delta, pc, poly);
      r.e = dgf_mul(jobcrc[a.job], r.m, poly);
      break;
    case kAffGrow:
      r.m = dxpow8s(a.delta, pc, poly);
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
  out[p] = dgf_mul(raw0[key[p]], a.m, poly) ^ a.e;
}

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
  uint64_t bytes = 0;
};

void add_job(CrcBatch &b, uint64_t ptr, uint64_t len, uint32_t start, uint32_t out_idx, uint64_t seg_bytes,
             uint32_t poly) {
  DevChunk c{};
  c.ptr = ptr;
  c.len = len;
  c.start = start;
  c.out_idx = out_idx;
  c.seg_begin = b.total_segs;
  set_fold_consts(c, seg_bytes, poly);
  const uint32_t ns = (uint32_t)((len + seg_bytes - 1) / seg_bytes);
  b.total_segs += ns;
  b.max_segs = std::max(b.max_segs, ns);
  b.bytes += len;
  b.chunks.push_back(c);
}

// Open-addressing map (chunk, 4 KiB block) -> last epoch + 1 that touched it.
class BlockEpochs {
 public:
  explicit BlockEpochs(size_t expect) { reset(expect); }
  uint32_t get(uint64_t k) const {
    for (uint64_t h = slot(k);; h = (h + 1) & mask_) {
      if (keys_[h] == k) return vals_[h];
      if (keys_[h] == kEmpty) return 0;
    }
  }
  void put(uint64_t k, uint32_t v) {
    if (2 * (used_ + 1) > keys_.size()) grow();
    for (uint64_t h = slot(k);; h = (h + 1) & mask_) {
      if (keys_[h] == k) {
        vals_[h] = v;
        return;
      }
      if (keys_[h] == kEmpty) {
        keys_[h] = k;
        vals_[h] = v;
        ++used_;
        return;
      }
    }
  }

 private:
  static constexpr uint64_t kEmpty = ~0ull;
  uint64_t slot(uint64_t k) const { return ((k * 0x9E3779B97F4A7C15ull) >> shift_) & mask_; }
  void reset(size_t expect) {
    size_t cap = 1024;
    int bits = 10;
    while (cap < 2 * expect) {
      cap <<= 1;
      ++bits;
    }
    keys_.assign(cap, kEmpty);
    vals_.assign(cap, 0);
    mask_ = cap - 1;
    shift_ = 64 - bits;
    used_ = 0;
  }
  void grow() {
    std::vector<uint64_t> k = std::move(keys_);
    std::vector<uint32_t> v = std::move(vals_);
    reset(k.size());
    for (size_t i = 0; i < k.size(); ++i)
      if (k[i] != kEmpty) put(k[i], v[i]);
  }
  std::vector<uint64_t> keys_;
  std::vector<uint32_t> vals_;
  uint64_t mask_ = 0;
  int shift_ = 0;
  size_t used_ = 0;
};

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

}  // namespace

extern "C" int h3c_update_ios(uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                              uint32_t n, h3c_update_result *results, uint32_t flags, void *stream) {
  if (poly_type != H3C_TYPE_CRC32C && poly_type != H3C_TYPE_CRC32) return H3C_ERR_INVALID_ARG;
  if ((n && (!ios || !results)) || (nchunks && !chunks) || n >= 0x7FFFFFFFu) return H3C_ERR_INVALID_ARG;
  if (n == 0) return H3C_OK;
  const bool std_domain = (flags & H3C_UPD_STD_DOMAIN) != 0;
  int dev = 0;
  int rc = h3c_rt::current_device(&dev);
  if (rc) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const PolyConsts *pc = static_cast<const PolyConsts *>(h3c_rt::device_consts(dev, poly_type));
  const uint32_t poly = poly_type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c;

  PhaseClock clk;
  // ---- per-op validation (range :140-145, kind, client checksum type) ----
  std::vector<uint32_t> status(n, H3C_OK);
  for (uint32_t i = 0; i < n; ++i) {
    const h3c_update_io &io = ios[i];
    const bool kind_ok = io.kind == H3C_UPD_WRITE || io.kind == H3C_UPD_TRUNCATE || io.kind == H3C_UPD_EXTEND;
    if (io.chunk >= nchunks || !kind_ok) {
      status[i] = H3C_ERR_INVALID_ARG;
      continue;
    }
    const h3c_chunk_state &c = chunks[io.chunk];
    if (io.offset >= c.chunk_size || (uint64_t)io.offset + io.length > c.chunk_size || !c.base ||
        (io.checksum_type != H3C_TYPE_NONE && io.checksum_type != poly_type) ||
        (io.kind == H3C_UPD_WRITE && io.length && !io.payload))
      status[i] = H3C_ERR_INVALID_ARG;
  }

  // ---- A. payload CRCs (raw, init ~0) of every valid WRITE ----
  std::vector<uint32_t> payraw(n, 0xFFFFFFFFu);
  uint64_t pay_bytes = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (status[i] == H3C_OK && ios[i].kind == H3C_UPD_WRITE) pay_bytes += ios[i].length;
  const uint64_t seg_a = h3c_rt::pick_seg(pay_bytes, dev);
  CrcBatch pay;
  for (uint32_t i = 0; i < n; ++i)
    if (status[i] == H3C_OK && ios[i].kind == H3C_UPD_WRITE && ios[i].length)
      add_job(pay, ios[i].payload, ios[i].length, 0xFFFFFFFFu, i, seg_a, poly);
  if (!pay.chunks.empty()) {
    Arena a;
    const size_t nc = pay.chunks.size();
    const size_t bytes = nc * sizeof(DevChunk) + 4ull * pay.total_segs + 4ull * n + 3 * 256;
    // pinned staging (see h3c_rt::PinnedLease): [DevChunks | payload CRCs back]
    const size_t pin_raw = (nc * sizeof(DevChunk) + 255) & ~size_t(255);
    h3c_rt::PinnedLease pin(pin_raw + 4ull * n);
    if (!pin.ok()) return H3C_ERR_HIP;
    std::memcpy(pin.data(), pay.chunks.data(), nc * sizeof(DevChunk));
    h3c_rt::DeviceLease scratch(dev, bytes);
    if (!scratch.ok()) return H3C_ERR_HIP;
    a.base = scratch.data();
    DevChunk *d_chunks = a.take<DevChunk>(nc);
    uint32_t *d_seg = a.take<uint32_t>(pay.total_segs);
    uint32_t *d_raw = a.take<uint32_t>(n);
    int err = H3C_OK;
    hipError_t e = hipMemcpyAsync(d_chunks, pin.data(), nc * sizeof(DevChunk), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemsetAsync(d_raw, 0xFF, 4ull * n, st);
    if (e == hipSuccess) {
      err = h3c_rt::launch_crc(st, dev, poly_type, d_chunks, (uint32_t)nc, pay.total_segs, pay.max_segs, pay.bytes,
                               seg_a, 0, d_seg, nullptr, d_raw, nullptr, nullptr, -1);
      if (!err) e = hipMemcpyAsync(pin.data() + pin_raw, d_raw, 4ull * n, hipMemcpyDeviceToHost, st);
    }
    const hipError_t se = hipStreamSynchronize(st);
    if (e == hipSuccess) e = se;
    if (e != hipSuccess) {
      h3c_rt::set_error("h3c_update_ios: payload checksums", e);
      return H3C_ERR_HIP;
    }
    if (err) return err;
    std::memcpy(payraw.data(), pin.data() + pin_raw, 4ull * n);
  }

  clk.mark("A payload");
  // ---- B. host pass: verify, sizes, cases, epochs, byte jobs, affine elements ----
  std::vector<Track> tr(nchunks);
  for (uint32_t c = 0; c < nchunks; ++c) {
    tr[c].size = chunks[c].size;
    tr[c].type = chunks[c].type;
  }
  // chunk-major scan layout: positions are assigned after the pass
  std::vector<AffIn> elems;
  std::vector<uint32_t> elem_chunk;
  std::vector<OpOut> outs(n);
  std::vector<uint32_t> raw0(nchunks, 0);
  std::vector<CrcBatch> ep_crc;
  std::vector<std::vector<CopyPiece>> ep_copy;
  BlockEpochs last_touch(n + 1024);
  elems.reserve(n + 64);
  elem_chunk.reserve(n + 64);
  uint32_t njobs = 0;
  uint64_t job_bytes_total = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (status[i] == H3C_OK && ios[i].kind == H3C_UPD_WRITE) job_bytes_total += ios[i].length;
  const uint64_t seg_j = h3c_rt::pick_seg(job_bytes_total, dev);

  auto epoch_for = [&](uint32_t c, uint64_t a, uint64_t b) -> uint32_t {  // touched [a, b)
    if (b <= a) return 0;
    uint32_t e = 0;
    const uint64_t b0 = a / kConflictBlock, b1 = (b - 1) / kConflictBlock;
    for (uint64_t k = b0; k <= b1; ++k) {
      e = std::max(e, last_touch.get(((uint64_t)c << 32) | k));
    }
    for (uint64_t k = b0; k <= b1; ++k) last_touch.put(((uint64_t)c << 32) | k, e + 1);
    if (ep_crc.size() <= e) {
      ep_crc.resize(e + 1);
      ep_copy.resize(e + 1);
    }
    return e;
  };
  auto add_copy = [&](uint32_t e, uint64_t dst, uint64_t src, uint64_t len) {
    for (uint64_t k = 0; k < len; k += kCopyPiece)
      ep_copy[e].push_back(CopyPiece{dst + k, src ? src + k : 0, std::min(kCopyPiece, len - k)});
  };
  auto new_elem = [&](uint32_t c, const AffIn &a) -> uint32_t {
    const uint32_t id = (uint32_t)elems.size();
    elems.push_back(a);
    elem_chunk.push_back(c);
    return id;
  };

  for (uint32_t i = 0; i < n; ++i) {
    if (status[i] != H3C_OK) continue;
    const h3c_update_io &io = ios[i];
    const uint32_t c = io.chunk;
    Track &t = tr[c];
    const uint64_t base = chunks[c].base;
    // A6: the client's checksum of the payload (:193-207); TRUNCATE / EXTEND carry NONE.
    if (io.checksum_type != H3C_TYPE_NONE && io.length != 0) {
      const uint32_t want = io.kind == H3C_UPD_WRITE ? (std_domain ? ~payraw[i] : payraw[i]) : 0u;
      if (io.kind != H3C_UPD_WRITE || want != io.checksum_value) {
        status[i] = H3C_ERR_CHECKSUM_MISMATCH;
        outs[i] = OpOut{t.src, t.true_pos, c};
        continue;
      }
    }
    // TRUNCATE / EXTEND store a checksum of the chunk's own type (:328-332); one of the
    // other polynomial cannot be derived from this batch's CRC state (documented limit).
    if (io.kind != H3C_UPD_WRITE && !std_domain && t.type != H3C_TYPE_NONE && t.type != poly_type) {
      status[i] = H3C_ERR_INVALID_ARG;
      continue;
    }
    if (!t.started) {  // the chunk's scan segment starts from a known CRC or an INIT reset
      t.started = true;
      const h3c_chunk_state &cs = chunks[c];
      if (cs.size == 0) {
        raw0[c] = 0xFFFFFFFFu;  // raw CRC of no bytes
      } else if (cs.type == poly_type) {
        raw0[c] = std_domain ? ~cs.value : cs.value;
      } else {
        const uint32_t e = epoch_for(c, 0, cs.size);
        add_job(ep_crc[e], base, cs.size, 0u, njobs, seg_j, poly);
        AffIn a{};
        a.kind = kAffInit;
        a.len = cs.size;
        a.job = njobs++;
        new_elem(c, a);
      }
    }
    const uint64_t nb = t.size;
    uint64_t na = nb;
    AffIn a{};
    a.job = kNoJob;
    uint8_t type_after = t.type;
    if (io.kind == H3C_UPD_WRITE) {  // :281-291, doRealWrite :124
      const uint64_t o = io.offset, len = io.length;
      na = std::max<uint64_t>(nb, o + len);
      const uint32_t e = epoch_for(c, std::min(o, nb), (o > nb || len) ? o + len : 0);
      if (o < nb && len) {
        const uint64_t end = std::min(o + len, nb);
        add_job(ep_crc[e], base + o, end - o, 0u, njobs, seg_j, poly);
        a.job = njobs++;
        a.pad = o + len - end;
      }
      if (o > nb) add_copy(e, base + nb, 0, o - nb);
      if (len) add_copy(e, base + o, io.payload, len);
      a.kind = kAffWrite;
      a.len = len;
      a.tail = na - o - len;
      a.op = i;
      type_after = io.checksum_type;
    } else {  // TRUNCATE / EXTEND (:260-273)
      const uint64_t l = io.length;
      if (l < nb && io.kind == H3C_UPD_TRUNCATE) {
        na = l;
        const uint32_t e = epoch_for(c, l, nb);
        add_job(ep_crc[e], base + l, nb - l, 0u, njobs, seg_j, poly);
        a.kind = kAffTrunc;
        a.job = njobs++;
      } else if (l > nb) {
        na = l;
        const uint32_t e = epoch_for(c, nb, l);
        add_copy(e, base + nb, 0, l - nb);
        a.kind = kAffGrow;
      } else {
        a.kind = kAffNop;
      }
    }
    a.delta = (int64_t)na - (int64_t)nb;
    const uint32_t id = new_elem(c, a);
    t.size = (uint32_t)na;
    t.type = type_after;
    // updateChecksum: case (i) stores 0 (:334-336); (ii)-(iv) the chunk's CRC.
    if (!std_domain && (type_after == H3C_TYPE_NONE || na == 0)) {
      t.src = Src::kZero;
    } else {
      t.src = Src::kTrue;
      t.true_pos = id;  // element id; mapped to a scan position below
    }
    outs[i] = OpOut{t.src, t.true_pos, c};
  }

  clk.mark("B host");
  // ---- C-D. device: epochs, affine scan ----
  const uint32_t npos = (uint32_t)elems.size();
  std::vector<uint32_t> pos_of(npos), keys(npos);
  std::vector<AffIn> lay(npos);
  {  // stable counting sort of the elements by chunk: (chunk, sequence) order
    std::vector<uint32_t> start(nchunks + 1, 0);
    for (uint32_t id = 0; id < npos; ++id) ++start[elem_chunk[id] + 1];
    for (uint32_t c = 0; c < nchunks; ++c) start[c + 1] += start[c];
    for (uint32_t id = 0; id < npos; ++id) {
      const uint32_t c = elem_chunk[id], p = start[c]++;
      pos_of[id] = p;
      keys[p] = c;
      lay[p] = elems[id];
    }
  }
  std::vector<uint32_t> truev(npos, 0);
  if (npos) {
    size_t scan_tmp = 0;
    HIP_TRY(rocprim::inclusive_scan_by_key(nullptr, scan_tmp, (uint32_t *)nullptr, (Aff *)nullptr, (Aff *)nullptr,
                                           (size_t)npos, AffOp{poly}, rocprim::equal_to<uint32_t>(), st));
    size_t crc_chunks = 0, copy_pieces = 0;
    uint32_t max_segs = 0;
    for (size_t e = 0; e < ep_crc.size(); ++e) {
      crc_chunks += ep_crc[e].chunks.size();
      copy_pieces += ep_copy[e].size();
      max_segs = std::max(max_segs, ep_crc[e].total_segs);
    }
    const size_t bytes = crc_chunks * sizeof(DevChunk) + copy_pieces * sizeof(CopyPiece) + 4ull * max_segs +
                         4ull * std::max(njobs, 1u) + 4ull * n + npos * (sizeof(AffIn) + 2 * sizeof(Aff) + 8) +
                         4ull * nchunks + scan_tmp + 16 * 256;
    Arena a;
    h3c_rt::DeviceLease scratch(dev, bytes);
    if (!scratch.ok()) return H3C_ERR_HIP;
    a.base = scratch.data();
    DevChunk *d_crc = a.take<DevChunk>(crc_chunks);
    CopyPiece *d_copy = a.take<CopyPiece>(copy_pieces);
    uint32_t *d_seg = a.take<uint32_t>(max_segs);
    uint32_t *d_jobcrc = a.take<uint32_t>(std::max(njobs, 1u));
    uint32_t *d_payraw = a.take<uint32_t>(n);
    AffIn *d_in = a.take<AffIn>(npos);
    Aff *d_aff = a.take<Aff>(npos);
    Aff *d_scan = a.take<Aff>(npos);
    uint32_t *d_keys = a.take<uint32_t>(npos);
    uint32_t *d_true = a.take<uint32_t>(npos);
    uint32_t *d_raw0 = a.take<uint32_t>(nchunks);
    void *d_tmp = a.take<char>(scan_tmp);
    // flatten per-epoch descriptors (host copies stay alive until the final sync)
    std::vector<DevChunk> all_crc;
    std::vector<CopyPiece> all_copy;
    all_crc.reserve(crc_chunks);
    all_copy.reserve(copy_pieces);
    for (size_t e = 0; e < ep_crc.size(); ++e) {
      all_crc.insert(all_crc.end(), ep_crc[e].chunks.begin(), ep_crc[e].chunks.end());
      all_copy.insert(all_copy.end(), ep_copy[e].begin(), ep_copy[e].end());
    }
    // pinned staging for every upload and the result download (see h3c_rt::PinnedLease)
    const size_t up[6] = {crc_chunks * sizeof(DevChunk), copy_pieces * sizeof(CopyPiece), 4ull * n,
                          npos * sizeof(AffIn), 4ull * npos, 4ull * nchunks};
    const void *src[6] = {all_crc.data(), all_copy.data(), payraw.data(), lay.data(), keys.data(), raw0.data()};
    void *dst[6] = {d_crc, d_copy, d_payraw, d_in, d_keys, d_raw0};
    size_t pin_bytes = 0, pin_off[7];
    for (int k = 0; k < 6; ++k) {
      pin_off[k] = pin_bytes;
      pin_bytes += (up[k] + 255) & ~size_t(255);
    }
    pin_off[6] = pin_bytes;
    h3c_rt::PinnedLease pin(pin_bytes + 4ull * npos);
    if (!pin.ok()) return H3C_ERR_HIP;
    int err = H3C_OK;
    auto body = [&]() -> int {
      for (int k = 0; k < 6; ++k)
        if (up[k]) {
          std::memcpy(pin.data() + pin_off[k], src[k], up[k]);
          HIP_TRY(hipMemcpyAsync(dst[k], pin.data() + pin_off[k], up[k], hipMemcpyHostToDevice, st));
        }
      size_t co = 0, po = 0;
      for (size_t e = 0; e < ep_crc.size(); ++e) {
        const CrcBatch &b = ep_crc[e];
        if (!b.chunks.empty()) {
          const int r = h3c_rt::launch_crc(st, dev, poly_type, d_crc + co, (uint32_t)b.chunks.size(), b.total_segs,
                                           b.max_segs, b.bytes, seg_j, 0, d_seg, nullptr, d_jobcrc, nullptr, nullptr,
                                           -1);
          if (r) return r;
        }
        if (!ep_copy[e].empty()) {
          hipLaunchKernelGGL(updio_copy_kernel, dim3((uint32_t)ep_copy[e].size()), dim3(256), 0, st, d_copy + po);
          HIP_TRY(hipGetLastError());
        }
        co += b.chunks.size();
        po += ep_copy[e].size();
      }
      const uint32_t tb = 256, gb = (npos + tb - 1) / tb;
      hipLaunchKernelGGL(updio_aff_kernel, dim3(gb), dim3(tb), 0, st, d_in, npos, d_payraw, d_jobcrc, pc, d_aff);
      HIP_TRY(hipGetLastError());
      size_t tmp = scan_tmp;
      HIP_TRY(rocprim::inclusive_scan_by_key(d_tmp, tmp, d_keys, d_aff, d_scan, (size_t)npos, AffOp{poly},
                                             rocprim::equal_to<uint32_t>(), st));
      hipLaunchKernelGGL(updio_true_kernel, dim3(gb), dim3(tb), 0, st, d_scan, d_keys, npos, d_raw0, poly, d_true);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(pin.data() + pin_off[6], d_true, 4ull * npos, hipMemcpyDeviceToHost, st));
      return H3C_OK;
    };
    err = body();
    const hipError_t e = hipStreamSynchronize(st);  // the leases are reused only after this
    if (err) return err;
    if (e != hipSuccess) {
      h3c_rt::set_error("h3c_update_ios", e);
      return H3C_ERR_HIP;
    }
    std::memcpy(truev.data(), pin.data() + pin_off[6], 4ull * npos);
  }

  clk.mark("C-D device");
  // ---- E. results and final chunk states ----
  std::vector<uint32_t> init_value(nchunks);
  std::vector<uint8_t> init_type(nchunks);
  for (uint32_t c = 0; c < nchunks; ++c) {
    init_value[c] = chunks[c].value;
    init_type[c] = chunks[c].type;
  }
  auto value_of = [&](Src s, uint32_t id, uint32_t c) -> uint32_t {
    if (s == Src::kZero) return 0u;
    if (s == Src::kInitial) return init_value[c];
    const uint32_t raw = truev[pos_of[id]];
    return std_domain ? ~raw : raw;
  };
  // replay types and sizes in sequence order for per-op results
  std::vector<uint32_t> size_now(nchunks);
  std::vector<uint8_t> type_now(nchunks);
  for (uint32_t c = 0; c < nchunks; ++c) {
    size_now[c] = chunks[c].size;
    type_now[c] = chunks[c].type;
  }
  for (uint32_t i = 0; i < n; ++i) {
    h3c_update_result &r = results[i];
    std::memset(&r, 0, sizeof(r));
    r.status = status[i];
    const h3c_update_io &io = ios[i];
    if (status[i] == H3C_ERR_INVALID_ARG) {  // IOResult default {NONE, 0}
      r.size = io.chunk < nchunks ? size_now[io.chunk] : 0;
      continue;
    }
    const uint32_t c = io.chunk;
    if (status[i] == H3C_OK) {
      // size after the op (replayed exactly as in the pass)
      const uint64_t nb = size_now[c];
      uint64_t na = nb;
      if (io.kind == H3C_UPD_WRITE) na = std::max<uint64_t>(nb, (uint64_t)io.offset + io.length);
      else if (io.kind == H3C_UPD_TRUNCATE || io.length > nb) na = io.length;
      size_now[c] = (uint32_t)na;
      if (io.kind == H3C_UPD_WRITE) type_now[c] = io.checksum_type;
    }
    r.size = size_now[c];
    r.type = (std_domain && status[i] == H3C_OK) ? poly_type : type_now[c];
    r.value = value_of(outs[i].src, outs[i].pos, c);
  }
  for (uint32_t c = 0; c < nchunks; ++c) {
    if (!tr[c].started) continue;
    chunks[c].size = tr[c].size;
    chunks[c].type = std_domain ? poly_type : tr[c].type;
    chunks[c].value = value_of(tr[c].src, tr[c].true_pos, c);
  }
  clk.mark("E results");
  if (clk.on) std::fprintf(stderr, "[updio] epochs %zu, crc jobs %u, elements %u\n", ep_crc.size(), njobs, npos);
  return H3C_OK;
}
