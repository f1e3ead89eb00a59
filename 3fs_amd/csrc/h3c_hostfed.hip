// h3c_hostfed.hip -- host-fed create/verify (BASELINE config 5).
//
// 3FS payloads live in host memory: RDMA BufferPool buffers (src/storage/service/
// StorageOperator.cc:546-558) and the 1 MiB ChunkDataIterator scratch
// (src/storage/store/ChunkFileView.cc:106-125).  This pipeline streams a batch of host
// chunks through two HBM staging windows:
//
//   copy stream    : H2D window w into stage[w%2]  (waits until the CRC of w-2 is done)
//   compute stream : seg_crc + finalize over window w's pieces  (waits for w's copy)
//
// so PCIe transfers overlap the CRC work.  Chunks are cut into pieces at window
// boundaries; host-contiguous pieces are copied with a single hipMemcpyAsync.  Each
// piece gets its init-0 CRC; a fold kernel then combines a chunk's pieces with
// x^(8*len) shifts and applies ChecksumInfo::create's starting value, and compares
// against the expected values (ChunkReplica.cc:193-207 / BatchReadJob.cc:43-54).
#include <hip/hip_runtime.h>

#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "h3c_common.hpp"

namespace {

struct Run {  // one hipMemcpyAsync
  const uint8_t *src;
  uint64_t stage_off, len;
};

struct Window {
  uint32_t piece_begin, piece_end;  // pieces [begin, end) in the global piece array
  uint32_t total_segs, max_piece_segs;
  uint64_t bytes;
  std::vector<Run> runs;
};

struct FoldChunk {  // per chunk: its pieces [pb, pe)
  uint64_t len;
  uint32_t start, pb, pe, flags;
};

__global__ void fold_kernel(const FoldChunk *__restrict__ chunks, uint32_t n, const uint32_t *__restrict__ piece_crc,
                            const uint64_t *__restrict__ piece_len, const PolyConsts *__restrict__ pc,
                            const uint32_t *__restrict__ expected, uint32_t *__restrict__ out_raw,
                            uint8_t *__restrict__ ok, uint32_t *__restrict__ mismatch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const FoldChunk ch = chunks[i];
  const uint32_t poly = pc->poly;
  uint32_t raw = 0;
  if (!(ch.flags & kFlagNone)) {
    uint32_t crc0 = 0;
    for (uint32_t p = ch.pb; p < ch.pe; ++p) crc0 = dgf_mul(crc0, dxpow8n(piece_len[p], pc, poly), poly) ^ piece_crc[p];
    raw = crc0 ^ (ch.len ? dgf_mul(ch.start, dxpow8n(ch.len, pc, poly), poly) : ch.start);
  }
  out_raw[i] = raw;
  if (expected) {
    const bool good = raw == expected[i];
    ok[i] = good ? 1 : 0;
    if (!good) atomicAdd(mismatch, 1u);
  }
}

}  // namespace

struct h3c_hostfed {
  int device = 0;
  uint64_t window = 0;
  uint8_t *stage[2] = {nullptr, nullptr};
  hipStream_t copy_st = nullptr;
  hipEvent_t copied[2] = {nullptr, nullptr}, freed[2] = {nullptr, nullptr};
  // grown on demand
  h3c_rt::DevChunk *d_pieces = nullptr;
  uint64_t *d_piece_len = nullptr;
  uint32_t *d_piece_crc = nullptr;
  size_t piece_cap = 0;
  uint32_t *d_segcrc[2] = {nullptr, nullptr};
  size_t seg_cap = 0;
  FoldChunk *d_fold = nullptr;
  uint32_t *d_exp = nullptr, *d_out = nullptr, *d_mis = nullptr;
  uint8_t *d_ok = nullptr;
  size_t chunk_cap = 0;
};

namespace {

void release(h3c_hostfed *h) {
  for (int b = 0; b < 2; ++b) {
    if (h->stage[b]) (void)hipFree(h->stage[b]);
    if (h->d_segcrc[b]) (void)hipFree(h->d_segcrc[b]);
    if (h->copied[b]) (void)hipEventDestroy(h->copied[b]);
    if (h->freed[b]) (void)hipEventDestroy(h->freed[b]);
  }
  if (h->copy_st) (void)hipStreamDestroy(h->copy_st);
  for (void *p : {(void *)h->d_pieces, (void *)h->d_piece_len, (void *)h->d_piece_crc, (void *)h->d_fold,
                  (void *)h->d_exp, (void *)h->d_out, (void *)h->d_mis, (void *)h->d_ok})
    if (p) (void)hipFree(p);
}

template <class T>
hipError_t grow(T *&p, size_t &cap_ignored, size_t n) {
  (void)cap_ignored;
  if (p) (void)hipFree(p);
  p = nullptr;
  return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T));
}

}  // namespace

extern "C" {

int h3c_hostfed_create(int device, uint64_t window_bytes, h3c_hostfed **out) {
  if (!out || window_bytes < (1u << 20) || window_bytes % 256) return H3C_ERR_INVALID_ARG;
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  int rc = h3c_init(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  auto *h = new h3c_hostfed();
  h->device = device;
  h->window = window_bytes;
  hipError_t e = hipSuccess;
  for (int b = 0; b < 2 && e == hipSuccess; ++b) {
    e = hipMalloc(&h->stage[b], window_bytes);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->copied[b], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->freed[b], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->copy_st, hipStreamNonBlocking);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    h3c_rt::set_error("h3c_hostfed_create", e);
    release(h);
    delete h;
    return H3C_ERR_HIP;
  }
  *out = h;
  return H3C_OK;
}

void h3c_hostfed_destroy(h3c_hostfed *h) {
  if (!h) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->copy_st);
  release(h);
  (void)hipSetDevice(prev);
  delete h;
}

int h3c_hostfed_run(h3c_hostfed *h, const h3c_desc *d, size_t n, const uint32_t *expected, uint32_t *out_raw,
                    uint8_t *ok, uint64_t *n_mismatch, void *stream) {
  if (!h || (n && (!d || !out_raw)) || (expected && !ok)) return H3C_ERR_INVALID_ARG;
  if (n_mismatch) *n_mismatch = 0;
  if (n == 0) return H3C_OK;
  if (n > 0xFFFFFFF0u) return H3C_ERR_INVALID_ARG;
  h3c_rt::DeviceRestore restore;  // every return below puts the caller back on its device
  HIP_TRY(hipGetDevice(&restore.prev));
  if (restore.prev != h->device) HIP_TRY(hipSetDevice(h->device));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint8_t type = 0;  // one polynomial per run (the batch API splits mixed batches)
  for (size_t i = 0; i < n; ++i)
    if (d[i].type == H3C_TYPE_CRC32C || d[i].type == H3C_TYPE_CRC32) {
      if (type && d[i].type != type) {
        h3c_rt::set_error_text("h3c_hostfed_run: mixed checksum types in one run");
        return H3C_ERR_INVALID_ARG;
      }
      type = d[i].type;
    }
  if (!type) type = H3C_TYPE_CRC32C;

  // ---- host-side layout: pieces, windows, copy runs ----
  const uint64_t W = h->window;
  std::vector<h3c_rt::DevChunk> pieces;
  std::vector<uint64_t> piece_len;
  std::vector<FoldChunk> fold(n);
  std::vector<Window> wins(1);
  uint64_t woff = 0;
  const uint8_t *last_end = nullptr;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    const h3c_desc &x = d[i];
    const bool none = !(x.type == H3C_TYPE_CRC32C || x.type == H3C_TYPE_CRC32) || (x.ptr == nullptr && x.len > 0);
    fold[i] = FoldChunk{none ? 0 : x.len, x.start_raw, (uint32_t)pieces.size(), (uint32_t)pieces.size(),
                        none ? kFlagNone : 0u};
    if (none || x.len == 0) continue;
    total += x.len;
    const uint8_t *src = static_cast<const uint8_t *>(x.ptr);
    uint64_t off = 0;
    while (off < x.len) {
      const bool contiguous = src + off == last_end && woff < W;
      if (!contiguous) woff = (woff + 255) & ~uint64_t(255);
      if (woff >= W) {
        wins.push_back(Window{});
        woff = 0;
      }
      Window &win = wins.back();
      const uint64_t take = std::min(x.len - off, W - woff);
      h3c_rt::DevChunk pc{};
      pc.len = take;
      pc.start = 0;
      pc.out_idx = (uint32_t)pieces.size();
      pc.ptr = woff;  // staging offset for now; rebased per window below
      pieces.push_back(pc);
      piece_len.push_back(take);
      if (!win.runs.empty() && src + off == last_end && win.runs.back().stage_off + win.runs.back().len == woff)
        win.runs.back().len += take;
      else
        win.runs.push_back(Run{src + off, woff, take});
      win.bytes += take;
      woff += take;
      off += take;
      last_end = src + off;
    }
    fold[i].pe = (uint32_t)pieces.size();
  }
  // piece ranges per window (pieces were appended in window order)
  {
    size_t p = 0;
    for (auto &win : wins) {
      win.piece_begin = (uint32_t)p;
      uint64_t acc = 0;
      while (p < pieces.size() && acc < win.bytes) acc += pieces[p++].len;
      win.piece_end = (uint32_t)p;
    }
  }
  const uint64_t seg_bytes = h3c_rt::pick_seg(std::min<uint64_t>(W, std::max<uint64_t>(total, 1)), h->device);
  size_t max_segs = 0;
  for (size_t wi = 0; wi < wins.size(); ++wi) {
    Window &win = wins[wi];
    uint32_t segs = 0, mx = 0;
    for (uint32_t p = win.piece_begin; p < win.piece_end; ++p) {
      pieces[p].seg_begin = segs;
      pieces[p].ptr += (uint64_t)(uintptr_t)h->stage[wi & 1];
      set_fold_consts(pieces[p], seg_bytes, type == H3C_TYPE_CRC32 ? kPolyCrc32 : kPolyCrc32c);
      const uint32_t ns = (uint32_t)((pieces[p].len + seg_bytes - 1) / seg_bytes);
      segs += ns;
      mx = std::max(mx, ns);
    }
    win.max_piece_segs = mx;
    win.total_segs = segs;
    max_segs = std::max<size_t>(max_segs, segs);
  }

  // ---- device scratch (grown on demand) ----
  size_t dummy = 0;
  if (pieces.size() > h->piece_cap) {
    HIP_TRY(grow(h->d_pieces, dummy, pieces.size()));
    HIP_TRY(grow(h->d_piece_len, dummy, pieces.size()));
    HIP_TRY(grow(h->d_piece_crc, dummy, pieces.size()));
    h->piece_cap = pieces.size();
  }
  if (max_segs > h->seg_cap) {
    HIP_TRY(grow(h->d_segcrc[0], dummy, max_segs));
    HIP_TRY(grow(h->d_segcrc[1], dummy, max_segs));
    h->seg_cap = max_segs;
  }
  if (n > h->chunk_cap) {
    HIP_TRY(grow(h->d_fold, dummy, n));
    HIP_TRY(grow(h->d_exp, dummy, n));
    HIP_TRY(grow(h->d_out, dummy, n));
    HIP_TRY(grow(h->d_ok, dummy, n));
    HIP_TRY(grow(h->d_mis, dummy, 1));
    h->chunk_cap = n;
  }
  // descriptor uploads and result downloads through pinned staging (h3c_rt::PinnedLease)
  const size_t up[4] = {pieces.size() * sizeof(h3c_rt::DevChunk), piece_len.size() * 8, n * sizeof(FoldChunk),
                        expected ? n * 4 : 0};
  const void *up_src[4] = {pieces.data(), piece_len.data(), fold.data(), expected};
  void *up_dst[4] = {h->d_pieces, h->d_piece_len, h->d_fold, h->d_exp};
  size_t pin_off[5], pin_bytes = 0;
  for (int k = 0; k < 4; ++k) {
    pin_off[k] = pin_bytes;
    pin_bytes += (up[k] + 255) & ~size_t(255);
  }
  pin_off[4] = pin_bytes;  // results: out (4n) | ok (n) | mismatch (4)
  h3c_rt::PinnedLease pin(pin_bytes + ((n * 4 + 255) & ~size_t(255)) + ((n + 255) & ~size_t(255)) + 256);
  if (!pin.ok()) return H3C_ERR_HIP;
  char *const pb = pin.data();
  char *const pr_out = pb + pin_off[4];
  char *const pr_ok = pr_out + ((n * 4 + 255) & ~size_t(255));
  char *const pr_mis = pr_ok + ((n + 255) & ~size_t(255));
  // from the first async copy on, an early return must wait for the copy stream and `st`
  // before `pin` goes back to the pool (another thread could lease it mid-transfer)
  h3c_rt::StreamDrain drain_st{st, true};
  h3c_rt::StreamDrain drain_copy{h->copy_st, true};
  for (int k = 0; k < 4; ++k)
    if (up[k]) {
      std::memcpy(pb + pin_off[k], up_src[k], up[k]);
      HIP_TRY(hipMemcpyAsync(up_dst[k], pb + pin_off[k], up[k], hipMemcpyHostToDevice, st));
    }
  if (expected) HIP_TRY(hipMemsetAsync(h->d_mis, 0, 4, st));

  // ---- the pipeline ----
  h3c_rt::ProfToken tok;
  HIP_TRY(h3c_rt::prof_begin(st, tok));
  // the copy stream must not start before the descriptor uploads above are ordered
  HIP_TRY(hipEventRecord(h->freed[0], st));
  HIP_TRY(hipEventRecord(h->freed[1], st));
  for (size_t wi = 0; wi < wins.size(); ++wi) {
    const Window &win = wins[wi];
    if (win.piece_end == win.piece_begin) continue;
    const int b = (int)(wi & 1);
    HIP_TRY(hipStreamWaitEvent(h->copy_st, h->freed[b], 0));
    for (const Run &r : win.runs)
      HIP_TRY(hipMemcpyAsync(h->stage[b] + r.stage_off, r.src, r.len, hipMemcpyHostToDevice, h->copy_st));
    HIP_TRY(hipEventRecord(h->copied[b], h->copy_st));
    HIP_TRY(hipStreamWaitEvent(st, h->copied[b], 0));
    const int rc = h3c_rt::launch_crc(st, h->device, type, h->d_pieces + win.piece_begin,
                                      win.piece_end - win.piece_begin, win.total_segs, win.max_piece_segs, win.bytes,
                                      seg_bytes, 0,
                                      h->d_segcrc[b], nullptr, h->d_piece_crc, nullptr, nullptr, -1);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(h->freed[b], st));
  }
  const PolyConsts *pc = static_cast<const PolyConsts *>(h3c_rt::device_consts(h->device, type));
  hipLaunchKernelGGL(fold_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, h->d_fold, (uint32_t)n,
                     h->d_piece_crc, h->d_piece_len, pc, expected ? h->d_exp : nullptr, h->d_out, h->d_ok, h->d_mis);
  HIP_TRY(hipGetLastError());
  HIP_TRY(h3c_rt::prof_end(st, tok, H3C_PROF_HOSTFED, total));
  HIP_TRY(hipMemcpyAsync(pr_out, h->d_out, n * 4, hipMemcpyDeviceToHost, st));
  uint32_t mis = 0;
  if (expected) {
    HIP_TRY(hipMemcpyAsync(pr_ok, h->d_ok, n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(pr_mis, h->d_mis, 4, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  drain_st.armed = drain_copy.armed = false;
  std::memcpy(out_raw, pr_out, n * 4);
  if (expected) {
    std::memcpy(ok, pr_ok, n);
    std::memcpy(&mis, pr_mis, 4);
  }
  if (n_mismatch) *n_mismatch = mis;
  return H3C_OK;
}

}  // extern "C"

// ---- NUMA-local pinned host buffers ----
// The reference's payloads sit in RDMA-registered BufferPool memory
// (src/storage/service/StorageOperator.cc:546-558, configs/storage_main.toml:218-222).
// For a host-fed GPU, those pages belong on the NUMA node of the GPU's PCIe root, or every
// H2D transfer crosses the socket interconnect.
namespace {
std::mutex g_host_mu;
std::unordered_map<void *, size_t> g_host_bufs;

int read_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  for (char *c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
  char path[160];
  std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = std::fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (std::fscanf(f, "%d", &node) != 1) node = -1;
  std::fclose(f);
  return node;
}
}  // namespace

extern "C" int h3c_device_numa_node(int device) { return read_numa_node(device); }

extern "C" int h3c_host_alloc(int device, uint64_t bytes, void **out, int *node_out) {
  if (!out || !bytes) return H3C_ERR_INVALID_ARG;
  *out = nullptr;
  int rc = h3c_init(device);
  if (rc) return rc;
  const long page = sysconf(_SC_PAGESIZE);
  const size_t len = (size_t)((bytes + page - 1) / page * page);
  void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) {
    h3c_rt::set_error_text("h3c_host_alloc: mmap failed");
    return H3C_ERR_HIP;
  }
  int node = read_numa_node(device);
  if (node >= 0 && node < 1024) {  // prefer the GPU's node; the kernel falls back when it is full
    unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
    mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    const long MPOL_PREFERRED_ = 1;
    if (syscall(SYS_mbind, p, len, MPOL_PREFERRED_, mask, (unsigned long)1024, 0u) != 0) node = -1;
  } else {
    node = -1;
  }
  std::memset(p, 0, len);  // fault the pages in under that policy
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterDefault);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    munmap(p, len);
    h3c_rt::set_error("h3c_host_alloc: hipHostRegister", e);
    return H3C_ERR_HIP;
  }
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_bufs[p] = len;
  }
  *out = p;
  if (node_out) *node_out = node;
  return H3C_OK;
}

extern "C" int h3c_host_free(void *p) {
  if (!p) return H3C_OK;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_bufs.find(p);
    if (it == g_host_bufs.end()) return H3C_ERR_INVALID_ARG;
    len = it->second;
    g_host_bufs.erase(it);
  }
  (void)hipHostUnregister(p);
  munmap(p, len);
  return H3C_OK;
}
