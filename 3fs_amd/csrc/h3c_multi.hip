// h3c_multi.hip -- one engine object over several GPUs of one process.
//
// 3FS runs one storage_main per node; its checksum callers are the 32 AIO threads and 32 update
// threads inside that one process (src/storage/aio/AioReadWorker.h:26, src/storage/update/
// UpdateWorker.h:15), and the resync scrub is one caller per target (src/storage/service/
// ReliableForwarding.cc:158-182 -> src/storage/aio/BatchReadJob.cc:43-54).  So the multi-GPU path
// lives behind the C ABI, not in a launcher: an h3c_multi owns one host worker thread per listed
// device (hipSetDevice once, its own non-blocking stream, its own host-fed pipeline with NUMA-local
// windows, created on first use), splits each batch, runs the single-device entry points on every
// worker at once, and writes the results straight into disjoint slices of the caller's host arrays.
// Chunks are independent: no collective, no RCCL, no torch.
//
// Partition (h3c_multi_partition): contiguous index ranges balanced by payload bytes, the cut for
// worker k at the first index whose byte prefix sum reaches k/world of the total -- the same float64
// arithmetic as 3fs_amd/shard.py::partition, so both sides agree bit for bit (tests/test_multi.py).
// A device-resident payload is read where it lives: a descriptor (or an update's chunk) whose memory
// belongs to another listed device than its range's worker goes to the least-loaded worker on that
// device instead; memory on a device the object does not drive is an error (H3C_ERR_INVALID_ARG).
// Updates shard by chunk, so every op on a chunk runs on one worker, in sequence order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "h3c_crc.h"

namespace h3c_rt {
void set_error_text(const char *text);  // h3c_engine.hip: the calling thread's h3c_last_error()
}

namespace {

constexpr uint64_t kHostfedMin = 8ull << 20;  // pinned payload bytes per worker that go through its pipeline

bool is_crc(uint8_t t) { return t == H3C_TYPE_CRC32C || t == H3C_TYPE_CRC32; }

// The owning device of device memory, cached per allocation range for one call (an address range can be
// freed and re-allocated on another device between calls, so nothing is kept across calls).
struct OwnerCache {
  struct R {
    uint64_t lo, hi;
    int dev;
  };
  std::vector<R> r;
  size_t last = 0;
  // -1: the runtime does not know the address as device memory
  int owner(uint64_t p) {
    if (!r.empty() && p >= r[last].lo && p < r[last].hi) return r[last].dev;
    for (size_t i = 0; i < r.size(); ++i)
      if (p >= r[i].lo && p < r[i].hi) {
        last = i;
        return r[i].dev;
      }
    hipPointerAttribute_t a{};
    int dev = -1;
    if (hipPointerGetAttributes(&a, reinterpret_cast<void *>(p)) == hipSuccess && a.type == hipMemoryTypeDevice)
      dev = a.device;
    else
      (void)hipGetLastError();
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    R x{p, p + 1, dev};
    if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(p)) == hipSuccess && base && size)
      x = R{(uint64_t)(uintptr_t)base, (uint64_t)(uintptr_t)base + size, dev};
    else
      (void)hipGetLastError();
    r.push_back(x);
    last = r.size() - 1;
    return dev;
  }
};

void partition_cuts(const uint64_t *len, size_t n, int world, uint64_t *cuts) {
  // 3fs_amd/shard.py::partition: prefix = cumsum(float64(lengths)); cut_k = searchsorted(prefix,
  // total * k / world, side="left"), clamped to [cut_{k-1}, n]
  std::vector<double> prefix(n + 1, 0.0);
  for (size_t i = 0; i < n; ++i) prefix[i + 1] = prefix[i] + (double)len[i];
  const double total = prefix[n];
  cuts[0] = 0;
  for (int k = 1; k < world; ++k) {
    const double target = total * (double)k / (double)world;
    uint64_t c = n == 0 ? 0 : (uint64_t)(std::lower_bound(prefix.begin(), prefix.end(), target) - prefix.begin());
    c = std::min<uint64_t>(std::max<uint64_t>(c, cuts[k - 1]), n);
    cuts[k] = c;
  }
  cuts[world] = n;
}

}  // namespace

struct h3c_multi {
  struct Worker {
    int device = 0;
    hipStream_t st = nullptr;
    h3c_hostfed *hf = nullptr;
    std::thread th;
    std::function<int(Worker &)> job;
    int rc = H3C_OK;
    std::string err;
    uint64_t units = 0, bytes = 0;
    double ms = 0;
  };
  std::vector<std::unique_ptr<Worker>> w;
  uint64_t window = 64ull << 20;
  std::mutex call;  // one batch at a time per object (make one object per concurrent caller)
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
  // Mirrors of gen / pending / stop (written under mu): a worker between jobs and a caller waiting for its
  // workers spin on them for a while before blocking on the condition variables, so that back-to-back
  // batches do not pay a futex wake each way (~30 us of a 1.3 ms config-2 call, profiles/r06_bench_default.json)
  std::atomic<uint64_t> agen{0};
  std::atomic<int> apending{0};
  std::atomic<bool> astop{false};
#ifndef H3C_MULTI_SPIN
#define H3C_MULTI_SPIN 1  // 0: block at once (the same-box A/B, scripts/r06_multi_spin_ab.sh)
#endif
  static constexpr double kWorkerSpinUs = H3C_MULTI_SPIN ? 300 : 0, kCallerSpinUs = H3C_MULTI_SPIN ? 20000 : 0;

  template <class F>
  static bool spin_until(F done, double us) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0;; ++k) {
      if (done()) return true;
      __builtin_ia32_pause();
      if ((k & 255) == 255 &&
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > us)
        return false;
    }
  }

  void loop(Worker *me) {
    uint64_t seen = 0;
    for (;;) {
      std::function<int(Worker &)> job;
      spin_until([&] { return astop.load(std::memory_order_acquire) || agen.load(std::memory_order_acquire) != seen; },
                 kWorkerSpinUs);
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_work.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        job = me->job;
      }
      const auto t0 = std::chrono::steady_clock::now();
      int rc = job ? job(*me) : H3C_OK;
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::string err = rc ? std::string(h3c_last_error()) : std::string();
      {
        std::lock_guard<std::mutex> lk(mu);
        me->rc = rc;
        me->err.swap(err);
        me->ms = ms;
        apending.store(--pending, std::memory_order_release);
        if (pending == 0) cv_done.notify_all();
      }
    }
  }

  // Runs jobs[k] on worker k (an empty job is a no-op) and waits for all of them.  Returns the first
  // worker's failure in worker order, with its text as the caller's h3c_last_error().
  int run(std::vector<std::function<int(Worker &)>> jobs) {
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t k = 0; k < w.size(); ++k) {
        w[k]->job = std::move(jobs[k]);
        w[k]->rc = H3C_OK;
      }
      pending = (int)w.size();
      apending.store(pending, std::memory_order_release);
      ++gen;
      agen.store(gen, std::memory_order_release);
    }
    cv_work.notify_all();
    spin_until([&] { return apending.load(std::memory_order_acquire) == 0; }, kCallerSpinUs);
    std::unique_lock<std::mutex> lk(mu);  // (the workers' results were written under mu)
    cv_done.wait(lk, [&] { return pending == 0; });
    for (size_t k = 0; k < w.size(); ++k) w[k]->job = nullptr;
    for (size_t k = 0; k < w.size(); ++k)
      if (w[k]->rc != H3C_OK) {
        const std::string t = "h3c_multi worker " + std::to_string(k) + " (device " + std::to_string(w[k]->device) +
                              "): " + w[k]->err;
        h3c_rt::set_error_text(t.c_str());
        return w[k]->rc;
      }
    return H3C_OK;
  }

  // Worker of every descriptor: the byte-balanced range first, then device-resident payloads moved to a
  // worker on their own device.  out[k] lists worker k's descriptor indices in ascending order.
  int assign(const h3c_desc *d, size_t n, std::vector<std::vector<uint32_t>> &out, bool device_only) {
    const int W = (int)w.size();
    std::vector<uint64_t> len(n), cuts(W + 1);
    for (size_t i = 0; i < n; ++i) len[i] = is_crc(d[i].type) && d[i].ptr ? d[i].len : 0;
    partition_cuts(len.data(), n, W, cuts.data());
    std::vector<int> who(n);
    std::vector<uint64_t> load(W, 0);
    for (int k = 0; k < W; ++k)
      for (uint64_t i = cuts[k]; i < cuts[k + 1]; ++i) {
        who[i] = k;
        load[k] += len[i];
      }
    OwnerCache oc;
    for (size_t i = 0; i < n; ++i) {
      if (!len[i]) continue;
      if (d[i].mem != H3C_MEM_DEVICE) {
        if (device_only) {
          h3c_rt::set_error_text(("h3c_multi_plan_create: descriptor " + std::to_string(i) +
                                  " is not device memory (plans are for resident chunk sets)").c_str());
          return H3C_ERR_INVALID_ARG;
        }
        continue;
      }
      const int o = oc.owner((uint64_t)(uintptr_t)d[i].ptr);
      if (o < 0 || w[who[i]]->device == o) continue;
      int best = -1;
      for (int k = 0; k < W; ++k)
        if (w[k]->device == o && (best < 0 || load[k] < load[best])) best = k;
      if (best < 0) {
        h3c_rt::set_error_text(("h3c_multi: descriptor " + std::to_string(i) + " lives on device " + std::to_string(o) +
                                ", which this engine does not drive").c_str());
        return H3C_ERR_INVALID_ARG;
      }
      load[who[i]] -= len[i];
      load[best] += len[i];
      who[i] = best;
    }
    out.assign(W, {});
    for (size_t i = 0; i < n; ++i) out[who[i]].push_back((uint32_t)i);
    for (int k = 0; k < W; ++k) {
      w[k]->units = out[k].size();
      uint64_t b = 0;
      for (uint32_t i : out[k]) b += len[i];
      w[k]->bytes = b;
    }
    return H3C_OK;
  }
};

#ifndef H3C_MULTI_ZC
#define H3C_MULTI_ZC 1  // 0: plan verifies copy expected / results through the device buffer (the same-box A/B)
#endif
struct h3c_multi_plan {
  h3c_multi *m = nullptr;
  size_t n = 0;
  struct Part {
    std::vector<uint32_t> idx;
    h3c_plan *plan = nullptr;
    char *dbuf = nullptr;  // device [expected | mismatch | out | ok]
    char *hbuf = nullptr;  // pinned mirror of it
    size_t off_mis = 0, off_out = 0, off_ok = 0, bytes = 0;
  };
  std::vector<Part> parts;
};

namespace {

// create (expected == nullptr) or verify over one worker's descriptors, results scattered into the caller's arrays
int worker_batch(h3c_multi::Worker &me, uint64_t window, const h3c_desc *d, const std::vector<uint32_t> &idx,
                 const uint32_t *expected, uint32_t *out_raw, uint8_t *ok, uint64_t *mis_out) {
  *mis_out = 0;
  if (idx.empty()) return H3C_OK;
  // pinned host payloads of one polynomial go through the worker's double-buffered H2D pipeline; the rest
  // (device payloads, pageable or small pinned ones) through the synchronous batch entry on its stream
  std::vector<uint32_t> fed, rest;
  uint64_t fed_bytes = 0;
  uint8_t fed_type = 0;
  bool one_type = true;
  for (uint32_t i : idx) {
    const h3c_desc &x = d[i];
    if (is_crc(x.type) && x.ptr && x.len && x.mem == H3C_MEM_HOST_PINNED) {
      fed.push_back(i);
      fed_bytes += x.len;
      if (fed_type && fed_type != x.type) one_type = false;
      fed_type = x.type;
    } else {
      rest.push_back(i);
    }
  }
  if (fed_bytes < kHostfedMin || !one_type) {
    rest = idx;
    fed.clear();
  }
  auto one = [&](const std::vector<uint32_t> &sel, bool hostfed) -> int {
    if (sel.empty()) return H3C_OK;
    const size_t k = sel.size();
    std::vector<h3c_desc> dd(k);
    std::vector<uint32_t> exp(expected ? k : 0), raw(k);
    std::vector<uint8_t> okv(expected ? k : 0);
    for (size_t j = 0; j < k; ++j) {
      dd[j] = d[sel[j]];
      if (expected) exp[j] = expected[sel[j]];
    }
    uint64_t mis = 0;
    int rc;
    if (hostfed) {
      if (!me.hf) {
        rc = h3c_hostfed_create(me.device, window, &me.hf);
        if (rc) return rc;
      }
      rc = h3c_hostfed_run(me.hf, dd.data(), k, expected ? exp.data() : nullptr, raw.data(),
                           expected ? okv.data() : nullptr, expected ? &mis : nullptr, me.st);
    } else if (expected) {
      rc = h3c_batch_verify(dd.data(), exp.data(), k, raw.data(), okv.data(), &mis, me.st);
    } else {
      rc = h3c_batch_create(dd.data(), k, nullptr, raw.data(), me.st);
    }
    if (rc) return rc;
    for (size_t j = 0; j < k; ++j) {
      out_raw[sel[j]] = raw[j];
      if (expected) ok[sel[j]] = okv[j];
    }
    *mis_out += mis;
    return H3C_OK;
  };
  int rc = one(rest, false);
  if (!rc) rc = one(fed, true);
  return rc;
}

}  // namespace

extern "C" {

int h3c_multi_partition(const uint64_t *lengths, size_t n, int world, uint64_t *cuts) {
  if (world < 1 || !cuts || (n && !lengths)) return H3C_ERR_INVALID_ARG;
  partition_cuts(lengths, n, world, cuts);
  return H3C_OK;
}

int h3c_multi_create(const int *devices, int ndev, uint64_t hostfed_window, h3c_multi **out) {
  if (!out || !devices || ndev < 1 || ndev > 64) return H3C_ERR_INVALID_ARG;
  if (hostfed_window && (hostfed_window < (1u << 20) || hostfed_window % 256)) return H3C_ERR_INVALID_ARG;
  *out = nullptr;
  const int have = h3c_device_count();
  for (int k = 0; k < ndev; ++k)
    if (devices[k] < 0 || devices[k] >= have) {
      h3c_rt::set_error_text(("h3c_multi_create: device " + std::to_string(devices[k]) + " of " +
                              std::to_string(have)).c_str());
      return have ? H3C_ERR_INVALID_ARG : H3C_ERR_NO_DEVICE;
    }
  auto m = std::make_unique<h3c_multi>();
  if (hostfed_window) m->window = hostfed_window;
  std::vector<int> init_rc(ndev, H3C_OK);
  std::vector<std::string> init_err(ndev);
  std::mutex im;
  std::condition_variable icv;
  int started = 0;
  for (int k = 0; k < ndev; ++k) {
    m->w.push_back(std::make_unique<h3c_multi::Worker>());
    h3c_multi::Worker *me = m->w.back().get();
    me->device = devices[k];
    h3c_multi *mp = m.get();
    me->th = std::thread([mp, me, k, &init_rc, &init_err, &im, &icv, &started] {
      int rc = h3c_init(me->device);
      if (!rc && hipSetDevice(me->device) != hipSuccess) rc = H3C_ERR_HIP;
      if (!rc && hipStreamCreateWithFlags(&me->st, hipStreamNonBlocking) != hipSuccess) rc = H3C_ERR_HIP;
      {
        std::lock_guard<std::mutex> lk(im);
        init_rc[k] = rc;
        if (rc) init_err[k] = h3c_last_error();
        ++started;
      }
      icv.notify_all();
      if (!rc) mp->loop(me);
    });
  }
  {
    std::unique_lock<std::mutex> lk(im);
    icv.wait(lk, [&] { return started == ndev; });
  }
  for (int k = 0; k < ndev; ++k)
    if (init_rc[k]) {
      h3c_rt::set_error_text(("h3c_multi_create: device " + std::to_string(devices[k]) + ": " + init_err[k]).c_str());
      const int rc = init_rc[k];
      h3c_multi_destroy(m.release());
      return rc;
    }
  *out = m.release();
  return H3C_OK;
}

void h3c_multi_destroy(h3c_multi *m) {
  if (!m) return;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->stop = true;
    m->astop.store(true, std::memory_order_release);
  }
  m->cv_work.notify_all();
  for (auto &w : m->w)
    if (w->th.joinable()) w->th.join();
  for (auto &w : m->w) {
    if (w->hf) h3c_hostfed_destroy(w->hf);
    if (w->st) {
      (void)hipSetDevice(w->device);
      (void)hipStreamDestroy(w->st);
    }
  }
  delete m;
}

int h3c_multi_workers(const h3c_multi *m) { return m ? (int)m->w.size() : 0; }

int h3c_multi_last_stats(const h3c_multi *m, uint64_t *units, uint64_t *bytes, double *ms) {
  if (!m) return H3C_ERR_INVALID_ARG;
  for (size_t k = 0; k < m->w.size(); ++k) {
    if (units) units[k] = m->w[k]->units;
    if (bytes) bytes[k] = m->w[k]->bytes;
    if (ms) ms[k] = m->w[k]->ms;
  }
  return H3C_OK;
}

static int multi_batch(h3c_multi *m, const h3c_desc *d, size_t n, const uint32_t *expected, uint8_t *out_type,
                       uint32_t *out_raw, uint8_t *ok, uint64_t *n_mismatch) {
  if (!m || (n && (!d || !out_raw)) || (expected && !ok)) return H3C_ERR_INVALID_ARG;
  if (n_mismatch) *n_mismatch = 0;
  if (n == 0) return H3C_OK;
  if (n > 0xFFFFFFF0u) return H3C_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> call(m->call);
  std::vector<std::vector<uint32_t>> idx;
  int rc = m->assign(d, n, idx, false);
  if (rc) return rc;
  std::vector<uint64_t> mis(m->w.size(), 0);
  std::vector<std::function<int(h3c_multi::Worker &)>> jobs(m->w.size());
  for (size_t k = 0; k < m->w.size(); ++k)
    jobs[k] = [&, k](h3c_multi::Worker &me) {
      return worker_batch(me, m->window, d, idx[k], expected, out_raw, ok, &mis[k]);
    };
  rc = m->run(std::move(jobs));
  if (rc) return rc;
  if (out_type)  // ChecksumInfo::create's type (Common.h:146-172): NONE for NONE or a null payload
    for (size_t i = 0; i < n; ++i)
      out_type[i] = is_crc(d[i].type) && !(d[i].ptr == nullptr && d[i].len > 0) ? d[i].type : (uint8_t)H3C_TYPE_NONE;
  if (n_mismatch)
    for (uint64_t x : mis) *n_mismatch += x;
  return H3C_OK;
}

int h3c_multi_batch_create(h3c_multi *m, const h3c_desc *d, size_t n, uint8_t *out_type, uint32_t *out_raw) {
  return multi_batch(m, d, n, nullptr, out_type, out_raw, nullptr, nullptr);
}

int h3c_multi_verify(h3c_multi *m, const h3c_desc *d, size_t n, const uint32_t *expected_raw, uint32_t *out_raw,
                     uint8_t *ok, uint64_t *n_mismatch) {
  if (n && (!expected_raw || !ok)) return H3C_ERR_INVALID_ARG;
  return multi_batch(m, d, n, expected_raw, nullptr, out_raw, ok, n_mismatch);
}

int h3c_multi_update_ios(h3c_multi *m, uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks,
                         const h3c_update_io *ios, uint32_t n, h3c_update_result *results, uint32_t flags,
                         h3c_update_counters *counters) {
  if (counters) std::memset(counters, 0, sizeof(*counters));
  if (!m || (nchunks && !chunks) || (n && (!ios || !results))) return H3C_ERR_INVALID_ARG;
  for (uint32_t c = 0; c < nchunks; ++c)  // as h3c_update_ios: the whole call fails before any work
    if (chunks[c].size > chunks[c].chunk_size) {
      h3c_rt::set_error_text("h3c_multi_update_ios: a chunk's size exceeds its chunk_size");
      return H3C_ERR_INVALID_ARG;
    }
  if (n == 0) return H3C_OK;
  std::lock_guard<std::mutex> call(m->call);
  const int W = (int)m->w.size();
  // chunks: byte-balanced by capacity (3fs_amd/shard.py::partition_updates), then each chunk to a worker on
  // the device that holds its bytes
  std::vector<uint64_t> cap(nchunks), cuts(W + 1);
  for (uint32_t c = 0; c < nchunks; ++c) cap[c] = chunks[c].chunk_size;
  partition_cuts(cap.data(), nchunks, W, cuts.data());
  std::vector<int> owner(nchunks);
  std::vector<uint64_t> load(W, 0);
  for (int k = 0; k < W; ++k)
    for (uint64_t c = cuts[k]; c < cuts[k + 1]; ++c) {
      owner[c] = k;
      load[k] += cap[c];
    }
  OwnerCache oc;
  for (uint32_t c = 0; c < nchunks; ++c) {
    if (!chunks[c].base) continue;
    const int o = oc.owner(chunks[c].base);
    if (o < 0 || m->w[owner[c]]->device == o) continue;
    int best = -1;
    for (int k = 0; k < W; ++k)
      if (m->w[k]->device == o && (best < 0 || load[k] < load[best])) best = k;
    if (best < 0) {
      h3c_rt::set_error_text(("h3c_multi_update_ios: chunk " + std::to_string(c) + " lives on device " +
                              std::to_string(o) + ", which this engine does not drive").c_str());
      return H3C_ERR_INVALID_ARG;
    }
    load[owner[c]] -= cap[c];
    load[best] += cap[c];
    owner[c] = best;
  }
  std::vector<std::vector<uint32_t>> cidx(W), oidx(W);
  std::vector<uint32_t> local(nchunks);
  for (uint32_t c = 0; c < nchunks; ++c) {
    local[c] = (uint32_t)cidx[owner[c]].size();
    cidx[owner[c]].push_back(c);
  }
  for (uint32_t i = 0; i < n; ++i) {
    // an op naming no chunk of the table goes to worker 0, where it stays out of range (kInvalidArg)
    const int k = ios[i].chunk < nchunks ? owner[ios[i].chunk] : 0;
    oidx[k].push_back(i);
    // a payload on another device than its chunk's worker cannot be read there
    if (ios[i].kind == H3C_UPD_WRITE && ios[i].length && ios[i].payload && ios[i].chunk < nchunks) {
      const int o = oc.owner(ios[i].payload);
      if (o >= 0 && o != m->w[k]->device) {
        h3c_rt::set_error_text(("h3c_multi_update_ios: op " + std::to_string(i) + "'s payload lives on device " +
                                std::to_string(o) + ", its chunk on device " + std::to_string(m->w[k]->device)).c_str());
        return H3C_ERR_INVALID_ARG;
      }
    }
  }
  std::vector<h3c_update_counters> ctr(W);
  std::vector<std::function<int(h3c_multi::Worker &)>> jobs(W);
  for (int k = 0; k < W; ++k) {
    m->w[k]->units = oidx[k].size();
    m->w[k]->bytes = 0;
    for (uint32_t i : oidx[k])
      if (ios[i].kind == H3C_UPD_WRITE) m->w[k]->bytes += 3ull * ios[i].length;  // payload + old bytes + new bytes
    std::memset(&ctr[k], 0, sizeof(ctr[k]));
    if (oidx[k].empty()) continue;  // chunks no op reaches keep their state (as in one h3c_update_ios call)
    jobs[k] = [&, k](h3c_multi::Worker &me) -> int {
      const std::vector<uint32_t> &cs = cidx[k], &os = oidx[k];
      std::vector<h3c_chunk_state> lc(cs.size());
      for (size_t j = 0; j < cs.size(); ++j) lc[j] = chunks[cs[j]];
      std::vector<h3c_update_io> lo(os.size());
      for (size_t j = 0; j < os.size(); ++j) {
        lo[j] = ios[os[j]];
        if (lo[j].chunk < nchunks) lo[j].chunk = local[lo[j].chunk];
      }
      std::vector<h3c_update_result> lr(os.size());
      const int rc = h3c_update_ios_ex(poly_type, lc.data(), (uint32_t)lc.size(), lo.data(), (uint32_t)lo.size(),
                                       lr.data(), flags, &ctr[k], me.st);
      if (rc) return rc;
      for (size_t j = 0; j < cs.size(); ++j) chunks[cs[j]] = lc[j];
      for (size_t j = 0; j < os.size(); ++j) results[os[j]] = lr[j];
      return H3C_OK;
    };
  }
  const int rc = m->run(std::move(jobs));
  if (rc) return rc;
  if (counters)
    for (const h3c_update_counters &c : ctr) {
      counters->none += c.none;
      counters->reuse += c.reuse;
      counters->combine += c.combine;
      counters->read_chunk += c.read_chunk;
      counters->recalculate += c.recalculate;
      counters->checksum_mismatch += c.checksum_mismatch;
      counters->invalid += c.invalid;
      counters->stale_chunks += c.stale_chunks;
    }
  return H3C_OK;
}

int h3c_multi_plan_create(h3c_multi *m, const h3c_desc *d, size_t n, h3c_multi_plan **out) {
  if (!m || !out || (n && !d) || n > 0xFFFFFFF0u) return H3C_ERR_INVALID_ARG;
  *out = nullptr;
  std::lock_guard<std::mutex> call(m->call);
  std::vector<std::vector<uint32_t>> idx;
  int rc = m->assign(d, n, idx, true);
  if (rc) return rc;
  auto p = std::make_unique<h3c_multi_plan>();
  p->m = m;
  p->n = n;
  p->parts.resize(m->w.size());
  std::vector<std::function<int(h3c_multi::Worker &)>> jobs(m->w.size());
  for (size_t k = 0; k < m->w.size(); ++k) {
    p->parts[k].idx = std::move(idx[k]);
    jobs[k] = [&, k](h3c_multi::Worker &me) -> int {
      h3c_multi_plan::Part &pt = p->parts[k];
      const size_t c = pt.idx.size();
      if (!c) return H3C_OK;
      std::vector<h3c_desc> dd(c);
      for (size_t j = 0; j < c; ++j) dd[j] = d[pt.idx[j]];
      int r = h3c_plan_create(dd.data(), c, me.device, &pt.plan);
      if (r) return r;
      auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
      pt.off_mis = al(4 * c);
      pt.off_out = pt.off_mis + 256;
      pt.off_ok = al(pt.off_out + 4 * c);
      pt.bytes = al(pt.off_ok + c);
      if (hipMalloc(reinterpret_cast<void **>(&pt.dbuf), pt.bytes) != hipSuccess ||
          hipHostMalloc(reinterpret_cast<void **>(&pt.hbuf), pt.bytes, hipHostMallocDefault) != hipSuccess) {
        h3c_rt::set_error_text("h3c_multi_plan_create: result buffers");
        return H3C_ERR_HIP;
      }
      return H3C_OK;
    };
  }
  rc = m->run(std::move(jobs));
  if (rc) {
    h3c_multi_plan_destroy(p.release());
    return rc;
  }
  *out = p.release();
  return H3C_OK;
}

int h3c_multi_plan_verify(h3c_multi_plan *p, const uint32_t *expected_raw, uint32_t *out_raw, uint8_t *ok,
                          uint64_t *n_mismatch) {
  if (!p || (p->n && (!out_raw || (expected_raw && !ok)))) return H3C_ERR_INVALID_ARG;
  if (n_mismatch) *n_mismatch = 0;
  if (p->n == 0) return H3C_OK;
  h3c_multi *m = p->m;
  std::lock_guard<std::mutex> call(m->call);
  std::vector<uint64_t> mis(m->w.size(), 0);
  std::vector<std::function<int(h3c_multi::Worker &)>> jobs(m->w.size());
  for (size_t k = 0; k < m->w.size(); ++k) {
    m->w[k]->units = p->parts[k].idx.size();
    m->w[k]->bytes = p->parts[k].plan ? h3c_plan_bytes(p->parts[k].plan) : 0;
    jobs[k] = [&, k](h3c_multi::Worker &me) -> int {
      h3c_multi_plan::Part &pt = p->parts[k];
      const size_t c = pt.idx.size();
      if (!c) return H3C_OK;
      uint32_t *hexp = reinterpret_cast<uint32_t *>(pt.hbuf);
      if (expected_raw)
        for (size_t j = 0; j < c; ++j) hexp[j] = expected_raw[pt.idx[j]];
#if H3C_MULTI_ZC
      // in place: the kernels read the expected values from the pinned mirror and write the results into it
      // (each wave loads its chunk's expected value before the segment; the stores are posted), no copies on
      // the call's critical path; the mismatch count is taken from `ok` below
      int r = h3c_plan_run(pt.plan, expected_raw ? hexp : nullptr, reinterpret_cast<uint32_t *>(pt.hbuf + pt.off_out),
                           expected_raw ? reinterpret_cast<uint8_t *>(pt.hbuf + pt.off_ok) : nullptr, nullptr, me.st);
#else
      std::memset(pt.hbuf + pt.off_mis, 0, 4);
      hipError_t e = hipMemcpyAsync(pt.dbuf, pt.hbuf, pt.off_out, hipMemcpyHostToDevice, me.st);
      int r = e == hipSuccess ? H3C_OK : H3C_ERR_HIP;
      if (!r)
        r = h3c_plan_run(pt.plan, expected_raw ? reinterpret_cast<uint32_t *>(pt.dbuf) : nullptr,
                         reinterpret_cast<uint32_t *>(pt.dbuf + pt.off_out),
                         expected_raw ? reinterpret_cast<uint8_t *>(pt.dbuf + pt.off_ok) : nullptr,
                         expected_raw ? reinterpret_cast<uint32_t *>(pt.dbuf + pt.off_mis) : nullptr, me.st);
      if (!r && hipMemcpyAsync(pt.hbuf + pt.off_mis, pt.dbuf + pt.off_mis, pt.bytes - pt.off_mis, hipMemcpyDeviceToHost,
                               me.st) != hipSuccess)
        r = H3C_ERR_HIP;
#endif
      if (hipStreamSynchronize(me.st) != hipSuccess && !r) r = H3C_ERR_HIP;
      if (r) {
        if (r == H3C_ERR_HIP) h3c_rt::set_error_text("h3c_multi_plan_verify: a copy or the stream failed");
        return r;
      }
      const uint32_t *hout = reinterpret_cast<const uint32_t *>(pt.hbuf + pt.off_out);
      for (size_t j = 0; j < c; ++j) out_raw[pt.idx[j]] = hout[j];
      if (expected_raw) {
        const uint8_t *hok = reinterpret_cast<const uint8_t *>(pt.hbuf + pt.off_ok);
        uint32_t x = 0;
        for (size_t j = 0; j < c; ++j) {
          ok[pt.idx[j]] = hok[j];
          x += H3C_MULTI_ZC && hok[j] == 0;
        }
        if (!H3C_MULTI_ZC) std::memcpy(&x, pt.hbuf + pt.off_mis, 4);
        mis[k] = x;
      }
      return H3C_OK;
    };
  }
  const int rc = m->run(std::move(jobs));
  if (rc) return rc;
  if (n_mismatch)
    for (uint64_t x : mis) *n_mismatch += x;
  return H3C_OK;
}

void h3c_multi_plan_destroy(h3c_multi_plan *p) {
  if (!p) return;
  for (size_t k = 0; k < p->parts.size(); ++k) {
    h3c_multi_plan::Part &pt = p->parts[k];
    if (pt.plan) h3c_plan_destroy(pt.plan);
    if (pt.dbuf || pt.hbuf) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(p->m->w[k]->device);
      if (pt.dbuf) (void)hipFree(pt.dbuf);
      if (pt.hbuf) (void)hipHostFree(pt.hbuf);
      (void)hipSetDevice(prev);
    }
  }
  delete p;
}

}  // extern "C"
