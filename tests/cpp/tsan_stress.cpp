// tsan_stress.cpp -- host-side ThreadSanitizer stress of the engine's shared host state (VERDICT
// r1 #8): the device / pinned lease pools, the coalescing queue, the per-thread UpdateIO aux
// streams, the block-update shift-table cache, plan create / destroy, the profiling records and
// (round 4) the UpdateIO fast branch's per-thread scratch, graph capture gate and outcome polling,
// (round 5) the UpdateIO aligned sub-branch and the block path's per-stream scratch (the default
// stream's one shared by eight threads), from 16 threads at once (half on their own streams, half on
// the default stream).
// Every result is checked against a bitwise CRC32C in this file.  Built by
// scripts/tsan_host.sh with the host code instrumented (-Xarch_host -fsanitize=thread); GPU
// code is built normally.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "h3c_crc.h"

namespace {

uint32_t crc_bitwise(const uint8_t *d, size_t n, uint32_t c) {  // raw register, reflected 0x82F63B78
  for (size_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return c;
}

std::atomic<int> g_errors{0};

void fail(int t, const char *what, int rc) {
  std::fprintf(stderr, "thread %d: %s (rc %d: %s)\n", t, what, rc, h3c_last_error());
  g_errors.fetch_add(1);
}

void worker(int t, int iters) {
  hipStream_t st = nullptr;
  if (t % 2 && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return fail(t, "stream", -1);
  void *sp = st;
  uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
  auto rnd = [&] {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    return x;
  };
  const size_t nb = 3, len = 48 << 10;
  std::vector<uint8_t> host(nb * len);
  uint8_t *dev = nullptr;
  if (hipMalloc(&dev, nb * len) != hipSuccess) return fail(t, "hipMalloc", -1);
  for (int it = 0; it < iters; ++it) {
    for (auto &b : host) b = (uint8_t)rnd();
    if (hipMemcpy(dev, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) return fail(t, "h2d", -1);
    std::vector<uint32_t> want(nb);
    std::vector<h3c_desc> hd(nb), dd(nb);
    for (size_t i = 0; i < nb; ++i) {
      want[i] = crc_bitwise(host.data() + i * len, len - i, 0xFFFFFFFFu);
      hd[i] = h3c_desc{host.data() + i * len, len - i, 0xFFFFFFFFu, H3C_TYPE_CRC32C, H3C_MEM_HOST_PAGEABLE, 0};
      dd[i] = h3c_desc{dev + i * len, len - i, 0xFFFFFFFFu, H3C_TYPE_CRC32C, H3C_MEM_DEVICE, 0};
    }
    // synchronous batch API, host and device payloads (coalesced when on and st == NULL)
    std::vector<uint32_t> raw(nb), exp(want);
    std::vector<uint8_t> ok(nb), ty(nb);
    exp[it % nb] ^= 1;
    uint64_t nbad = 0;
    int rc = h3c_batch_verify(hd.data(), exp.data(), nb, raw.data(), ok.data(), &nbad, sp);
    if (rc || raw != want || nbad != 1 || ok[it % nb]) fail(t, "verify host", rc);
    rc = h3c_batch_create(dd.data(), nb, ty.data(), raw.data(), sp);
    if (rc || raw != want) fail(t, "create device", rc);
    uint32_t one = 0;
    rc = h3c_crc32c(host.data(), len, 0xFFFFFFFFu, &one, sp);
    if (rc || one != want[0]) fail(t, "crc32c", rc);
    // a plan over the device buffers
    h3c_plan *plan = nullptr;
    rc = h3c_plan_create(dd.data(), nb, 0, &plan);
    if (rc) {
      fail(t, "plan_create", rc);
    } else {
      uint32_t *d_out = nullptr;
      if (hipMalloc(&d_out, 4 * nb) != hipSuccess) return fail(t, "hipMalloc out", -1);
      rc = h3c_plan_run(plan, nullptr, d_out, nullptr, nullptr, sp);
      if (!rc && hipStreamSynchronize(st) == hipSuccess &&
          hipMemcpy(raw.data(), d_out, 4 * nb, hipMemcpyDeviceToHost) == hipSuccess) {
        if (raw != want) fail(t, "plan_run", 0);
      } else {
        fail(t, "plan_run", rc);
      }
      (void)hipFree(d_out);
      h3c_plan_destroy(plan);
    }
    // general updates on the device buffer (a single chunk per segment), host arrays
    std::vector<h3c_chunk_state> cs(nb);
    for (size_t i = 0; i < nb; ++i)
      cs[i] = h3c_chunk_state{(uint64_t)(uintptr_t)(dev + i * len), (uint32_t)len, (uint32_t)(len - i), want[i],
                              H3C_TYPE_CRC32C, {0, 0, 0}};
    std::vector<uint8_t> pay(4096);
    for (auto &b : pay) b = (uint8_t)rnd();
    uint8_t *d_pay = nullptr;
    if (hipMalloc(&d_pay, pay.size()) != hipSuccess || hipMemcpy(d_pay, pay.data(), pay.size(), hipMemcpyHostToDevice))
      return fail(t, "payload", -1);
    std::vector<h3c_update_io> ios(nb);
    for (size_t i = 0; i < nb; ++i) {
      const uint32_t off = (uint32_t)(rnd() % (len - pay.size()));
      ios[i] = h3c_update_io{(uint64_t)(uintptr_t)d_pay, (uint32_t)i, off, (uint32_t)pay.size(),
                             crc_bitwise(pay.data(), pay.size(), 0xFFFFFFFFu), H3C_TYPE_CRC32C, H3C_UPD_WRITE, 0,
                             0, 0};
      std::memcpy(host.data() + i * len + off, pay.data(), pay.size());
    }
    std::vector<h3c_update_result> res(nb);
    h3c_update_counters ctr;
    rc = h3c_update_ios_ex(H3C_TYPE_CRC32C, cs.data(), (uint32_t)nb, ios.data(), (uint32_t)nb, res.data(),
                           (it % 3 == 0) ? H3C_UPD_EXACT : 0u, &ctr, sp);
    if (rc) fail(t, "update_ios", rc);
    for (size_t i = 0; i < nb && !rc; ++i) {
      const size_t sz = std::max<size_t>(len - i, ios[i].offset + pay.size());
      if (res[i].status || cs[i].value != crc_bitwise(host.data() + i * len, sz, 0xFFFFFFFFu)) fail(t, "update value", 0);
    }
    // the fast branch on device tables (aligned one-block writes: h3c_update_ios_dev), as one graph per
    // batch on odd iterations (captured beside the other threads' legacy-stream calls); the call returns
    // at the batch's outcome, so the tables are read back after the stream is synchronised
    if (!rc) {
      std::vector<h3c_update_io> fios(nb);
      for (size_t i = 0; i < nb; ++i) {
        const uint32_t b = (uint32_t)(rnd() % (cs[i].size / 4096 - 1)) + 1;  // (never a whole-chunk rewrite)
        fios[i] = h3c_update_io{(uint64_t)(uintptr_t)d_pay, (uint32_t)i, b * 4096u, 4096u,
                                crc_bitwise(pay.data(), pay.size(), 0xFFFFFFFFu), H3C_TYPE_CRC32C, H3C_UPD_WRITE, 0,
                                0, 0};
        std::memcpy(host.data() + i * len + b * 4096u, pay.data(), pay.size());
      }
      h3c_chunk_state *d_cs = nullptr;
      h3c_update_io *d_ios = nullptr;
      h3c_update_result *d_res = nullptr;
      if (hipMalloc(&d_cs, sizeof(h3c_chunk_state) * nb) != hipSuccess ||
          hipMalloc(&d_ios, sizeof(h3c_update_io) * nb) != hipSuccess ||
          hipMalloc(&d_res, sizeof(h3c_update_result) * nb) != hipSuccess ||
          hipMemcpy(d_cs, cs.data(), sizeof(h3c_chunk_state) * nb, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d_ios, fios.data(), sizeof(h3c_update_io) * nb, hipMemcpyHostToDevice) != hipSuccess)
        return fail(t, "fast tables", -1);
      rc = h3c_update_ios_dev(H3C_TYPE_CRC32C, d_cs, (uint32_t)nb, d_ios, (uint32_t)nb, d_res,
                              (it % 2) ? H3C_UPD_GRAPHS : 0u, nullptr, sp);
      if (rc) fail(t, "update_ios_dev", rc);
      if (hipStreamSynchronize(st) != hipSuccess ||
          hipMemcpy(cs.data(), d_cs, sizeof(h3c_chunk_state) * nb, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(res.data(), d_res, sizeof(h3c_update_result) * nb, hipMemcpyDeviceToHost) != hipSuccess)
        fail(t, "fast read back", -1);
      for (size_t i = 0; i < nb && !rc; ++i)
        if (res[i].status || cs[i].value != crc_bitwise(host.data() + i * len, cs[i].size, 0xFFFFFFFFu))
          fail(t, "fast update value", 0);
      (void)hipFree(d_cs);
      (void)hipFree(d_ios);
      (void)hipFree(d_res);
    }
    (void)hipFree(d_pay);
    // block-aligned updates (h3c_update_blocks_ex): 4 chunks of 64 KiB, random 4 KiB writes; the fused path's
    // per-stream scratch, shared on the default stream by the even threads
    {
      const uint32_t bc = 4, blen = 64 << 10, bpc = blen / 4096, nw = 1 + (uint32_t)(rnd() % 200);
      std::vector<uint8_t> bh(bc * blen), bp((size_t)nw * 4096);
      for (auto &b : bh) b = (uint8_t)rnd();
      for (auto &b : bp) b = (uint8_t)rnd();
      std::vector<uint32_t> wc(nw), wb(nw), raw0(bc), fin(bc);
      std::vector<uint64_t> bases(bc);
      for (uint32_t i = 0; i < nw; ++i) wc[i] = (uint32_t)(rnd() % bc), wb[i] = (uint32_t)(rnd() % bpc);
      for (uint32_t c = 0; c < bc; ++c) raw0[c] = crc_bitwise(bh.data() + (size_t)c * blen, blen, 0xFFFFFFFFu);
      const size_t wsb = h3c_update_workspace_bytes(nw, bc, blen, 4096);
      uint8_t *d_ch = nullptr, *d_bp = nullptr, *d_ws = nullptr;
      uint32_t *d_u = nullptr;  // raw_in, raw_out, chunk idx, block idx, out_raw
      uint64_t *d_bases = nullptr;
      if (hipMalloc(&d_ch, bh.size()) != hipSuccess || hipMalloc(&d_bp, bp.size()) != hipSuccess ||
          hipMalloc(&d_ws, wsb) != hipSuccess || hipMalloc(&d_u, 4 * (2 * bc + 3 * nw)) != hipSuccess ||
          hipMalloc(&d_bases, 8 * bc) != hipSuccess)
        return fail(t, "block tables", -1);
      for (uint32_t c = 0; c < bc; ++c) bases[c] = (uint64_t)(uintptr_t)(d_ch + (size_t)c * blen);
      uint32_t *d_rin = d_u, *d_rout = d_u + bc, *d_wc = d_u + 2 * bc, *d_wb = d_wc + nw, *d_out = d_wb + nw;
      if (hipMemcpy(d_ch, bh.data(), bh.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d_bp, bp.data(), bp.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d_rin, raw0.data(), 4 * bc, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d_wc, wc.data(), 4 * nw, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d_wb, wb.data(), 4 * nw, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d_bases, bases.data(), 8 * bc, hipMemcpyHostToDevice) != hipSuccess)
        return fail(t, "block upload", -1);
      rc = h3c_update_blocks_ex(H3C_TYPE_CRC32C, d_bases, bc, blen, 4096, d_rin, d_wc, d_wb, d_bp, nw, d_out, d_rout,
                                d_ws, wsb, nullptr, 0u, nullptr, sp);
      if (rc) fail(t, "update_blocks", rc);
      for (uint32_t i = 0; i < nw; ++i)
        std::memcpy(bh.data() + (size_t)wc[i] * blen + (size_t)wb[i] * 4096, bp.data() + (size_t)i * 4096, 4096);
      if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(fin.data(), d_rout, 4 * bc, hipMemcpyDeviceToHost) != hipSuccess)
        fail(t, "block read back", -1);
      for (uint32_t c = 0; c < bc && !rc; ++c)
        if (fin[c] != crc_bitwise(bh.data() + (size_t)c * blen, blen, 0xFFFFFFFFu)) fail(t, "block update value", 0);
      (void)hipFree(d_ch), (void)hipFree(d_bp), (void)hipFree(d_ws), (void)hipFree(d_u), (void)hipFree(d_bases);
    }
    if (t == 0 && it % 4 == 1) h3c_set_coalescing(it % 8 == 1);  // flip the queue under load
    if (t == 1) {  // profiling records: enable, read, disable while others launch
      h3c_profile_enable(1);
      double ms;
      uint64_t l, b;
      (void)h3c_profile_read(H3C_PROF_SEG, &ms, &l, &b, 1);
      h3c_profile_enable(0);
    }
  }
  (void)hipFree(dev);
  if (st) (void)hipStreamDestroy(st);
}

}  // namespace

int g_selftest_racy = 0;  // "selftest": an unsynchronised counter, so the log shows TSAN is live

int main(int argc, char **argv) {
  if (argc > 1 && std::strcmp(argv[1], "selftest") == 0) {
    std::thread a([] { for (int i = 0; i < 100000; ++i) ++g_selftest_racy; });
    std::thread b([] { for (int i = 0; i < 100000; ++i) ++g_selftest_racy; });
    a.join();
    b.join();
    std::printf("tsan selftest: racy counter %d (TSAN must report one data race above)\n", g_selftest_racy);
    return 0;
  }
  const int threads = argc > 1 ? std::atoi(argv[1]) : 16, iters = argc > 2 ? std::atoi(argv[2]) : 12;
  if (h3c_init(0)) {
    std::fprintf(stderr, "no device\n");
    return 2;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) th.emplace_back(worker, t, iters);
  for (auto &x : th) x.join();
  h3c_set_coalescing(0);
  std::printf("tsan_stress: %d threads x %d iterations, %d errors; UpdateIO graph replays %llu, captures %llu, "
              "capture failures %llu, fast-branch batches %llu\n",
              threads, iters, g_errors.load(), (unsigned long long)h3c_diag_counter(0),
              (unsigned long long)h3c_diag_counter(1), (unsigned long long)h3c_diag_counter(2),
              (unsigned long long)h3c_diag_counter(7));
  return g_errors.load() ? 1 : 0;
}
