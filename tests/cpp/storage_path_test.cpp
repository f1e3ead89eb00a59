// C++ mirror test: the storage types of include/h3c_storage.hpp driven the way the
// reference's own tests drive ChunkReplica / AioReadJob, checked against the CPU oracle.
// usage: storage_path_test cpu|gpu     (gpu mode needs a HIP device)
//
//   verify_checksum_patterns   TestStorageClientInterface.cc:357-463 (VerifyChecksum):
//                              SEQ / JUMP / RAND writes of random length into one chunk,
//                              the write checksum, the chunk checksum, a read of the written
//                              range and a whole-chunk read, all against folly::crc32c
//                              (oracle), one update at a time as the test does
//   batched_vs_replica         the same three traces in ONE ChunkReplicaBatch::update,
//                              every result against orc_chunk_replica_update op by op
//   truncate_extend_errors     TRUNCATE / EXTEND / range / mismatch cases (ChunkReplica.cc:131-294)
//   recalculate_read           AioReadJob::setResult's recalculate verify (BatchReadJob.cc:43-55)
//   large_parallel_batch       20000 mixed UpdateIOs (the parallel host pass) vs the replica oracle
//   serde                      Checksum::calcSerde (MessageHeader.h:32-37)
//   data_iterator              ChecksumInfo::create over a DataIterator (Common.h:120-172):
//                              1 MiB memory slices, ragged pieces, short / overlong iteration
//   version_gate               VersionGate: ChunkReplica::update / commit's version and state checks
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/h3c_storage.hpp"
#include "../../oracle/crc_oracle.h"

static int fails = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                         \
    }                                                                  \
  } while (0)

using namespace h3c;

static uint32_t folly_crc32c(const uint8_t *d, size_t n, uint32_t start = ~0U) { return orc_crc32c_sse42(d, n, start); }

static std::vector<uint8_t> d2h(const uint8_t *dev, size_t n) {
  std::vector<uint8_t> h(n);
  if (n) CHECK(hipMemcpy(h.data(), dev, n, hipMemcpyDeviceToHost) == hipSuccess);
  return h;
}

// A device chunk store: `count` chunks of `chunkSize` bytes in one allocation.
struct DeviceChunks {
  uint8_t *base = nullptr;
  uint32_t chunkSize;
  std::vector<ChunkMetadata> metas;
  DeviceChunks(uint32_t count, uint32_t chunkSize_) : chunkSize(chunkSize_), metas(count) {
    CHECK(hipMalloc(&base, (size_t)count * chunkSize) == hipSuccess);
    CHECK(hipMemset(base, 0, (size_t)count * chunkSize) == hipSuccess);
    for (uint32_t c = 0; c < count; ++c) {
      metas[c].bytes = base + (size_t)c * chunkSize;
      metas[c].chunkSize = chunkSize;
    }
  }
  ~DeviceChunks() { (void)hipFree(base); }
};

struct Write {
  uint32_t offset, length;
  std::vector<uint8_t> data;
};

// The offsets / lengths of TestStorageClientInterface.cc:387-421 with std::mt19937_64 in
// place of folly::Random; writeData keeps its previous tail bytes as in the test (the fill
// loop stops 8 bytes short).
static std::vector<Write> make_trace(int pattern, uint32_t chunkSize, std::mt19937_64 &rng) {
  auto rand64 = [&](uint64_t lo, uint64_t hi) { return hi <= lo ? lo : lo + rng() % (hi - lo); };
  std::vector<uint8_t> writeData(chunkSize, 0xFF);
  std::vector<Write> out;
  size_t offset = 0, length = 0;
  for (int w = 1; w <= 100; ++w) {
    if (pattern == 1) offset += length;
    else if (pattern == 2) offset += length + rand64(0, length / 2);
    else offset = rand64(0, chunkSize);
    if (offset + 1 >= chunkSize) continue;
    length = rand64(1, (chunkSize - offset) / 2);
    for (size_t b = 0; b + sizeof(uint64_t) < length; b += sizeof(uint64_t)) {
      const uint64_t r = rng();
      std::memcpy(&writeData[b], &r, 8);
    }
    out.push_back(Write{(uint32_t)offset, (uint32_t)length, std::vector<uint8_t>(writeData.begin(), writeData.begin() + length)});
  }
  return out;
}

static void verify_checksum_patterns(uint32_t chunkSize) {
  std::mt19937_64 rng(357);
  DeviceChunks store(3, chunkSize);
  uint8_t *payload = nullptr;
  CHECK(hipMalloc(&payload, chunkSize) == hipSuccess);
  int nwrites = 0;
  for (int pattern = 1; pattern <= 3; ++pattern) {
    const uint32_t chunk = pattern - 1;
    std::vector<uint8_t> chunkData;
    for (const Write &w : make_trace(pattern, chunkSize, rng)) {
      ++nwrites;
      // the client's write checksum (StorageClientImpl: ChecksumInfo::create over the user buffer)
      const ChecksumInfo local = ChecksumInfo::create(ChecksumType::CRC32C, w.data.data(), w.length, ~0U,
                                                      H3C_MEM_HOST_PAGEABLE);
      CHECK(folly_crc32c(w.data.data(), w.length) == local.value);
      CHECK(hipMemcpy(payload, w.data.data(), w.length, hipMemcpyHostToDevice) == hipSuccess);
      UpdateIO io;
      io.offset = w.offset;
      io.length = w.length;
      io.chunk = chunk;
      io.checksum = local;
      io.data = payload;
      std::vector<IOResult> res;
      CHECK(ChunkReplicaBatch::update(store.metas, {io}, res) == H3C_OK);
      CHECK(res.size() == 1 && res[0].ok());
      CHECK(res[0].length == w.length);  // ASSERT_RESULT_EQ(writeIO.length, writeIO.result.lengthInfo)
      if (w.offset + w.length > chunkData.size()) chunkData.resize(w.offset + w.length);
      std::memcpy(&chunkData[w.offset], w.data.data(), w.length);
      CHECK(folly_crc32c(chunkData.data(), chunkData.size()) == res[0].checksum.value);
      const ChunkMetadata &m = store.metas[chunk];
      CHECK(m.size == chunkData.size() && m.checksum() == res[0].checksum);

      // read back the write data, then the entire chunk (read length clamps to meta.size)
      std::vector<ReadJob> jobs(2);
      jobs[0] = ReadJob{m.bytes + w.offset, H3C_MEM_DEVICE, w.offset, w.length, m.size, m.checksum()};
      jobs[1] = ReadJob{m.bytes, H3C_MEM_DEVICE, 0, m.size, m.size, m.checksum()};
      std::vector<IOResult> rr;
      CHECK(BatchReadResults::setResults(ChecksumType::CRC32C, false, jobs, rr) == H3C_OK);
      CHECK(rr.size() == 2 && rr[0].ok() && rr[1].ok());
      const std::vector<uint8_t> readData = d2h(m.bytes + w.offset, w.length);
      CHECK(folly_crc32c(readData.data(), readData.size()) == rr[0].checksum.value);
      CHECK(local.value == rr[0].checksum.value);
      const std::vector<uint8_t> whole = d2h(m.bytes, m.size);
      CHECK(whole == chunkData);
      CHECK(folly_crc32c(whole.data(), whole.size()) == rr[1].checksum.value);
      CHECK(res[0].checksum.value == rr[1].checksum.value);
    }
  }
  CHECK(nwrites > 50);
  (void)hipFree(payload);
}

// One batch holding all three traces interleaved, vs the oracle's ChunkReplica::update op by op.
static void batched_vs_replica(uint32_t chunkSize) {
  std::mt19937_64 rng(4242);
  std::vector<std::vector<Write>> traces;
  for (int p = 1; p <= 3; ++p) traces.push_back(make_trace(p, chunkSize, rng));
  std::vector<std::pair<uint32_t, const Write *>> order;
  for (size_t k = 0;; ++k) {
    bool any = false;
    for (uint32_t c = 0; c < 3; ++c)
      if (k < traces[c].size()) order.push_back({c, &traces[c][k]}), any = true;
    if (!any) break;
  }
  size_t total = 0;
  for (auto &o : order) total += o.second->length;
  uint8_t *slab = nullptr;
  CHECK(hipMalloc(&slab, total) == hipSuccess);
  std::vector<UpdateIO> ios;
  size_t pos = 0;
  for (size_t i = 0; i < order.size(); ++i) {
    const Write &w = *order[i].second;
    CHECK(hipMemcpy(slab + pos, w.data.data(), w.length, hipMemcpyHostToDevice) == hipSuccess);
    UpdateIO io;
    io.offset = w.offset;
    io.length = w.length;
    io.chunk = order[i].first;
    io.data = slab + pos;
    // every 7th op carries no client checksum (adopted), every 11th a wrong one
    if (i % 7 != 3) io.checksum = ChecksumInfo{ChecksumType::CRC32C, folly_crc32c(w.data.data(), w.length) ^ (i % 11 == 5 ? 1u : 0u)};
    ios.push_back(io);
    pos += w.length;
  }
  DeviceChunks store(3, chunkSize);
  std::vector<IOResult> res;
  CHECK(ChunkReplicaBatch::update(store.metas, ios, res) == H3C_OK);
  CHECK(res.size() == ios.size());

  std::vector<std::vector<uint8_t>> host(3, std::vector<uint8_t>(chunkSize, 0));
  std::vector<orc_chunk_meta> om(3, orc_chunk_meta{0, 0, 0});
  int mismatches = 0;
  for (size_t i = 0; i < ios.size(); ++i) {
    const Write &w = *order[i].second;
    const uint32_t c = ios[i].chunk;
    orc_update_io oi{ORC_UPD_WRITE, w.offset, w.length, (uint8_t)ios[i].checksum.type, ios[i].checksum.value};
    orc_update_result orr;
    orc_chunk_replica_update(&om[c], host[c].data(), chunkSize, &oi, w.data.data(), &orr);
    CHECK((uint32_t)orr.status == res[i].status);
    mismatches += res[i].status == H3C_ERR_CHECKSUM_MISMATCH;
    CHECK(orr.size == res[i].chunkLength);
    CHECK(orr.type == (uint8_t)res[i].checksum.type && orr.value == res[i].checksum.value);
  }
  CHECK(mismatches > 0);
  for (uint32_t c = 0; c < 3; ++c) {
    CHECK(store.metas[c].size == om[c].size);
    CHECK(store.metas[c].checksumValue == om[c].checksum_value);
    CHECK(d2h(store.metas[c].bytes, om[c].size) == std::vector<uint8_t>(host[c].begin(), host[c].begin() + om[c].size));
  }
  (void)hipFree(slab);
}

static void truncate_extend_errors() {
  const uint32_t cs = 64 << 10;
  DeviceChunks store(1, cs);
  std::vector<uint8_t> data(40000);
  std::mt19937_64 rng(131);
  for (auto &b : data) b = (uint8_t)rng();
  uint8_t *p = nullptr;
  CHECK(hipMalloc(&p, data.size()) == hipSuccess);
  CHECK(hipMemcpy(p, data.data(), data.size(), hipMemcpyHostToDevice) == hipSuccess);
  auto wr = [&](uint32_t off, uint32_t len, bool good) {
    UpdateIO io;
    io.offset = off;
    io.length = len;
    io.data = p;
    io.checksum = ChecksumInfo{ChecksumType::CRC32C, folly_crc32c(data.data(), len) ^ (good ? 0u : 0x10u)};
    return io;
  };
  auto sized = [&](UpdateType t, uint32_t len) {
    UpdateIO io;
    io.updateType = t;
    io.length = len;
    return io;
  };
  std::vector<UpdateIO> ios = {
      wr(0, 30000, true),                    // 30000
      sized(UpdateType::TRUNCATE, 1000),     // 1000
      sized(UpdateType::EXTEND, 500),        // no-op: lengthInfo = meta.size
      sized(UpdateType::EXTEND, 5000),       // zeros 1000..5000
      wr(9000, 100, true),                   // gap 5000..9000 zero-filled
      wr(100, 100, false),                   // 4080, chunk unchanged
      wr(cs - 10, 100, true),                // past chunkSize: kInvalidArg
      wr(cs, 0, true),                       // offset == chunkSize: kInvalidArg
      sized(UpdateType::TRUNCATE, 0),        // empty chunk
      wr(0, 0, true),                        // empty write at 0
  };
  std::vector<IOResult> res;
  CHECK(ChunkReplicaBatch::update(store.metas, ios, res) == H3C_OK);
  std::vector<uint8_t> host(cs, 0);
  orc_chunk_meta om{0, 0, 0};
  const uint32_t wantLen[] = {30000, 1000, 1000, 5000, 100, 0, 0, 0, 0, 0};
  for (size_t i = 0; i < ios.size(); ++i) {
    const uint8_t kind = (uint8_t)ios[i].updateType;
    orc_update_io oi{kind, ios[i].offset, ios[i].length, (uint8_t)ios[i].checksum.type, ios[i].checksum.value};
    orc_update_result orr;
    orc_chunk_replica_update(&om, host.data(), cs, &oi, data.data(), &orr);
    CHECK((uint32_t)orr.status == res[i].status);
    CHECK(res[i].length == wantLen[i]);
    if (orr.status == 0) CHECK(orr.size == res[i].chunkLength && orr.value == res[i].checksum.value);
  }
  CHECK(res[5].status == kChecksumMismatch && res[6].status == kInvalidArg && res[7].status == kInvalidArg);
  CHECK(store.metas[0].size == 0 && store.metas[0].checksumValue == om.checksum_value);
  (void)hipFree(p);
}

static void recalculate_read() {
  const uint32_t cs = 256 << 10;
  DeviceChunks store(1, cs);
  std::vector<uint8_t> data(cs);
  std::mt19937_64 rng(43);
  for (auto &b : data) b = (uint8_t)rng();
  CHECK(hipMemcpy(store.metas[0].bytes, data.data(), cs, hipMemcpyHostToDevice) == hipSuccess);
  const ChecksumInfo stored{ChecksumType::CRC32C, folly_crc32c(data.data(), cs)};
  const uint8_t *b = store.metas[0].bytes;
  std::vector<ReadJob> jobs = {
      {b, H3C_MEM_DEVICE, 0, cs, cs, stored},                                        // whole chunk: stored value
      {b, H3C_MEM_DEVICE, 0, cs, cs, ChecksumInfo{ChecksumType::CRC32C, stored.value ^ 4}},  // bit rot
      {b + 4096, H3C_MEM_DEVICE, 4096, 8192, cs, stored},                            // partial read
  };
  std::vector<IOResult> rr;
  CHECK(BatchReadResults::setResults(ChecksumType::CRC32C, true, jobs, rr) == H3C_OK);
  CHECK(rr[0].ok() && rr[0].checksum == stored);
  CHECK(rr[1].status == kChecksumMismatch);
  CHECK(rr[2].ok() && rr[2].checksum.value == folly_crc32c(data.data() + 4096, 8192));
  // without recalculate the stored (wrong) value is passed through, as in the reference
  CHECK(BatchReadResults::setResults(ChecksumType::CRC32C, false, jobs, rr) == H3C_OK);
  CHECK(rr[1].ok() && rr[1].checksum.value == (stored.value ^ 4));
  // a CRC32 batch over a CRC32C chunk recomputes with CRC32
  CHECK(BatchReadResults::setResults(ChecksumType::CRC32, false, jobs, rr) == H3C_OK);
  CHECK(rr[0].checksum.type == ChecksumType::CRC32 && rr[0].checksum.value == orc_crc32_table(data.data(), cs, ~0U));
}

static void serde(bool gpu) {
  std::string msg(1000, 'x');
  for (size_t i = 0; i < msg.size(); ++i) msg[i] = (char)(i * 131 + 7);
  const uint8_t *m = (const uint8_t *)msg.data();
  for (bool comp : {false, true}) {
    const uint32_t want = (orc_crc32c_table(m, msg.size(), 0) & ~0xffu) | 0x86u | (comp ? 1u : 0u);
    if (gpu) {
      int rc = -1;
      const uint32_t got = Checksum::calcSerde(m, msg.size(), comp, H3C_MEM_HOST_PAGEABLE, &rc);
      CHECK(rc == H3C_OK && got == want);
      CHECK(Checksum::isCompressed(got) == comp && (got & 0xfeu) == Checksum::kSerdeMessageMagicNum);
    }
    CHECK(h3c_serde_checksum_mark(orc_crc32c_table(m, msg.size(), 0), comp) == want);
  }
}

// A batch past the 16384-op threshold, so the host pass runs on the worker pool: random
// WRITE / TRUNCATE / EXTEND over 24 chunks (a few with bad client checksums, a few naming
// no chunk), every result against orc_chunk_replica_update op by op.
static void large_parallel_batch() {
  const uint32_t nch = 24, cs = 64 << 10, nops = 20000;
  std::mt19937_64 rng(2024);
  DeviceChunks store(nch, cs);
  std::vector<uint8_t> pool(1 << 20);
  for (auto &b : pool) b = (uint8_t)rng();
  uint8_t *dpool = nullptr;
  CHECK(hipMalloc(&dpool, pool.size()) == hipSuccess);
  CHECK(hipMemcpy(dpool, pool.data(), pool.size(), hipMemcpyHostToDevice) == hipSuccess);
  std::vector<UpdateIO> ios(nops);
  std::vector<uint32_t> src(nops, 0);
  for (uint32_t i = 0; i < nops; ++i) {
    UpdateIO &io = ios[i];
    io.chunk = (uint32_t)(rng() % nch);
    if (i % 997 == 5) io.chunk = nch + (uint32_t)(rng() % 3);  // no such chunk
    const uint32_t u = (uint32_t)(rng() % 100);
    if (u < 80) {
      io.offset = (uint32_t)(rng() % cs);
      io.length = (uint32_t)(rng() % std::min<uint32_t>(cs - io.offset, 9000));
      src[i] = (uint32_t)(rng() % (pool.size() - 9000));
      io.data = dpool + src[i];
      if (rng() % 10) {
        io.checksum = ChecksumInfo{ChecksumType::CRC32C, folly_crc32c(pool.data() + src[i], io.length)};
        if (rng() % 50 == 0) io.checksum.value ^= 4;  // corrupted in flight
      }
    } else {
      io.updateType = u < 90 ? UpdateType::TRUNCATE : UpdateType::EXTEND;
      io.length = (uint32_t)(rng() % (cs + 1));
    }
  }
  std::vector<IOResult> res;
  CHECK(ChunkReplicaBatch::update(store.metas, ios, res) == H3C_OK);
  std::vector<std::vector<uint8_t>> host(nch, std::vector<uint8_t>(cs, 0));
  std::vector<orc_chunk_meta> om(nch, orc_chunk_meta{0, 0, 0});
  size_t bad = 0;
  for (uint32_t i = 0; i < nops; ++i) {
    const UpdateIO &io = ios[i];
    if (io.chunk >= nch) {
      CHECK(res[i].status == kInvalidArg);
      continue;
    }
    orc_update_io oi{(uint8_t)io.updateType, io.offset, io.length, (uint8_t)io.checksum.type, io.checksum.value};
    orc_update_result orr;
    orc_chunk_replica_update(&om[io.chunk], host[io.chunk].data(), cs, &oi,
                             io.isWrite() ? pool.data() + src[i] : nullptr, &orr);
    if ((uint32_t)orr.status != res[i].status || orr.size != res[i].chunkLength ||
        (orr.status == 0 && orr.value != res[i].checksum.value))
      ++bad;
  }
  CHECK(bad == 0);
  for (uint32_t c = 0; c < nch; ++c) {
    CHECK(store.metas[c].size == om[c].size && store.metas[c].checksumValue == om[c].checksum_value);
    CHECK(d2h(store.metas[c].bytes, om[c].size) == std::vector<uint8_t>(host[c].begin(), host[c].begin() + om[c].size));
  }
  (void)hipFree(dpool);
}

// Pieces handed out from a list (a ChunkDataIterator stand-in: 1 MiB preads, a short read
// ends the data early).
struct ListIterator : ChecksumInfo::DataIterator {
  std::vector<std::pair<const uint8_t *, size_t>> pieces;
  size_t k = 0;
  std::pair<const uint8_t *, size_t> next() override {
    return k < pieces.size() ? pieces[k++] : std::pair<const uint8_t *, size_t>{nullptr, 0};
  }
};

static void data_iterator(bool gpu) {
  // host-only cases: NONE, and byte counts that do not add up to the length
  ListIterator none;
  none.pieces = {{(const uint8_t *)"abc", 3}};
  CHECK((ChecksumInfo::create(ChecksumType::NONE, &none, 3) == ChecksumInfo{}));
  ListIterator shortread;
  static const uint8_t bytes[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  shortread.pieces = {{bytes, 4}};
  CHECK((ChecksumInfo::create(ChecksumType::CRC32C, &shortread, 8, ~0U, H3C_MEM_HOST_PAGEABLE) == ChecksumInfo{}));
  ListIterator empty;
  CHECK((ChecksumInfo::create(ChecksumType::CRC32C, &empty, 0, 0x1234) == ChecksumInfo{ChecksumType::CRC32C, 0x1234}));
  if (!gpu) return;
  const size_t n = (5u << 20) + 777;
  std::vector<uint8_t> host(n);
  std::mt19937_64 rng(146);
  for (auto &b : host) b = (uint8_t)rng();
  uint8_t *dev = nullptr;
  CHECK(hipMalloc(&dev, n) == hipSuccess);
  CHECK(hipMemcpy(dev, host.data(), n, hipMemcpyHostToDevice) == hipSuccess);
  for (ChecksumType t : {ChecksumType::CRC32C, ChecksumType::CRC32}) {
    const uint32_t want = t == ChecksumType::CRC32C ? folly_crc32c(host.data(), n, 0xABCDEF01u)
                                                    : orc_crc32_table(host.data(), n, 0xABCDEF01u);
    ChecksumInfo::MemoryDataIterator mem(dev, n);  // 1 MiB slices, as ChunkFileView reads
    int rc = -1;
    CHECK((ChecksumInfo::create(t, &mem, n, 0xABCDEF01u, H3C_MEM_DEVICE, nullptr, &rc) == ChecksumInfo{t, want}));
    CHECK(rc == H3C_OK);
    ListIterator ragged;  // uneven pieces, a zero-size one in the middle
    size_t off = 0;
    for (size_t len : {size_t(1), size_t(4095), size_t(0), size_t(3u << 20), size_t(123457)}) {
      ragged.pieces.push_back({dev + off, len});
      off += len;
    }
    ragged.pieces.push_back({dev + off, n - off});
    CHECK((ChecksumInfo::create(t, &ragged, n, 0xABCDEF01u) == ChecksumInfo{t, want}));
    ListIterator over;  // the last piece runs past `length`: taken whole, then the count mismatches
    over.pieces = {{dev, 1000}, {dev + 1000, 1000}};
    CHECK((ChecksumInfo::create(t, &over, 1500) == ChecksumInfo{}));
  }
  (void)hipFree(dev);
}

// VersionGate: the version / state checks of ChunkReplica::update (:171-247) and ::commit (:397-467)
// replayed on the host in sequence order, each case of the reference once, including
// the cascade of a failed checksum verify (the chunk's updateVer stays, so the next op misses one).
static void version_gate() {
  std::vector<ChunkVersion> v(6);
  v[1].chunkState = ChunkState::DIRTY;
  v[4].chunkState = ChunkState::DIRTY;  // (a 64 KiB chunk: the chunkSize / range cases)
  v[4].chunkSize = 64 << 10;
  v[4].updateVer = v[4].commitVer = 2;
  v[2].chunkState = ChunkState::COMMIT;
  v[2].chainVer = 7;
  v[2].updateVer = v[2].commitVer = 5;
  auto up = [](uint32_t c, uint32_t ver, uint32_t chain = 1, bool ok = true, bool sync = false) {
    VersionedOp o;
    o.chunk = c;
    o.updateVer = ver;
    o.commitChainVer = chain;
    o.checksumOk = ok;
    o.isSyncing = sync;
    return o;
  };
  auto commit = [](uint32_t c, uint32_t ver, uint32_t chain = 1, bool force = false) {
    VersionedOp o;
    o.chunk = c;
    o.isCommit = true;
    o.updateVer = ver;
    o.commitChainVer = chain;
    o.isForce = force;
    return o;
  };
  auto sized = [](uint32_t c, uint32_t ver, uint64_t cs, uint64_t off, uint64_t len, bool sync = false,
                  bool remove = false) {
    VersionedOp o;
    o.chunk = c;
    o.updateVer = ver;
    o.commitChainVer = 1;
    o.isSyncing = sync;
    o.isRemove = remove;
    o.chunkSize = cs;
    o.offset = off;
    o.length = len;
    return o;
  };
  const std::vector<VersionedOp> ops = {
      up(0, 1), up(0, 2), up(0, 2),              // admitted, admitted, stale (4006)
      up(0, 4),                                  // missing one (4007)
      up(0, 0),                                  // updateVer 0: 3 > commitVer 0 + 1 -> advance (4012)
      commit(0, 2), up(0, 1),                    // commit 2; then 1 <= commitVer: committed (4008)
      up(0, 3, 1, false), up(0, 4),              // checksum fails (4080, nothing changes); 4 misses 3 (4007)
      up(0, 3),                                  // 3 admitted
      up(1, 1),                                  // DIRTY and not syncing (4005)
      up(1, 9, 1, true, true),                   // syncing on a DIRTY chunk: updateVer 9, commitVer 8
      up(2, 6, 3),                               // COMMIT with a newer chain version than the op's (4081)
      up(2, 6, 7),                               // same chain version: admitted
      commit(2, 9, 7),                           // commit beyond updateVer (4082)
      commit(2, 5, 7),                           // commit 5 <= commitVer 5: stale commit (4023)
      commit(2, 6, 8),                           // commit 6 == updateVer: COMMIT, chainVer 8
      up(9, 1),                                  // no such chunk (kInvalidArg)
      up(3, 0), up(3, 0),                        // updateVer 0: 1 admitted, then 2 > 0 + 1 (4012)
      sized(4, 3, 1 << 20, 0, 4096),             // DIRTY chunk 4 (64 KiB) with the wrong chunkSize: 4015 first
      sized(4, 3, 64 << 10, 64 << 10, 1),        // range outside the op's chunkSize: kInvalidArg before 4005
      sized(4, 3, 64 << 10, 0, 4096),            // right size, DIRTY, not syncing: 4005
      sized(4, 10, 1 << 20, 0, 4096, true),      // syncing, wrong size: 4015 (no version change)
      sized(4, 0, 1 << 20, 0, 0, false, true),   // REMOVE: no size or range check; DIRTY -> 4005
      sized(5, 1, 64 << 10, 0, 4096),            // a new chunk (size unknown): admitted, and it takes 64 KiB
      sized(5, 2, 1 << 20, 0, 4096),             // the next op of it with another chunkSize: 4015 (ChunkReplica.cc:163)
      sized(5, 2, 64 << 10, 4096, 4096),         // the same size: admitted
  };
  const std::vector<uint32_t> want = {0, 0, 4006, 4007, 4012, 0, 4008, 4080, 4007, 0, 4005, 0, 4081, 0, 4082, 4023,
                                      0, 3, 0, 4012, 4015, 3, 4005, 4015, 4005, 0, 4015, 0};
  std::vector<uint32_t> st;
  VersionGate::run(v, ops, st);
  CHECK(st == want);
  for (size_t i = 0; i < st.size() && i < want.size(); ++i)
    if (st[i] != want[i]) std::fprintf(stderr, "  op %zu: %u, want %u\n", i, st[i], want[i]);
  CHECK(v[0].updateVer == 3 && v[0].commitVer == 2 && v[0].chunkState == ChunkState::CLEAN);
  CHECK(v[1].updateVer == 9 && v[1].commitVer == 8 && v[1].chunkState == ChunkState::CLEAN);
  CHECK(v[4].updateVer == 2 && v[4].commitVer == 2 && v[4].chunkState == ChunkState::DIRTY);
  CHECK(v[2].updateVer == 6 && v[2].commitVer == 6 && v[2].chunkState == ChunkState::COMMIT && v[2].chainVer == 8);
  CHECK(v[3].updateVer == 1 && v[3].commitVer == 0);
  CHECK(v[5].chunkSize == (64 << 10) && v[5].updateVer == 2);
}

int main(int argc, char **argv) {
  const bool gpu = argc > 1 && std::string(argv[1]) == "gpu";
  version_gate();
  serde(false);
  data_iterator(gpu);
  if (gpu) {
    verify_checksum_patterns(1 << 20);
    verify_checksum_patterns(512 << 10);
    batched_vs_replica(1 << 20);
    truncate_extend_errors();
    recalculate_read();
    large_parallel_batch();
    serde(true);
  }
  if (fails) {
    std::fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  std::printf("storage_path_test %s: ok\n", gpu ? "gpu" : "cpu");
  return 0;
}
