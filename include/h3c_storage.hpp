// h3c_storage.hpp -- header-only C++ mirror of the 3FS storage types on the checksum path,
// over the C ABI in h3c_crc.h.  Names, argument meaning and error codes follow the
// reference so a storage-service maintainer (or a test) can write against it the way
// the reference's own code reads:
//
//   UpdateType / UpdateIO / ChunkMetadata / IOResult   src/fbs/storage/Common.h:51-58,221-250,326-345,662-676
//   ChunkReplicaBatch::update                          ChunkReplica::update + updateChecksum
//                                                      (src/storage/store/ChunkReplica.cc:131-394), batched
//   BatchReadResults::setResults                       AioReadJob::setResult (src/storage/aio/BatchReadJob.cc:24-55)
//   Checksum::calcSerde                                src/common/net/MessageHeader.h:32-37
//   VersionGate                                        the version / state checks of ChunkReplica::update
//                                                      (:171-247) and ChunkReplica::commit (:397-467), on
//                                                      the host (no payload work: see INTEGRATION.md §1)
//
// Every payload byte is checksummed on the GPU; the classes hold no device state.
#pragma once

#include <cstddef>
#include <cstdint>
#include <optional>
#include <vector>

#include "h3c_checksum_info.hpp"
#include "h3c_crc.h"

namespace h3c {

// StatusCode / StorageCode values used on the path (src/common/utils/StatusCodeDetails.h).
enum StatusCode : uint32_t {
  kOK = 0,
  kInvalidArg = 3,
  kChunkNotClean = 4005,
  kChunkStaleUpdate = 4006,
  kChunkMissingUpdate = 4007,
  kChunkCommittedUpdate = 4008,
  kChunkReadFailed = 4010,
  kChunkAdvanceUpdate = 4012,
  kChunkSizeMismatch = 4015,
  kChunkStaleCommit = 4023,
  kChecksumMismatch = 4080,
  kChainVersionMismatch = 4081,
  kChunkVersionMismatch = 4082,
};

// UpdateType (Common.h:51-58).
enum class UpdateType : uint8_t { INVALID = 0, WRITE = 1, REMOVE = 2, TRUNCATE = 4, EXTEND = 8, COMMIT = 16 };

// UpdateIO fields on the path (Common.h:326-345); `chunk` indexes the batch's chunk table
// (the reference keys by GlobalKey), `data` is the payload's device address.
struct UpdateIO {
  uint32_t offset = 0;
  uint32_t length = 0;
  uint32_t chunk = 0;
  UpdateType updateType = UpdateType::WRITE;
  ChecksumInfo checksum;
  const uint8_t *data = nullptr;
  bool isSyncing = false;  // UpdateOptions.isSyncing (ChunkReplica.cc:211-215, 289): WRITE at offset 0
  // UpdateIO.chunkSize (H3C_IO_CHUNK_SIZE): the range check (:141-145) and the 4015 check (:171-180) use it;
  // not carried: the chunk's own innerFileId.chunkSize stands in (a carried 0 fails as the reference's would)
  std::optional<uint32_t> chunkSize;

  bool isWrite() const { return updateType == UpdateType::WRITE; }
  bool isRemove() const { return updateType == UpdateType::REMOVE; }
  bool isTruncate() const { return updateType == UpdateType::TRUNCATE; }
  bool isExtend() const { return updateType == UpdateType::EXTEND; }
};

// ChunkMetadata fields on the path (Common.h:662-676) + where the chunk's bytes live.
struct ChunkMetadata {
  uint8_t *bytes = nullptr;  // device memory, capacity chunkSize
  uint32_t chunkSize = 0;    // innerFileId.chunkSize
  uint32_t size = 0;
  ChecksumType checksumType = ChecksumType::NONE;
  uint32_t checksumValue = 0;
  ChecksumInfo checksum() const { return ChecksumInfo{checksumType, checksumValue}; }
};

// IOResult subset (Common.h:221-250).  lengthInfo is the error, or its value: the bytes
// written for a WRITE, meta.size for TRUNCATE / EXTEND (ChunkReplica.cc:259-292), the bytes
// read for a read.  chunkLength is meta.size after an update (not part of IOResult).
struct IOResult {
  uint32_t status = kOK;     // lengthInfo's error, or kOK
  uint32_t length = 0;       // lengthInfo's value
  ChecksumInfo checksum;     // result.checksum (meta.checksum() after an update)
  uint32_t chunkLength = 0;
  bool ok() const { return status == kOK; }
};

// ChunkReplica::update + updateChecksum for a batch of UpdateIOs in sequence order.
struct ChunkReplicaBatch {
  // `metas` are updated in place (size / checksumType / checksumValue), chunk bytes on
  // device.  `checksumType` is the batch's polynomial (the client's chunk_checksum_type).
  // `flags`: H3C_UPD_EXACT to not trust stored checksums; `counters`: the reference's
  // storage.chunk_update.checksum_* counts of the batch (ChunkReplica.cc:25-28).
  static int update(std::vector<ChunkMetadata> &metas, const std::vector<UpdateIO> &ios,
                    std::vector<IOResult> &results, ChecksumType checksumType = ChecksumType::CRC32C,
                    void *stream = nullptr, uint32_t flags = 0, h3c_update_counters *counters = nullptr) {
    std::vector<h3c_chunk_state> cs(metas.size());
    for (size_t c = 0; c < metas.size(); ++c)
      cs[c] = h3c_chunk_state{(uint64_t)(uintptr_t)metas[c].bytes, metas[c].chunkSize, metas[c].size,
                              metas[c].checksumValue, (uint8_t)metas[c].checksumType, {0, 0, 0}};
    std::vector<h3c_update_io> io(ios.size());
    for (size_t i = 0; i < ios.size(); ++i)
      io[i] = h3c_update_io{(uint64_t)(uintptr_t)ios[i].data, ios[i].chunk, ios[i].offset, ios[i].length,
                            ios[i].checksum.value, (uint8_t)ios[i].checksum.type, (uint8_t)ios[i].updateType,
                            (uint8_t)((ios[i].isSyncing ? H3C_IO_SYNCING : 0u) |
                                      (ios[i].chunkSize ? H3C_IO_CHUNK_SIZE : 0u)),
                            0, ios[i].chunkSize.value_or(0u)};
    std::vector<h3c_update_result> res(ios.size());
    const int rc = h3c_update_ios_ex((uint8_t)checksumType, cs.data(), (uint32_t)cs.size(), io.data(),
                                     (uint32_t)io.size(), res.data(), flags, counters, stream);
    if (rc != H3C_OK) return rc;
    results.resize(ios.size());
    for (size_t i = 0; i < ios.size(); ++i) {
      const uint32_t len = res[i].status != H3C_OK ? 0 : ios[i].isWrite() ? ios[i].length : res[i].size;
      results[i] = IOResult{res[i].status, len, ChecksumInfo{(ChecksumType)res[i].type, res[i].value}, res[i].size};
    }
    for (size_t c = 0; c < metas.size(); ++c) {
      metas[c].size = cs[c].size;
      metas[c].checksumType = (ChecksumType)cs[c].type;
      metas[c].checksumValue = cs[c].value;
    }
    return H3C_OK;
  }
};

// One completed read of a BatchReadJob (AioReadJob's state on the path).
struct ReadJob {
  const uint8_t *data = nullptr;  // localbuf + headLength
  h3c_mem mem = H3C_MEM_DEVICE;
  uint32_t offset = 0;            // readIO.offset
  uint32_t length = 0;            // *lengthInfo
  uint32_t chunkLen = 0;          // state.chunkLen
  ChecksumInfo chunkChecksum;     // state.chunkChecksum
};

// AioReadJob::setResult's checksum selection + recalculate verify for a batch.
struct BatchReadResults {
  // checksumMismatch (optional) += the batch's storage.aio.checksum_mismatch count (BatchReadJob.cc:14).
  static int setResults(ChecksumType batchType, bool recalculateChecksum, const std::vector<ReadJob> &jobs,
                        std::vector<IOResult> &results, void *stream = nullptr, uint64_t *checksumMismatch = nullptr) {
    std::vector<h3c_read_job> j(jobs.size());
    for (size_t i = 0; i < jobs.size(); ++i)
      j[i] = h3c_read_job{jobs[i].data, jobs[i].length, jobs[i].chunkLen, jobs[i].offset, jobs[i].chunkChecksum.value,
                          (uint8_t)jobs[i].chunkChecksum.type, (uint8_t)jobs[i].mem,
                          (uint8_t)(recalculateChecksum ? 1 : 0), {0, 0, 0, 0, 0}};
    std::vector<uint8_t> t(jobs.size());
    std::vector<uint32_t> v(jobs.size()), st(jobs.size());
    uint64_t mis = 0;
    const int rc = h3c_batch_read_result_ex((uint8_t)batchType, j.data(), j.size(), t.data(), v.data(), st.data(), &mis,
                                            stream);
    if (rc != H3C_OK) return rc;
    if (checksumMismatch) *checksumMismatch += mis;
    results.resize(jobs.size());
    for (size_t i = 0; i < jobs.size(); ++i)
      results[i] = IOResult{st[i], jobs[i].length, ChecksumInfo{(ChecksumType)t[i], v[i]}, jobs[i].chunkLen};
    return H3C_OK;
  }
};

// ChunkState (Common.h:60-64) and the version fields of ChunkMetadata (Common.h:662-676).
enum class ChunkState : uint8_t { COMMIT = 0, DIRTY = 1, CLEAN = 2 };
struct ChunkVersion {
  uint32_t updateVer = 0, commitVer = 0, chainVer = 0;
  ChunkState chunkState = ChunkState::CLEAN;
  uint64_t chunkSize = 0;  // meta.innerFileId.chunkSize (0: not known to the gate, not checked)
};
// One update or commit of a chunk as the gate sees it.
struct VersionedOp {
  uint32_t chunk = 0;           // index into the batch's chunk table
  bool isCommit = false;        // ChunkReplica::commit (CommitIO) rather than ChunkReplica::update
  bool isRemove = false;        // UpdateIO.isRemove(): no range check, the stored chunk size is its own
  uint32_t updateVer = 0;       // UpdateIO.updateVer (0: the next one) / CommitIO.commitVer
  uint32_t commitChainVer = 0;  // job.commitChainVer()
  bool isSyncing = false;       // UpdateOptions.isSyncing
  bool isForce = false;         // CommitIO.isForce
  bool checksumOk = true;       // the op's client-checksum verify passed (ChunkReplica.cc:193-207), if known
  uint64_t chunkSize = 0;       // UpdateIO.chunkSize (0: not checked by the gate)
  uint64_t offset = 0, length = 0;  // UpdateIO.offset / length (range-checked against chunkSize when it is set)
};

// The version / state gate that stays on the host.  ChunkReplica::update rejects an op
// before touching its bytes, in this order: a range outside the op's own chunkSize (kInvalidArg, :141-146),
// a chunkSize that differs from the stored chunk's (4015, :171-180; both checked only when the op and the
// chunk carry a chunkSize), the chunk DIRTY and the op not syncing (4005, :181-185), when a
// committed chunk's chain version is newer than the op's (4081, :186-191), and -- after the checksum
// verify at :193-207 -- when updateVer is committed (4008), stale (4006), missing one (4007) or, for
// updateVer 0, too far ahead (4012) (:211-239); a successful op sets updateVer and, at its end, a CLEAN
// state and the op's chain version (:241-244, :298).  ChunkReplica::commit checks chain (4081) and commit
// versions (4082), a DIRTY chunk (4005) and stale commits (4023) (:419-446) and marks a fully committed
// chunk COMMIT (:448-451).  run() replays these in sequence order per chunk and returns each op's status
// (0: admitted); `versions` end as the reference's metadata would.  The checksum verify sits between the
// two groups of checks: an op with checksumOk == false fails with 4080 after the first group, as the
// reference's does, and changes no version.  Ops admitted here go to h3c_update_ios; the others are
// answered with their status and not submitted.  Every code the reference returns before a version change
// is decided here (range, 4015, 4005, 4081, 4080 from the verdicts given, 4006-4012); an op admitted here is
// one the engine applies, so the versions the gate leaves are the reference's -- provided `checksumOk` carries
// the verify verdicts (h3c_batch_verify first) whenever a payload may fail it.
struct VersionGate {
  static void run(std::vector<ChunkVersion> &versions, const std::vector<VersionedOp> &ops,
                  std::vector<uint32_t> &status) {
    status.assign(ops.size(), kOK);
    for (size_t i = 0; i < ops.size(); ++i) {
      const VersionedOp &op = ops[i];
      if (op.chunk >= versions.size()) {
        status[i] = kInvalidArg;
        continue;
      }
      ChunkVersion &m = versions[op.chunk];
      if (op.isCommit) {  // ChunkReplica::commit (:419-451)
        if (op.commitChainVer < m.chainVer) {
          status[i] = kChainVersionMismatch;
        } else if (op.updateVer > m.updateVer) {
          status[i] = kChunkVersionMismatch;
        } else if (op.isForce) {
          m.chunkState = ChunkState::CLEAN;
          m.commitVer = op.updateVer;
        } else if (m.chunkState == ChunkState::DIRTY) {
          status[i] = kChunkNotClean;
        } else if (m.commitVer < op.updateVer) {
          m.commitVer = op.updateVer;
        } else {
          status[i] = kChunkStaleCommit;
        }
        if (status[i] == kOK && m.commitVer == m.updateVer) {
          m.chunkState = ChunkState::COMMIT;
          m.chainVer = op.commitChainVer;
        }
        continue;
      }
      if (!op.isRemove && op.chunkSize &&
          (op.offset >= op.chunkSize || op.offset + op.length > op.chunkSize)) {  // :141-146
        status[i] = kInvalidArg;
        continue;
      }
      if (!op.isRemove && op.chunkSize && m.chunkSize && m.chunkSize != op.chunkSize) {  // :171-180
        status[i] = kChunkSizeMismatch;
        continue;
      }
      if (m.chunkState == ChunkState::DIRTY && !op.isSyncing) {  // :181-185
        status[i] = kChunkNotClean;
        continue;
      }
      if (op.commitChainVer < m.chainVer && m.chunkState == ChunkState::COMMIT) {  // :186-191
        status[i] = kChainVersionMismatch;
        continue;
      }
      if (!op.checksumOk) {  // :193-207 (the reference returns before any version change)
        status[i] = kChecksumMismatch;
        continue;
      }
      uint32_t uv = m.updateVer, cv = m.commitVer;
      if (op.isSyncing) {  // :211-215
        uv = op.updateVer;
        cv = op.updateVer - 1;
      } else if (op.updateVer > 0) {  // :216-232
        if (op.updateVer <= m.commitVer) status[i] = kChunkCommittedUpdate;
        else if (op.updateVer <= m.updateVer) status[i] = kChunkStaleUpdate;
        else if (op.updateVer > m.updateVer + 1) status[i] = kChunkMissingUpdate;
        else uv = op.updateVer;
      } else {  // :233-239
        uv = m.updateVer + 1;
        if (uv > m.commitVer + 1) status[i] = kChunkAdvanceUpdate;
      }
      if (status[i] != kOK) continue;  // (the meta copy with the changed versions is never stored)
      m.updateVer = uv;
      m.commitVer = cv;
      m.chainVer = op.commitChainVer;  // :241
      m.chunkState = ChunkState::CLEAN;  // DIRTY during the write, CLEAN at :298
      // a chunk the gate knew no size for takes the admitted op's: the reference's createChunk path stores
      // meta.innerFileId.chunkSize = writeIO.chunkSize (:163), and an existing chunk of another size would have
      // failed this op with 4015, so later ops of the batch are checked against it
      if (!op.isRemove && op.chunkSize && !m.chunkSize) m.chunkSize = op.chunkSize;
    }
  }
};

// hf3fs::net::Checksum (MessageHeader.h:32-37).
struct Checksum {
  static constexpr uint8_t kSerdeMessageMagicNum = 0x86;  // MessageHeader.h:14
  static uint32_t calcSerde(const uint8_t *data, size_t size, bool compressed = false, h3c_mem mem = H3C_MEM_HOST_PAGEABLE,
                            int *rc = nullptr) {
    h3c_desc d{data, size, 0, (uint8_t)ChecksumType::CRC32C, (uint8_t)mem, 0};
    const uint8_t comp = compressed ? 1 : 0;
    uint32_t out = 0;
    const int r = h3c_batch_serde_checksum(&d, 1, &comp, &out, nullptr);
    if (rc) *rc = r;
    return out;
  }
  static bool isCompressed(uint32_t checksum) { return checksum & 1; }  // MessageHeader.h:26
};

}  // namespace h3c
