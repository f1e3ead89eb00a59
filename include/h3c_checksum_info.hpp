// h3c_checksum_info.hpp -- header-only C++ mirror of hf3fs::storage::ChecksumInfo
// (src/fbs/storage/Common.h:113-201) over the C ABI in h3c_crc.h.
//
// Same names, argument meaning and error behaviour as the reference:
//   create(type, buf, len, start=~0)  NONE -> {NONE,0}; len 0 -> {type,start};
//                                     buf==nullptr && len>0 -> {NONE,0}
//   combine(o, len)                   4080 (kChecksumMismatch) on type mismatch,
//                                     len 0 no-op, NONE receiver copies o,
//                                     else value = crc32c_combine(~value, o.value, len)
//   operator==                        field-wise
// The payload CRC runs on the GPU; combine is O(log n) host GF(2) arithmetic, as
// in the reference (folly::crc32c_combine is host code there too).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "h3c_crc.h"

namespace h3c {

enum class ChecksumType : uint8_t { NONE = 0, CRC32C = 1, CRC32 = 2 };

struct ChecksumInfo {
  ChecksumType type = ChecksumType::NONE;
  uint32_t value = 0;

  static constexpr size_t kChunkSize = size_t(1) << 20;  // Common.h:118

  // ChecksumInfo::DataIterator / MemoryDataIterator (Common.h:120-144): next() yields
  // pieces, {nullptr, 0} at the end; the memory iterator slices at kChunkSize.
  class DataIterator {
   public:
    virtual ~DataIterator() = default;
    virtual std::pair<const uint8_t *, size_t> next() = 0;
  };
  class MemoryDataIterator : public DataIterator {
   public:
    MemoryDataIterator(const uint8_t *buffer, size_t length) : buffer_(buffer), length_(length) {}
    std::pair<const uint8_t *, size_t> next() override {
      if (length_ == 0) return {nullptr, 0};
      const uint8_t *data = buffer_;
      const size_t size = length_ < kChunkSize ? length_ : kChunkSize;
      buffer_ += size;
      length_ -= size;
      return {data, size};
    }

   private:
    const uint8_t *buffer_;
    size_t length_;
  };

  // ChecksumInfo::create(type, DataIterator*, length, startingChecksum) (Common.h:146-172):
  // pieces are taken while the piece pointer is non-null and fewer than `length` bytes
  // were taken (a piece is always taken whole); a byte count other than `length` gives
  // {NONE, 0}.  The pieces (all of memory kind `mem`) are checksummed in one batch on the
  // GPU -- the first from `start`, the others from 0 -- and chained with the combine
  // shift, which equals the reference's sequential crc32c(piece, previous) chain.
  static ChecksumInfo create(ChecksumType type, DataIterator *iter, size_t length, uint32_t start = ~0U,
                             h3c_mem mem = H3C_MEM_DEVICE, void *stream = nullptr, int *rc = nullptr) {
    if (rc) *rc = H3C_OK;
    if (type == ChecksumType::NONE) return ChecksumInfo{ChecksumType::NONE, 0U};
    std::vector<h3c_desc> pieces;
    size_t iter_bytes = 0;
    for (auto data = iter->next(); data.first != nullptr && iter_bytes < length; data = iter->next()) {
      iter_bytes += data.second;
      if (data.second)
        pieces.push_back(h3c_desc{data.first, (uint64_t)data.second, pieces.empty() ? start : 0u, (uint8_t)type,
                                  (uint8_t)mem, 0});
    }
    if (iter_bytes != length) return ChecksumInfo{ChecksumType::NONE, 0U};
    if (pieces.empty()) return ChecksumInfo{type, start};
    std::vector<uint8_t> t(pieces.size());
    std::vector<uint32_t> v(pieces.size());
    const int r = h3c_batch_create(pieces.data(), pieces.size(), t.data(), v.data(), stream);
    if (rc) *rc = r;
    if (r != H3C_OK) return ChecksumInfo{ChecksumType::NONE, 0U};
    uint32_t acc = v[0];
    for (size_t k = 1; k < pieces.size(); ++k)
      acc = type == ChecksumType::CRC32C ? h3c_crc32c_combine(acc, v[k], pieces[k].len)
                                         : h3c_crc32_combine(acc, v[k], pieces[k].len);
    return ChecksumInfo{type, acc};
  }

  // ChecksumInfo::create(type, buffer, length, startingChecksum) (Common.h:174-177).
  // `mem` says where `buf` lives; `rc` (optional) receives the engine status.
  static ChecksumInfo create(ChecksumType type, const uint8_t *buf, size_t length, uint32_t start = ~0U,
                             h3c_mem mem = H3C_MEM_DEVICE, void *stream = nullptr, int *rc = nullptr) {
    h3c_desc d{buf, (uint64_t)length, start, (uint8_t)type, (uint8_t)mem, 0};
    uint8_t t = 0;
    uint32_t v = 0;
    const int r = h3c_batch_create(&d, 1, &t, &v, stream);
    if (rc) *rc = r;
    if (r != H3C_OK) return ChecksumInfo{ChecksumType::NONE, 0U};
    return ChecksumInfo{(ChecksumType)t, v};
  }

  // Batched form: one GPU pass over many chunks (the point of the engine).
  static int createBatch(const std::vector<h3c_desc> &descs, std::vector<ChecksumInfo> &out, void *stream = nullptr) {
    std::vector<uint8_t> t(descs.size());
    std::vector<uint32_t> v(descs.size());
    const int r = h3c_batch_create(descs.data(), descs.size(), t.data(), v.data(), stream);
    if (r != H3C_OK) return r;
    out.resize(descs.size());
    for (size_t i = 0; i < descs.size(); ++i) out[i] = ChecksumInfo{(ChecksumType)t[i], v[i]};
    return H3C_OK;
  }

  // ChecksumInfo::combine (Common.h:179-198); returns 0 or H3C_ERR_CHECKSUM_MISMATCH (4080).
  int combine(const ChecksumInfo &o, size_t length) {
    if (type != ChecksumType::NONE && type != o.type) return H3C_ERR_CHECKSUM_MISMATCH;
    if (length == 0) return H3C_OK;
    switch (type) {
      case ChecksumType::NONE:
        *this = o;
        return H3C_OK;
      case ChecksumType::CRC32C:
        value = h3c_crc32c_combine(~value, o.value, length);
        return H3C_OK;
      case ChecksumType::CRC32:
        value = h3c_crc32_combine(~value, o.value, length);
        return H3C_OK;
    }
    return H3C_OK;
  }

  // serde binary form (src/common/serde/Serde.h:267-290, DownwardBytes): a Varint32 table
  // length, then the fields in order -- type (1 byte), value (4 bytes, little endian).
  // TestCommonStruct.cc:46-56 pins the size (1 + 1 + 4) and the round trip.
  std::string serialize() const {
    std::string out(6, '\0');
    out[0] = 5;
    out[1] = (char)type;
    for (int k = 0; k < 4; ++k) out[2 + k] = (char)((value >> (8 * k)) & 0xFF);
    return out;
  }
  // Returns 0, or H3C_ERR_INVALID_ARG for a short or malformed buffer; fields missing at
  // the end of the table keep their values (Serde.h:499-507).
  static int deserialize(ChecksumInfo &o, const void *data, size_t len) {
    const uint8_t *p = static_cast<const uint8_t *>(data);
    uint64_t tlen = 0;
    size_t k = 0;
    for (int shift = 0;; shift += 7) {  // Varint32 length prefix
      if (k >= len || shift > 28) return H3C_ERR_INVALID_ARG;
      tlen |= (uint64_t)(p[k] & 0x7F) << shift;
      if (!(p[k++] & 0x80)) break;
    }
    if (tlen > len - k) return H3C_ERR_INVALID_ARG;
    const uint8_t *t = p + k;
    if (tlen >= 1) o.type = (ChecksumType)t[0];
    if (tlen >= 5) o.value = (uint32_t)t[1] | (uint32_t)t[2] << 8 | (uint32_t)t[3] << 16 | (uint32_t)t[4] << 24;
    else if (tlen > 1) return H3C_ERR_INVALID_ARG;  // a truncated value field
    return H3C_OK;
  }

  bool operator==(const ChecksumInfo &o) const { return type == o.type && value == o.value; }
  bool operator!=(const ChecksumInfo &o) const { return !(*this == o); }
};

// Rust chunk-engine domain (crate crc32c 0.6.8, Cargo.lock:399-402): std = ~raw
// (src/storage/store/ChunkEngine.cc:42,66).
inline uint32_t std_from_raw(uint32_t raw) { return ~raw; }
inline uint32_t raw_from_std(uint32_t std_value) { return ~std_value; }

}  // namespace h3c
