// h3c_formats.hip -- the small checksum formats next to the chunk path, on the same
// kernels:
//   * RPC message checksum Checksum::calcSerde (src/common/net/MessageHeader.h:32-37):
//     folly::crc32c(data, size, 0) with the low byte replaced by 0x86 | compressed;
//     checked on receipt by Processor::unpackSerdeMsg (src/common/net/Processor.h:113-117).
//   * the Rust crc32c crate 0.6.8 API of the chunk engine (std domain, std = ~raw):
//     crc32c / crc32c_append / crc32c_combine (chunk_engine/src/alloc/chunk.rs:152-269).
//   * ChecksumInfo::combine as a C function (src/fbs/storage/Common.h:179-198) and the
//     client's fold of split-read checksums (src/client/storage/StorageClientImpl.cc:1607-1633).
//   * the read path's checksum selection + recalculate verify, AioReadJob::setResult
//     (src/storage/aio/BatchReadJob.cc:24-55), for a batch of completed read jobs.
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "h3c_crc.h"

namespace {
constexpr uint32_t kSerdeMagic = 0x86;  // kSerdeMessageMagicNum, MessageHeader.h:14

uint32_t serde_mark(uint32_t crc0, int compressed) { return (crc0 & ~0xFFu) | kSerdeMagic | (compressed ? 1u : 0u); }

// batch create with every descriptor forced to CRC32C and start `start` (or ~append_to[i]).
int create_with(const h3c_desc *d, size_t n, const uint32_t *append_std, uint32_t start, uint32_t *out_raw,
                void *stream) {
  std::vector<h3c_desc> dd(d, d + n);
  for (size_t i = 0; i < n; ++i) {
    dd[i].type = H3C_TYPE_CRC32C;
    dd[i].start_raw = append_std ? ~append_std[i] : start;
  }
  return h3c_batch_create(dd.data(), n, nullptr, out_raw, stream);
}
}  // namespace

namespace {
// Where `p` lives: device memory (read in place) or host memory (staged).
uint8_t mem_kind(const void *p) {
  hipPointerAttribute_t a;
  if (p && hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeDevice) return H3C_MEM_DEVICE;
  (void)hipGetLastError();  // a plain host pointer is not an error
  return H3C_MEM_HOST_PAGEABLE;
}

int one(uint8_t type, const void *data, size_t n, uint32_t start_raw, uint32_t *out_raw, void *stream) {
  if (!out_raw || (!data && n)) return H3C_ERR_INVALID_ARG;
  const h3c_desc d{data, n, start_raw, type, mem_kind(data), 0};
  uint8_t t = 0;
  return h3c_batch_create(&d, 1, &t, out_raw, stream);
}
// folly's signature has no error channel: a wrong checksum would be silent, so fail loudly
[[noreturn]] void folly_abort(const char *what, int rc) {
  std::fprintf(stderr, "%s: engine error %d: %s\n", what, rc, h3c_last_error());
  std::abort();
}
}  // namespace

extern "C" {

int h3c_crc32c(const void *data, size_t n, uint32_t start_raw, uint32_t *out_raw, void *stream) {
  return one(H3C_TYPE_CRC32C, data, n, start_raw, out_raw, stream);
}

int h3c_crc32(const void *data, size_t n, uint32_t start_raw, uint32_t *out_raw, void *stream) {
  return one(H3C_TYPE_CRC32, data, n, start_raw, out_raw, stream);
}

uint32_t h3c_folly_crc32c(const uint8_t *data, size_t nbytes, uint32_t startingChecksum) {
  uint32_t v = 0;
  const int rc = one(H3C_TYPE_CRC32C, data, nbytes, startingChecksum, &v, nullptr);
  if (rc) folly_abort("h3c_folly_crc32c", rc);
  return v;
}

uint32_t h3c_folly_crc32(const uint8_t *data, size_t nbytes, uint32_t startingChecksum) {
  uint32_t v = 0;
  const int rc = one(H3C_TYPE_CRC32, data, nbytes, startingChecksum, &v, nullptr);
  if (rc) folly_abort("h3c_folly_crc32", rc);
  return v;
}

uint32_t h3c_serde_checksum_mark(uint32_t crc0, int compressed) { return serde_mark(crc0, compressed); }

int h3c_batch_serde_checksum(const h3c_desc *d, size_t n, const uint8_t *compressed, uint32_t *out, void *stream) {
  if (n == 0) return H3C_OK;
  if (!d || !out) return H3C_ERR_INVALID_ARG;
  const int rc = create_with(d, n, nullptr, 0u, out, stream);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i) out[i] = serde_mark(out[i], compressed ? compressed[i] : 0);
  return H3C_OK;
}

int h3c_batch_serde_verify(const h3c_desc *d, size_t n, const uint32_t *received, uint8_t *ok, uint64_t *n_bad,
                           void *stream) {
  if (n_bad) *n_bad = 0;
  if (n == 0) return H3C_OK;
  if (!d || !received || !ok) return H3C_ERR_INVALID_ARG;
  std::vector<uint32_t> crc(n);
  const int rc = create_with(d, n, nullptr, 0u, crc.data(), stream);
  if (rc) return rc;
  uint64_t bad = 0;
  for (size_t i = 0; i < n; ++i) {
    // MessageHeader::isCompressed (MessageHeader.h:26): bit 0 of the received checksum
    ok[i] = serde_mark(crc[i], received[i] & 1u) == received[i];
    bad += !ok[i];
  }
  if (n_bad) *n_bad = bad;
  return H3C_OK;
}

uint32_t h3c_std_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  // std(AB) = shift(std(A), |B|) ^ std(B): the same shift-XOR as folly's combine
  return h3c_crc32c_combine(crc1, crc2, len2);
}

int h3c_batch_std_crc32c(const h3c_desc *d, size_t n, const uint32_t *append_to, uint32_t *out_std, void *stream) {
  if (n == 0) return H3C_OK;
  if (!d || !out_std) return H3C_ERR_INVALID_ARG;
  const int rc = create_with(d, n, append_to, 0xFFFFFFFFu, out_std, stream);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i) out_std[i] = ~out_std[i];
  return H3C_OK;
}

int h3c_checksum_combine(uint8_t *type, uint32_t *value, uint8_t o_type, uint32_t o_value, uint64_t length) {
  if (!type || !value) return H3C_ERR_INVALID_ARG;
  if (*type != H3C_TYPE_NONE && *type != o_type) return H3C_ERR_CHECKSUM_MISMATCH;  // :181-184
  if (length == 0) return H3C_OK;                                                   // :185
  switch (*type) {
    case H3C_TYPE_NONE:  // :187-189
      *type = o_type;
      *value = o_value;
      break;
    case H3C_TYPE_CRC32C:  // :191
      *value = h3c_crc32c_combine(~*value, o_value, length);
      break;
    case H3C_TYPE_CRC32:  // :195
      *value = h3c_crc32_combine(~*value, o_value, length);
      break;
    default:
      return H3C_ERR_INVALID_ARG;
  }
  return H3C_OK;
}

int h3c_combine_fold(const uint8_t *types, const uint32_t *values, const uint64_t *lens, const uint64_t *group_begin,
                     size_t ngroups, uint8_t *out_type, uint32_t *out_value, uint32_t *status) {
  if (ngroups && (!group_begin || !out_type || !out_value || !status)) return H3C_ERR_INVALID_ARG;
  for (size_t g = 0; g < ngroups; ++g) {
    const uint64_t b = group_begin[g], e = group_begin[g + 1];
    uint8_t t = H3C_TYPE_NONE;
    uint32_t v = 0;
    uint32_t s = H3C_OK;
    for (uint64_t k = b; k < e; ++k) {
      if (k == b) {  // first piece: parentIO->result = splittedIO.result (:1624-1627)
        t = types[k];
        v = values[k];
        continue;
      }
      const int rc = h3c_checksum_combine(&t, &v, types[k], values[k], lens[k]);  // :1630
      if (rc) {
        s = (uint32_t)rc;
        break;
      }
    }
    out_type[g] = t;
    out_value[g] = v;
    status[g] = s;
  }
  return H3C_OK;
}

int h3c_batch_read_result(uint8_t batch_type, const h3c_read_job *jobs, size_t n, uint8_t *out_type,
                          uint32_t *out_value, uint32_t *status, void *stream) {
  return h3c_batch_read_result_ex(batch_type, jobs, n, out_type, out_value, status, nullptr, stream);
}

int h3c_batch_read_result_ex(uint8_t batch_type, const h3c_read_job *jobs, size_t n, uint8_t *out_type,
                             uint32_t *out_value, uint32_t *status, uint64_t *n_checksum_mismatch, void *stream) {
  if (n_checksum_mismatch) *n_checksum_mismatch = 0;
  if (n == 0) return H3C_OK;
  if (!jobs || !out_type || !out_value || !status) return H3C_ERR_INVALID_ARG;
  if (batch_type > H3C_TYPE_CRC32) return H3C_ERR_INVALID_ARG;
  // one batch of payload CRCs: the read-data checksums (:33-34) and the full-chunk
  // recalculations (:43-44)
  std::vector<h3c_desc> dd;
  std::vector<int64_t> compute_at(n, -1), recalc_at(n, -1);
  for (size_t i = 0; i < n; ++i) {
    const h3c_read_job &j = jobs[i];
    const bool full = j.offset == 0 && j.length == j.chunk_len;
    if (batch_type != H3C_TYPE_NONE && !(batch_type == j.chunk_type && full)) {
      compute_at[i] = (int64_t)dd.size();
      dd.push_back(h3c_desc{j.data, j.length, 0xFFFFFFFFu, batch_type, j.mem, 0});
    }
    if (j.recalculate && full) {
      recalc_at[i] = (int64_t)dd.size();
      dd.push_back(h3c_desc{j.data, j.length, 0xFFFFFFFFu, j.chunk_type, j.mem, 0});
    }
  }
  std::vector<uint8_t> t(dd.size());
  std::vector<uint32_t> v(dd.size());
  if (!dd.empty()) {
    const int rc = h3c_batch_create(dd.data(), dd.size(), t.data(), v.data(), stream);
    if (rc) return rc;
  }
  for (size_t i = 0; i < n; ++i) {
    const h3c_read_job &j = jobs[i];
    status[i] = H3C_OK;
    if (batch_type == H3C_TYPE_NONE) {  // :28-29
      out_type[i] = H3C_TYPE_NONE;
      out_value[i] = 0;
    } else if (compute_at[i] < 0) {  // :30-31 full chunk of the same type: the stored checksum
      out_type[i] = j.chunk_type;
      out_value[i] = j.chunk_value;
    } else {  // :33-34
      out_type[i] = t[compute_at[i]];
      out_value[i] = v[compute_at[i]];
    }
    if (recalc_at[i] >= 0 && (t[recalc_at[i]] != j.chunk_type || v[recalc_at[i]] != j.chunk_value)) {
      status[i] = H3C_ERR_CHECKSUM_MISMATCH;  // :45-53
      if (n_checksum_mismatch) ++*n_checksum_mismatch;  // storage.aio.checksum_mismatch (:14, :46)
    }
  }
  return H3C_OK;
}

}  // extern "C"
