/*
 * crc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's CRC32C chunk-checksum path, used as the
 * parity checker for the MI355X engine.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (3fs_amd/, include/h3c_crc.h) never links or calls it.
 *
 * Register convention ("raw") is folly's: init ~0 by default, NO final XOR.
 * std CRC32C = ~raw.  See SURVEY.md §8(a) rows A1-A12 for the functions this
 * restates; each definition in crc_oracle.c cites the reference file:line.
 */
#ifndef HF3FS_CRC_ORACLE_H
#define HF3FS_CRC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_POLY_CRC32C 0x82F63B78u /* reflected Castagnoli */
#define ORC_POLY_CRC32 0xEDB88320u  /* reflected IEEE 802.3 */

enum { ORC_NONE = 0, ORC_CRC32C = 1, ORC_CRC32 = 2 };
enum { ORC_OK = 0, ORC_ERR_CHECKSUM_MISMATCH = 4080, ORC_ERR_CHUNK_READ_FAILED = 4010,
       ORC_ERR_CHUNK_SIZE_MISMATCH = 4015 };

/* --- A1: folly::crc32c / folly::crc32, three independent mechanisms --- */
uint32_t orc_crc32c_bitwise(const uint8_t *d, size_t n, uint32_t start);
uint32_t orc_crc32c_table(const uint8_t *d, size_t n, uint32_t start);
uint32_t orc_crc32c_sse42(const uint8_t *d, size_t n, uint32_t start);
/* folly-faithful hardware path: 3 interleaved crc32q streams + shift combine.
 * This is the CPU baseline ("port" of folly's SSE4.2 crc32c_hw). */
uint32_t orc_crc32c_sse42_3way(const uint8_t *d, size_t n, uint32_t start);
uint32_t orc_crc32_table(const uint8_t *d, size_t n, uint32_t start);
/* Best-case CPU (not the reference's path): AVX-512 VPCLMULQDQ folding + crc32q
 * reduction; falls back to the 3-way path without AVX-512 / VPCLMULQDQ. */
uint32_t orc_crc32c_vpclmul(const uint8_t *d, size_t n, uint32_t start);
int orc_has_vpclmul(void);

/* --- A2: GF(2) shift / combine --- */
uint32_t orc_gf_mul(uint32_t a, uint32_t b, uint32_t poly);
uint32_t orc_xpow8n(uint64_t n, uint32_t poly); /* x^(8n) mod P, reflected */
uint32_t orc_shift(uint32_t crc, uint64_t nbytes, uint32_t poly);
uint32_t orc_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2);
uint32_t orc_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2);

/* --- A3/A4: ChecksumInfo::create / combine --- */
void orc_checksum_create(uint8_t type, const uint8_t *buf, uint64_t len, uint32_t start, uint8_t *out_type,
                         uint32_t *out_value);
int orc_checksum_combine(uint8_t *type, uint32_t *value, uint8_t o_type, uint32_t o_value, uint64_t length);

/* --- A8: ChunkReplica::updateChecksum restated over an in-memory chunk --- */
typedef struct {
  uint32_t size;           /* meta.size AFTER the write was applied */
  uint8_t checksum_type;   /* meta.checksumType before */
  uint32_t checksum_value; /* meta.checksumValue before */
} orc_chunk_meta;

typedef struct {
  uint32_t offset;
  uint32_t length;
  uint8_t checksum_type;
  uint32_t checksum_value;
  uint8_t is_truncate_or_extend;
} orc_write_io;

int orc_update_checksum(orc_chunk_meta *meta, orc_write_io wio, uint32_t chunk_size_before_write, int is_append_write,
                        const uint8_t *chunk_after_write);
/* which branch of updateChecksum ran: the reference's counters
 * storage.chunk_update.checksum_{none,reuse,combine,read_chunk} (ChunkReplica.cc:25-28,336-389) */
enum { ORC_CASE_NOT_RUN = 0, ORC_CASE_NONE = 1, ORC_CASE_REUSE = 2, ORC_CASE_COMBINE = 3, ORC_CASE_READ_CHUNK = 4,
       ORC_CASE_KEEP = 5 /* Rust engine: checksum untouched */ };
int orc_update_checksum_case(orc_chunk_meta *meta, orc_write_io wio, uint32_t chunk_size_before_write,
                             int is_append_write, const uint8_t *chunk_after_write, int *ucase);

/* --- A6 + A8: ChunkReplica::update restated over an in-memory chunk ---
 * One UpdateIO (WRITE / TRUNCATE / EXTEND) applied to `chunk` (capacity chunk_size):
 * range check, client-checksum verify, zero fill of gaps, the write / truncate /
 * extend itself, then updateChecksum.  `meta` is updated in place. */
enum { ORC_UPD_WRITE = 1, ORC_UPD_REMOVE = 2, ORC_UPD_TRUNCATE = 4, ORC_UPD_EXTEND = 8, ORC_UPD_COMMIT = 16 };
typedef struct {
  uint8_t kind; /* UpdateType (Common.h:51-58) */
  uint32_t offset;
  uint32_t length;
  uint8_t checksum_type;
  uint32_t checksum_value;
  uint8_t syncing; /* UpdateOptions.isSyncing (ChunkReplica.cc:211-215, 289) */
} orc_update_io;
typedef struct {
  int status;    /* 0, 3 kInvalidArg, 4015 kChunkSizeMismatch, 4080 kChecksumMismatch */
  uint32_t size; /* meta.size after */
  uint8_t type;  /* result.checksum */
  uint32_t value;
  int ucase; /* ORC_CASE_*: the counter the op increments */
} orc_update_result;
int orc_chunk_replica_update(orc_chunk_meta *meta, uint8_t *chunk, uint32_t chunk_size, const orc_update_io *io,
                             const uint8_t *payload, orc_update_result *res);
/* with UpdateIO.chunkSize (io_chunk_size) distinct from the chunk's (chunk_size): :141-145, :171-180 */
int orc_chunk_replica_update_cs(orc_chunk_meta *meta, uint8_t *chunk, uint32_t chunk_size, uint32_t io_chunk_size,
                                const orc_update_io *io, const uint8_t *payload, orc_update_result *res);

/* --- A10 + A11: Rust chunk engine update (std domain; meta->checksum_value is std) --- */
typedef struct {
  uint64_t reuse, combine, recalculate; /* metrics.rs:12-14 checksum_{reuse,combine,recalculate} */
} orc_engine_counters;
int orc_chunk_engine_update(orc_chunk_meta *meta, uint8_t *chunk, uint32_t chunk_size, const orc_update_io *io,
                            const uint8_t *payload, int payload_aligned, orc_update_result *res,
                            orc_engine_counters *cnt);

/* --- A7: AioReadJob::setResult checksum selection (recalculate path) --- */
int orc_read_result_checksum(uint8_t batch_type, uint8_t chunk_type, uint32_t chunk_value, uint32_t chunk_len,
                             uint32_t read_offset, uint32_t read_len, const uint8_t *read_data,
                             int recalculate, const uint8_t *full_chunk, uint8_t *out_type, uint32_t *out_value);

/* --- synthetic data --- */
uint64_t orc_splitmix64(uint64_t x);
void orc_fill_splitmix(uint8_t *out, uint64_t len, uint64_t seed, uint64_t chunk_idx);

/* --- batch helpers for the CPU baseline --- */
void orc_batch_crc32c(const uint8_t *base, uint64_t chunk_len, uint64_t nchunks, uint32_t start, int nthreads,
                      int variant, uint32_t *out);

double orc_time_crc32c_calls(const uint8_t *buf, uint64_t len, uint64_t calls);

#ifdef __cplusplus
}
#endif

#endif
