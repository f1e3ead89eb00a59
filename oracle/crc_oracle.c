/*
 * crc_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of the reference's checksum path.  Nothing in the
 * product (3fs_amd/, include/) links this file; the HIP engine must fail
 * loudly rather than fall back to it.
 *
 * Sources restated (paths relative to the reference checkout):
 *   folly::crc32c / crc32c_combine  -- external (third_party/folly is an empty
 *       submodule, .gitmodules:4-6; pin unrecoverable).  Semantics pinned by the
 *       reference's own call sites: src/fbs/storage/Common.h:158,191 and the
 *       combine identity in tests/common/utils/TestFolly.cc:9-18.
 *   ChecksumInfo::create / combine  -- src/fbs/storage/Common.h:113-201
 *   ChunkReplica::updateChecksum    -- src/storage/store/ChunkReplica.cc:319-394
 *   ChunkFileView::checksum         -- src/storage/store/ChunkFileView.cc:92-104
 *   AioReadJob::setResult checksum  -- src/storage/aio/BatchReadJob.cc:24-55
 *   ChunkReplica::update            -- src/storage/store/ChunkReplica.cc:131-317
 *   Rust Engine::update_chunk       -- src/storage/chunk_engine/src/core/engine.rs:288-429,
 *       Chunk::copy_on_write / safe_write (src/storage/chunk_engine/src/alloc/chunk.rs:89-281)
 *
 * Three independent CRC mechanisms (bitwise, byte table, x86 SSE4.2 crc32
 * instruction) cross-check one another; tests pin them to the standard KATs
 * and to the constants logged in tests/common/utils/TestFolly.cc:20-21.
 */
#include "crc_oracle.h"

#include <nmmintrin.h>
#include <pthread.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* A1: register-level CRC (folly "raw" convention: no final XOR).      */
/* ------------------------------------------------------------------ */

uint32_t orc_crc32c_bitwise(const uint8_t *d, size_t n, uint32_t start) {
  uint32_t c = start;
  for (size_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (ORC_POLY_CRC32C & (0u - (c & 1u)));
  }
  return c;
}

static uint32_t g_tab_c[256], g_tab_ieee[256];
static uint32_t g_long_shift[4][256], g_short_shift[4][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

#define ORC_LONG 8192
#define ORC_SHORT 256

static void build_byte_table(uint32_t *t, uint32_t poly) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (poly & (0u - (c & 1u)));
    t[i] = c;
  }
}

static void build_shift_table(uint32_t t[4][256], uint64_t nbytes) {
  uint32_t m = orc_xpow8n(nbytes, ORC_POLY_CRC32C);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) t[k][b] = orc_gf_mul(b << (8 * k), m, ORC_POLY_CRC32C);
}

static void init_tables(void) {
  build_byte_table(g_tab_c, ORC_POLY_CRC32C);
  build_byte_table(g_tab_ieee, ORC_POLY_CRC32);
  build_shift_table(g_long_shift, ORC_LONG);
  build_shift_table(g_short_shift, ORC_SHORT);
}

uint32_t orc_crc32c_table(const uint8_t *d, size_t n, uint32_t start) {
  pthread_once(&g_once, init_tables);
  uint32_t c = start;
  for (size_t i = 0; i < n; ++i) c = g_tab_c[(c ^ d[i]) & 0xFFu] ^ (c >> 8);
  return c;
}

uint32_t orc_crc32_table(const uint8_t *d, size_t n, uint32_t start) {
  pthread_once(&g_once, init_tables);
  uint32_t c = start;
  for (size_t i = 0; i < n; ++i) c = g_tab_ieee[(c ^ d[i]) & 0xFFu] ^ (c >> 8);
  return c;
}

uint32_t orc_crc32c_sse42(const uint8_t *d, size_t n, uint32_t start) {
  uint64_t c = start;
  while (n && ((uintptr_t)d & 7u)) {
    c = _mm_crc32_u8((uint32_t)c, *d++);
    --n;
  }
  for (; n >= 8; n -= 8, d += 8) {
    uint64_t w;
    memcpy(&w, d, 8);
    c = _mm_crc32_u64(c, w);
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *d++);
  return (uint32_t)c;
}

static inline uint32_t shift_by_table(uint32_t t[4][256], uint32_t c) {
  return t[0][c & 0xFFu] ^ t[1][(c >> 8) & 0xFFu] ^ t[2][(c >> 16) & 0xFFu] ^ t[3][c >> 24];
}

/* Three independent crc32q dependency chains over adjacent blocks, merged by
 * register shifts -- the structure of folly's SSE4.2 crc32c_hw path (the
 * instruction has 3-cycle latency / 1-cycle throughput, so 3 chains saturate
 * it).  Block sizes 8 KiB then 256 B. */
static inline const uint8_t *three_way(const uint8_t *d, size_t *n, uint64_t *c0p, size_t blk,
                                       uint32_t t[4][256]) {
  uint64_t c0 = *c0p;
  while (*n >= 3 * blk) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t *end = d + blk;
    do {
      uint64_t w0, w1, w2;
      memcpy(&w0, d, 8);
      memcpy(&w1, d + blk, 8);
      memcpy(&w2, d + 2 * blk, 8);
      c0 = _mm_crc32_u64(c0, w0);
      c1 = _mm_crc32_u64(c1, w1);
      c2 = _mm_crc32_u64(c2, w2);
      d += 8;
    } while (d < end);
    c0 = shift_by_table(t, (uint32_t)c0) ^ (uint32_t)c1;
    c0 = shift_by_table(t, (uint32_t)c0) ^ (uint32_t)c2;
    d += 2 * blk;
    *n -= 3 * blk;
  }
  *c0p = c0;
  return d;
}

uint32_t orc_crc32c_sse42_3way(const uint8_t *d, size_t n, uint32_t start) {
  pthread_once(&g_once, init_tables);
  uint64_t c = start;
  while (n && ((uintptr_t)d & 7u)) {
    c = _mm_crc32_u8((uint32_t)c, *d++);
    --n;
  }
  d = three_way(d, &n, &c, ORC_LONG, g_long_shift);
  d = three_way(d, &n, &c, ORC_SHORT, g_short_shift);
  for (; n >= 8; n -= 8, d += 8) {
    uint64_t w;
    memcpy(&w, d, 8);
    c = _mm_crc32_u64(c, w);
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *d++);
  return (uint32_t)c;
}

/* ------------------------------------------------------------------ */
/* Best-case CPU (not the reference's path): carry-less-multiply folding */
/* with AVX-512 VPCLMULQDQ (16 x 128-bit accumulators, 256 B per step),  */
/* reduced to 32 bits with two crc32q.  The accumulator holds a virtual  */
/* 16-byte message: loaded little-endian, integer bit q <-> x^(127-q).   */
/* A 64-bit clmul of two such bit-reversed operands yields the product   */
/* times x, so folding X = Xh*x^64 + Xl forward by F bits uses           */
/* Xh * x^(F+63) and Xl * x^(F-1) (each constant reversed into the top   */
/* half of a 64-bit lane).  Constants are derived with orc_gf_mul.       */
/* ------------------------------------------------------------------ */
#include <immintrin.h>

static uint32_t xpow_bits(uint64_t k) { /* x^k mod P (CRC32C), reflected */
  uint32_t r = 0x80000000u, b = 0x40000000u;
  while (k) {
    if (k & 1u) r = orc_gf_mul(r, b, ORC_POLY_CRC32C);
    b = orc_gf_mul(b, b, ORC_POLY_CRC32C);
    k >>= 1;
  }
  return r;
}
static uint64_t g_fold[8][2]; /* [0] 2048, [1] 1536, [2] 1024, [3] 512, [4] 384, [5] 256, [6] 128 bits */
static pthread_once_t g_fold_once = PTHREAD_ONCE_INIT;
static void init_fold(void) {
  static const uint64_t F[7] = {2048, 1536, 1024, 512, 384, 256, 128};
  for (int i = 0; i < 7; ++i) {
    g_fold[i][0] = (uint64_t)xpow_bits(F[i] + 63) << 32; /* multiplies the low qword (high degrees) */
    g_fold[i][1] = (uint64_t)xpow_bits(F[i] - 1) << 32;  /* multiplies the high qword */
  }
}

__attribute__((target("pclmul,sse4.2"))) static inline __m128i fold128(__m128i x, int f, __m128i d) {
  const __m128i k = _mm_set_epi64x((long long)g_fold[f][1], (long long)g_fold[f][0]);
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), d);
}

__attribute__((target("avx512f,avx512vl,vpclmulqdq,pclmul,sse4.2"))) static uint32_t crc32c_vpclmul(
    const uint8_t *d, size_t n, uint32_t start) {
  uint64_t c = start;
  if (n < 512) {
    for (; n >= 8; n -= 8, d += 8) {
      uint64_t w;
      memcpy(&w, d, 8);
      c = _mm_crc32_u64(c, w);
    }
    while (n--) c = _mm_crc32_u8((uint32_t)c, *d++);
    return (uint32_t)c;
  }
  pthread_once(&g_fold_once, init_fold);
  __m512i x0 = _mm512_loadu_si512((const void *)d), x1 = _mm512_loadu_si512((const void *)(d + 64));
  __m512i x2 = _mm512_loadu_si512((const void *)(d + 128)), x3 = _mm512_loadu_si512((const void *)(d + 192));
  x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)start)));
  d += 256;
  n -= 256;
  const __m512i k2048 = _mm512_broadcast_i32x4(_mm_set_epi64x((long long)g_fold[0][1], (long long)g_fold[0][0]));
#define FOLD512(x, k, v) _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00), \
                                                   _mm512_clmulepi64_epi128(x, k, 0x11), v, 0x96)
  while (n >= 256) {
    x0 = FOLD512(x0, k2048, _mm512_loadu_si512((const void *)d));
    x1 = FOLD512(x1, k2048, _mm512_loadu_si512((const void *)(d + 64)));
    x2 = FOLD512(x2, k2048, _mm512_loadu_si512((const void *)(d + 128)));
    x3 = FOLD512(x3, k2048, _mm512_loadu_si512((const void *)(d + 192)));
    d += 256;
    n -= 256;
  }
  /* 4 zmm -> 1: x0 by 1536 bits, x1 by 1024, x2 by 512, onto x3 */
  const __m512i k1536 = _mm512_broadcast_i32x4(_mm_set_epi64x((long long)g_fold[1][1], (long long)g_fold[1][0]));
  const __m512i k1024 = _mm512_broadcast_i32x4(_mm_set_epi64x((long long)g_fold[2][1], (long long)g_fold[2][0]));
  const __m512i k512 = _mm512_broadcast_i32x4(_mm_set_epi64x((long long)g_fold[3][1], (long long)g_fold[3][0]));
  __m512i a = FOLD512(x0, k1536, x3);
  a = FOLD512(x1, k1024, a);
  a = FOLD512(x2, k512, a);
#undef FOLD512
  /* 4 lanes -> 1: lane 0 by 384 bits, lane 1 by 256, lane 2 by 128, onto lane 3 */
  __m128i r = _mm512_extracti32x4_epi32(a, 3);
  r = fold128(_mm512_extracti32x4_epi32(a, 0), 4, r);
  r = fold128(_mm512_extracti32x4_epi32(a, 1), 5, r);
  r = fold128(_mm512_extracti32x4_epi32(a, 2), 6, r);
  for (; n >= 16; n -= 16, d += 16) r = fold128(r, 6, _mm_loadu_si128((const __m128i *)d));
  /* the accumulator is a 16-byte message: its CRC (init 0), then the tail */
  c = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(r));
  c = _mm_crc32_u64(c, (uint64_t)_mm_extract_epi64(r, 1));
  for (; n >= 8; n -= 8, d += 8) {
    uint64_t w;
    memcpy(&w, d, 8);
    c = _mm_crc32_u64(c, w);
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *d++);
  return (uint32_t)c;
}

int orc_has_vpclmul(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("vpclmulqdq");
}

uint32_t orc_crc32c_vpclmul(const uint8_t *d, size_t n, uint32_t start) {
  if (!orc_has_vpclmul()) return orc_crc32c_sse42_3way(d, n, start);
  return crc32c_vpclmul(d, n, start);
}

/* ------------------------------------------------------------------ */
/* A2: GF(2)[x]/P arithmetic in the reflected representation.          */
/* bit 31 holds the x^0 coefficient; multiplying by x is a right shift */
/* with conditional reduction by the reflected polynomial.             */
/* ------------------------------------------------------------------ */

uint32_t orc_gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b >> 1) ^ (poly & (0u - (b & 1u)));
  }
  return p;
}

uint32_t orc_xpow8n(uint64_t n, uint32_t poly) {
  uint32_t result = 0x80000000u; /* x^0 */
  uint32_t base = 0x00800000u;   /* x^8 */
  while (n) {
    if (n & 1u) result = orc_gf_mul(result, base, poly);
    base = orc_gf_mul(base, base, poly);
    n >>= 1;
  }
  return result;
}

uint32_t orc_shift(uint32_t crc, uint64_t nbytes, uint32_t poly) {
  return orc_gf_mul(crc, orc_xpow8n(nbytes, poly), poly);
}

/* folly::crc32c_combine(c1, c2, len2): the register after appending len2
 * bytes whose init-0 register is c2 to a stream whose register is c1.
 * Pinned by tests/common/utils/TestFolly.cc:16-18. */
uint32_t orc_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
  return orc_shift(c1, len2, ORC_POLY_CRC32C) ^ c2;
}

uint32_t orc_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
  return orc_shift(c1, len2, ORC_POLY_CRC32) ^ c2;
}

/* ------------------------------------------------------------------ */
/* A3/A4: ChecksumInfo (src/fbs/storage/Common.h:146-198).             */
/* ------------------------------------------------------------------ */

#define ORC_KCHUNK (1u << 20) /* ChecksumInfo::kChunkSize, Common.h:118 */

void orc_checksum_create(uint8_t type, const uint8_t *buf, uint64_t len, uint32_t start, uint8_t *out_type,
                         uint32_t *out_value) {
  /* Common.h:150: NONE -> {NONE, 0} */
  if (type == ORC_NONE) {
    *out_type = ORC_NONE;
    *out_value = 0;
    return;
  }
  /* MemoryDataIterator (Common.h:126-144) hands out <=1 MiB pieces; a null
   * buffer with length>0 yields no bytes -> iterBytes != length -> NONE
   * (Common.h:166-169). */
  if (buf == NULL && len > 0) {
    *out_type = ORC_NONE;
    *out_value = 0;
    return;
  }
  uint32_t v = start;
  uint64_t off = 0;
  while (off < len) {
    uint64_t piece = len - off < ORC_KCHUNK ? len - off : ORC_KCHUNK;
    if (type == ORC_CRC32C)
      v = orc_crc32c_sse42(buf + off, piece, v); /* Common.h:158 */
    else
      v = orc_crc32_table(buf + off, piece, v); /* Common.h:161 */
    off += piece;
  }
  *out_type = type;
  *out_value = v;
}

int orc_checksum_combine(uint8_t *type, uint32_t *value, uint8_t o_type, uint32_t o_value, uint64_t length) {
  /* Common.h:180-183 */
  if (*type != ORC_NONE && *type != o_type) return ORC_ERR_CHECKSUM_MISMATCH;
  if (length == 0) return ORC_OK; /* Common.h:184 */
  switch (*type) {
    case ORC_NONE: /* Common.h:186-188 */
      *type = o_type;
      *value = o_value;
      return ORC_OK;
    case ORC_CRC32C: /* Common.h:190-192 */
      *value = orc_crc32c_combine(~*value, o_value, length);
      return ORC_OK;
    case ORC_CRC32: /* Common.h:194-196 */
      *value = orc_crc32_combine(~*value, o_value, length);
      return ORC_OK;
  }
  return ORC_OK;
}

/* ChunkFileView::checksum(type, size, offset) over an in-memory chunk
 * (ChunkFileView.cc:92-104): create() over [offset, offset+size); a NONE
 * result maps to kChunkReadFailed. */
static int view_checksum(uint8_t type, const uint8_t *chunk, uint64_t size, uint64_t offset, uint8_t *t,
                         uint32_t *v) {
  orc_checksum_create(type, size ? chunk + offset : NULL, size, ~0u, t, v);
  if (*t == ORC_NONE) return ORC_ERR_CHUNK_READ_FAILED;
  return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* A8: ChunkReplica::updateChecksum (ChunkReplica.cc:319-394).          */
/* ------------------------------------------------------------------ */
int orc_update_checksum_case(orc_chunk_meta *meta, orc_write_io wio, uint32_t chunk_size_before_write,
                             int is_append_write, const uint8_t *chunk_after_write, int *ucase) {
  uint8_t ctype = meta->checksum_type;
  uint32_t cvalue = meta->checksum_value;
  int combine_checksum = chunk_size_before_write > 0 && is_append_write; /* :326 */

  if (wio.is_truncate_or_extend) { /* :328-332 */
    orc_checksum_create(meta->checksum_type, NULL, 0, ~0u, &wio.checksum_type, &wio.checksum_value);
    wio.offset = meta->size;
    wio.length = 0;
  }

  if (wio.checksum_type == ORC_NONE || meta->size == 0) { /* :334-336 */
    meta->checksum_value = 0;
    if (ucase) *ucase = ORC_CASE_NONE;
  } else if (wio.offset == 0 && wio.length == meta->size) { /* :337-339 reuse */
    meta->checksum_value = wio.checksum_value;
    if (ucase) *ucase = ORC_CASE_REUSE;
  } else if (wio.checksum_type == ctype && combine_checksum) { /* :340-355 append */
    int rc = orc_checksum_combine(&ctype, &cvalue, wio.checksum_type, wio.checksum_value, wio.length);
    if (rc) return rc;
    meta->checksum_value = cvalue;
    if (ucase) *ucase = ORC_CASE_COMBINE;
  } else { /* :356-390 prefix / write / suffix */
    uint8_t pt, st;
    uint32_t pv, sv;
    int rc = view_checksum(wio.checksum_type, chunk_after_write, wio.offset, 0, &pt, &pv);
    if (rc) return rc;
    uint32_t end = wio.offset + wio.length;
    uint32_t suffix_start = end < meta->size ? end : meta->size;
    uint32_t suffix_len = meta->size - suffix_start;
    rc = view_checksum(wio.checksum_type, chunk_after_write, suffix_len, suffix_start, &st, &sv);
    if (rc) return rc;
    orc_checksum_combine(&pt, &pv, wio.checksum_type, wio.checksum_value, wio.length);
    orc_checksum_combine(&pt, &pv, st, sv, suffix_len);
    meta->checksum_value = pv;
    if (ucase) *ucase = ORC_CASE_READ_CHUNK;
  }
  meta->checksum_type = wio.checksum_type; /* :392 */
  return ORC_OK;
}

int orc_update_checksum(orc_chunk_meta *meta, orc_write_io wio, uint32_t chunk_size_before_write, int is_append_write,
                        const uint8_t *chunk_after_write) {
  return orc_update_checksum_case(meta, wio, chunk_size_before_write, is_append_write, chunk_after_write, NULL);
}

/* ------------------------------------------------------------------ */
/* A6 + A8: ChunkReplica::update (ChunkReplica.cc:131-317) for WRITE,   */
/* REMOVE, TRUNCATE and EXTEND (plus options.isSyncing), and            */
/* ChunkReplica::commit's (no-)effect on the checksum (:397-467), with  */
/* the chunk file modelled as a byte array.                             */
/* ------------------------------------------------------------------ */
int orc_chunk_replica_update(orc_chunk_meta *meta, uint8_t *chunk, uint32_t chunk_size, const orc_update_io *io,
                             const uint8_t *payload, orc_update_result *res) {
  return orc_chunk_replica_update_cs(meta, chunk, chunk_size, chunk_size, io, payload, res);
}

/* The same with the op's own UpdateIO.chunkSize (`io_chunk_size`) beside the chunk's
 * innerFileId.chunkSize (`chunk_size`, also the capacity of `chunk`): the range check of
 * :141-145 uses the op's, and :171-180 fails a non-REMOVE op whose chunkSize differs from the
 * chunk's with kChunkSizeMismatch -- after :174 has set result.checksum = meta.checksum(). */
int orc_chunk_replica_update_cs(orc_chunk_meta *meta, uint8_t *chunk, uint32_t chunk_size, uint32_t io_chunk_size,
                                const orc_update_io *io, const uint8_t *payload, orc_update_result *res) {
  res->status = ORC_OK;
  res->size = meta->size;
  res->type = ORC_NONE; /* IOResult default until :174 */
  res->value = 0;
  res->ucase = ORC_CASE_NOT_RUN;
  if (io->kind == ORC_UPD_COMMIT) { /* ChunkReplica::commit sets no checksum (:397-467) */
    return ORC_OK;
  }
  const int is_remove = io->kind == ORC_UPD_REMOVE;
  /* :140-145 range check against writeIO.chunkSize (not for REMOVE) */
  if (!is_remove && (io->offset >= io_chunk_size || (uint64_t)io->offset + io->length > io_chunk_size)) {
    res->status = 3; /* StatusCode::kInvalidArg */
    return res->status;
  }
  res->type = meta->checksum_type; /* :174 result.checksum = meta.checksum() */
  res->value = meta->checksum_value;
  /* :171 chunkSize = isRemove ? meta.innerFileId.chunkSize : writeIO.chunkSize; :176-180 */
  if (!is_remove && io_chunk_size != chunk_size) {
    res->status = ORC_ERR_CHUNK_SIZE_MISMATCH;
    return res->status;
  }
  /* :193-207 verify the client's checksum of the payload */
  if (io->checksum_type != ORC_NONE && io->length != 0) {
    uint8_t t;
    uint32_t v;
    orc_checksum_create(io->checksum_type, payload, io->length, ~0u, &t, &v);
    if (t != io->checksum_type || v != io->checksum_value) {
      res->status = ORC_ERR_CHECKSUM_MISMATCH;
      return res->status;
    }
  }
  const int is_append = io->offset == meta->size; /* :246 */
  const uint32_t size_before = meta->size;       /* :256 */
  if (io->kind == ORC_UPD_TRUNCATE || io->kind == ORC_UPD_EXTEND) { /* :260-273 */
    if (io->length <= meta->size) {
      if (io->kind == ORC_UPD_TRUNCATE) meta->size = io->length;
    } else { /* extend with zeros */
      memset(chunk + meta->size, 0, io->length - meta->size);
      meta->size = io->length;
    }
  } else if (is_remove) { /* :274-279: no bytes change */
  } else { /* :281-291 WRITE: zero fill a gap, then the write */
    if (meta->size < io->offset) memset(chunk + meta->size, 0, io->offset - meta->size);
    if (io->length) memcpy(chunk + io->offset, payload, io->length);
    const uint32_t end = io->offset + io->length; /* doRealWrite :124 */
    if (end > meta->size) meta->size = end;
    if (io->syncing) meta->size = io->length; /* :289 options.isSyncing: full-chunk replace */
  }
  orc_write_io w;
  w.offset = io->offset;
  w.length = io->length;
  w.checksum_type = io->checksum_type;
  w.checksum_value = io->checksum_value;
  w.is_truncate_or_extend = io->kind == ORC_UPD_TRUNCATE || io->kind == ORC_UPD_EXTEND;
  int rc = orc_update_checksum_case(meta, w, size_before, is_append, chunk, &res->ucase); /* :298 */
  if (rc) {
    res->status = rc;
    return rc;
  }
  res->size = meta->size;
  res->type = meta->checksum_type; /* :311 result.checksum = meta.checksum() */
  res->value = meta->checksum_value;
  return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* A10 + A11: the Rust chunk engine's update in the std domain:         */
/* ChunkEngine::update's request mapping (src/storage/store/            */
/* ChunkEngine.cc:32-52, 61-67), Engine::update_chunk                   */
/* (src/storage/chunk_engine/src/core/engine.rs:288-429) and            */
/* Chunk::copy_on_write / safe_write (src/storage/chunk_engine/src/     */
/* alloc/chunk.rs:89-281), with the chunk's capacity = chunk_size       */
/* (offset + length past it is rejected before, like the C++ range      */
/* check).  meta->checksum_value is the std-domain crc32c (crate        */
/* 0.6.8: std = ~raw).  `payload_aligned` is is_aligned_buf's pointer   */
/* half (aligned.rs:47-49): it only changes the combine counter.        */
/* ------------------------------------------------------------------ */
#define ORC_ALIGN 4096u /* ALIGN_SIZE, chunk_engine/src/utils/aligned.rs:4 */

static uint32_t std_append(uint32_t std_c, const uint8_t *d, uint64_t n) { /* crc32c::crc32c_append */
  return ~orc_crc32c_table(d, n, ~std_c);
}

int orc_chunk_engine_update(orc_chunk_meta *meta, uint8_t *chunk, uint32_t chunk_size, const orc_update_io *io,
                            const uint8_t *payload, int payload_aligned, orc_update_result *res,
                            orc_engine_counters *cnt) {
  res->status = ORC_OK;
  res->size = meta->size;
  res->type = ORC_CRC32C;
  res->value = ~meta->checksum_value; /* ChunkEngine.cc:66: {CRC32C, ~out_checksum} */
  res->ucase = ORC_CASE_NOT_RUN;
  if (io->kind == ORC_UPD_COMMIT) { /* ChunkEngine::commit sets no checksum on the result */
    res->type = ORC_NONE;
    res->value = 0;
    return ORC_OK;
  }
  if (io->kind != ORC_UPD_REMOVE && (io->offset >= chunk_size || (uint64_t)io->offset + io->length > chunk_size)) {
    res->status = 3;
    res->type = ORC_NONE;
    res->value = 0;
    return res->status;
  }
  /* ChunkEngine.cc:33-52: the request */
  const int is_truncate = io->kind == ORC_UPD_TRUNCATE;
  const int is_remove = io->kind == ORC_UPD_REMOVE;
  const int is_write = io->kind == ORC_UPD_WRITE;
  uint32_t req_len = is_write ? io->length : 0;
  uint32_t req_off = is_write ? io->offset : io->length;
  const uint8_t *data = req_len ? payload : NULL;
  uint32_t req_checksum = 0;
  int without_checksum = 0;
  if (io->checksum_type == ORC_CRC32C) req_checksum = ~io->checksum_value;
  else if (payload) without_checksum = 1;
  /* engine.rs:297-312: verify the payload */
  if (req_len) {
    const uint32_t c = std_append(0, data, req_len);
    if (without_checksum) req_checksum = c;
    else if (c != req_checksum) {
      /* the error returns before out_checksum is set (engine.rs:303 vs :324): it stays 0, and
       * ChunkEngine.cc:66 reports {CRC32C, ~0} */
      res->status = ORC_ERR_CHECKSUM_MISMATCH;
      res->value = 0xFFFFFFFFu;
      return res->status;
    }
  }
  const uint32_t len = meta->size;
  if (is_remove) { /* engine.rs:376: the old chunk, unchanged */
    res->ucase = ORC_CASE_KEEP;
    return ORC_OK;
  }
  if (io->syncing || (req_len > 0 && req_off < len)) { /* engine.rs:377-391 copy_on_write */
    const uint32_t new_len = len > req_off + req_len ? len : req_off + req_len;
    const int skip_read = io->syncing || (req_off == 0 && req_len >= len); /* chunk.rs:112 */
    if (len < req_off) memset(chunk + len, 0, req_off - len);
    if (req_len) memcpy(chunk + req_off, data, req_len);
    uint32_t ck;
    if (skip_read) {
      ck = req_checksum; /* chunk.rs:152-154 */
      if (cnt) cnt->reuse++;
      res->ucase = ORC_CASE_REUSE;
    } else {
      ck = std_append(0, chunk, new_len); /* chunk.rs:156-157 */
      if (cnt) cnt->recalculate++;
      res->ucase = ORC_CASE_READ_CHUNK;
    }
    meta->size = io->syncing ? req_off + req_len : new_len; /* chunk.rs:166-170 */
    meta->checksum_value = ck;
  } else { /* safe_write, chunk.rs:176-281 */
    res->ucase = ORC_CASE_KEEP;
    if (is_truncate && req_off < len) { /* :184-197 */
      meta->size = req_off;
      meta->checksum_value = std_append(0, chunk, req_off);
      if (cnt) cnt->recalculate++;
      res->ucase = ORC_CASE_READ_CHUNK;
    } else if (len % ORC_ALIGN == 0 && req_off % ORC_ALIGN == 0 &&
               (req_len == 0 || (payload_aligned && req_len % ORC_ALIGN == 0))) { /* :200-234 */
      if (req_off > len) {
        memset(chunk + len, 0, req_off - len);
        meta->checksum_value = std_append(meta->checksum_value, chunk + len, req_off - len);
        meta->size = req_off;
        if (cnt) cnt->combine++;
        res->ucase = ORC_CASE_COMBINE;
      }
      if (req_len) {
        memcpy(chunk + req_off, data, req_len);
        meta->checksum_value = orc_crc32c_combine(meta->checksum_value, req_checksum, req_len);
        meta->size = req_off + req_len;
        if (cnt) cnt->combine++;
        res->ucase = ORC_CASE_COMBINE;
      }
    } else if (len < req_off + req_len) { /* :235-276 */
      if (len < req_off) memset(chunk + len, 0, req_off - len);
      if (req_len) memcpy(chunk + req_off, data, req_len);
      meta->checksum_value = std_append(meta->checksum_value, chunk + len, req_off + req_len - len);
      meta->size = req_off + req_len;
      if (cnt) cnt->combine++;
      res->ucase = ORC_CASE_COMBINE;
    }
  }
  res->size = meta->size;
  res->value = ~meta->checksum_value;
  return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* A7: AioReadJob::setResult (BatchReadJob.cc:24-55).                   */
/* ------------------------------------------------------------------ */
int orc_read_result_checksum(uint8_t batch_type, uint8_t chunk_type, uint32_t chunk_value, uint32_t chunk_len,
                             uint32_t read_offset, uint32_t read_len, const uint8_t *read_data, int recalculate,
                             const uint8_t *full_chunk, uint8_t *out_type, uint32_t *out_value) {
  if (batch_type == ORC_NONE) { /* :28-29 */
    *out_type = ORC_NONE;
    *out_value = 0;
  } else if (batch_type == chunk_type && read_offset == 0 && read_len == chunk_len) { /* :30-31 reuse */
    *out_type = chunk_type;
    *out_value = chunk_value;
  } else { /* :33-34 compute */
    orc_checksum_create(batch_type, read_data, read_len, ~0u, out_type, out_value);
  }
  if (recalculate && read_offset == 0 && read_len == chunk_len) { /* :43-54 */
    uint8_t rt;
    uint32_t rv;
    orc_checksum_create(chunk_type, full_chunk, read_len, ~0u, &rt, &rv);
    if (rt != chunk_type || rv != chunk_value) return ORC_ERR_CHECKSUM_MISMATCH;
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* Synthetic data: u64 w[k] = splitmix64(seed ^ (chunk_idx << 40) ^ k),  */
/* little-endian.                                        */
/* ------------------------------------------------------------------ */
uint64_t orc_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void orc_fill_splitmix(uint8_t *out, uint64_t len, uint64_t seed, uint64_t chunk_idx) {
  uint64_t key = seed ^ (chunk_idx << 40);
  uint64_t nw = len / 8;
  for (uint64_t k = 0; k < nw; ++k) {
    uint64_t w = orc_splitmix64(key ^ k);
    memcpy(out + 8 * k, &w, 8);
  }
  if (len % 8) {
    uint64_t w = orc_splitmix64(key ^ nw);
    memcpy(out + 8 * nw, &w, len % 8);
  }
}

/* ------------------------------------------------------------------ */
/* Batch helper (CPU baseline): equal-size chunks, optional threads.    */
/* variant 0 = folly-faithful 3-way crc32q, 1 = single crc32q stream,   */
/* 2 = byte table, 3 = VPCLMULQDQ folding (best-case CPU).  Each chunk goes through ChecksumInfo::create's 1 MiB */
/* iterator pieces, exactly as Common.h:146-172 chains folly::crc32c.    */
/* ------------------------------------------------------------------ */
typedef struct {
  const uint8_t *base;
  uint64_t chunk_len, lo, hi;
  uint32_t start;
  int variant;
  uint32_t *out;
} orc_job;

static uint32_t chunk_crc(const uint8_t *p, uint64_t len, uint32_t start, int variant) {
  uint32_t v = start;
  for (uint64_t off = 0; off < len; off += ORC_KCHUNK) {
    uint64_t piece = len - off < ORC_KCHUNK ? len - off : ORC_KCHUNK;
    if (variant == 0)
      v = orc_crc32c_sse42_3way(p + off, piece, v);
    else if (variant == 1)
      v = orc_crc32c_sse42(p + off, piece, v);
    else if (variant == 3)
      v = orc_crc32c_vpclmul(p + off, piece, v);
    else
      v = orc_crc32c_table(p + off, piece, v);
  }
  return v;
}

static void *batch_worker(void *arg) {
  orc_job *j = (orc_job *)arg;
  for (uint64_t i = j->lo; i < j->hi; ++i)
    j->out[i] = chunk_crc(j->base + i * j->chunk_len, j->chunk_len, j->start, j->variant);
  return NULL;
}

void orc_batch_crc32c(const uint8_t *base, uint64_t chunk_len, uint64_t nchunks, uint32_t start, int nthreads,
                      int variant, uint32_t *out) {
  pthread_once(&g_once, init_tables);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  orc_job jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].base = base;
    jobs[t].chunk_len = chunk_len;
    jobs[t].lo = nchunks * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].hi = nchunks * (uint64_t)(t + 1) / (uint64_t)nthreads;
    jobs[t].start = start;
    jobs[t].variant = variant;
    jobs[t].out = out;
  }
  if (nthreads == 1) {
    batch_worker(&jobs[0]);
    return;
  }
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* Per-call CPU time of ChecksumInfo::create's CRC (folly's 3-way SSE4.2 crc32c, variant 0) on
 * one `len`-byte buffer, repeated `calls` times: seconds per call.  The bench's CPU leg for the
 * synchronous small-call surface (BatchReadJob.cc:34, ChunkReplica.cc:194). */
#include <time.h>
double orc_time_crc32c_calls(const uint8_t *buf, uint64_t len, uint64_t calls) {
  pthread_once(&g_once, init_tables);
  struct timespec a, b;
  volatile uint32_t sink = 0;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (uint64_t i = 0; i < calls; ++i) sink ^= orc_crc32c_sse42_3way(buf, len, 0xFFFFFFFFu ^ (uint32_t)i);
  clock_gettime(CLOCK_MONOTONIC, &b);
  (void)sink;
  return ((double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec)) / (double)(calls ? calls : 1);
}
