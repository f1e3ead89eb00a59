/*
 * h3c_crc.h -- C ABI of the MI355X batched chunk-checksum engine for 3FS.
 *
 * Drop-in boundary for the checksum path of the 3FS storage service.  Every
 * entry point names the reference interface it replaces (paths relative to the
 * MingWangSong/3FS checkout).  Values use folly's "raw" register convention:
 * init ~0 by default, no final XOR (std CRC32C = ~raw).
 *
 *   folly::crc32c(const uint8_t*, size_t, uint32_t start = ~0U)
 *       called at src/fbs/storage/Common.h:158
 *   folly::crc32c_combine(uint32_t, uint32_t, size_t)
 *       called at src/fbs/storage/Common.h:191
 *   folly::crc32 / crc32_combine          src/fbs/storage/Common.h:161,195
 *   ChecksumInfo::create(type, buf, len, start)  src/fbs/storage/Common.h:146-177
 *   ChecksumInfo::combine(o, len)                src/fbs/storage/Common.h:179-198
 *   ChunkReplica::update payload verify          src/storage/store/ChunkReplica.cc:193-207
 *   AioReadJob::setResult (compute/recalculate)  src/storage/aio/BatchReadJob.cc:24-55
 *
 * No torch types appear here: plain pointers and sizes.  Streams are
 * hipStream_t passed as void* (NULL = the device's null stream).
 *
 * Thread safety: every function may be called concurrently from many host
 * threads (the reference calls the CPU path from 32 AIO + 32 update threads,
 * src/storage/aio/AioReadWorker.h:27, src/storage/update/UpdateWorker.h:15).
 * Global state is limited to immutable per-device tables built once.
 */
#ifndef H3C_CRC_H
#define H3C_CRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ChecksumType, src/fbs/storage/Common.h:66-70 */
enum h3c_type { H3C_TYPE_NONE = 0, H3C_TYPE_CRC32C = 1, H3C_TYPE_CRC32 = 2 };

/* Where a descriptor's payload lives. */
enum h3c_mem { H3C_MEM_DEVICE = 0, H3C_MEM_HOST_PINNED = 1, H3C_MEM_HOST_PAGEABLE = 2 };

/* Return codes (mapped to the reference's StatusCode values). */
enum h3c_status {
  H3C_OK = 0,
  H3C_ERR_INVALID_ARG = 3,            /* StatusCode::kInvalidArg */
  H3C_ERR_CHUNK_READ_FAILED = 4010,   /* StorageCode::kChunkReadFailed, StatusCodeDetails.h:160 */
  H3C_ERR_CHUNK_SIZE_MISMATCH = 4015, /* StorageCode::kChunkSizeMismatch, StatusCodeDetails.h:165 */
  H3C_ERR_CHECKSUM_MISMATCH = 4080,   /* StorageCode::kChecksumMismatch, StatusCodeDetails.h:186 */
  H3C_ERR_HIP = 9001,                 /* HIP runtime failure (h3c_last_error() has text) */
  H3C_ERR_NO_DEVICE = 9002
};

/* One chunk payload.  `start_raw` is ChecksumInfo::create's startingChecksum
 * (~0U for a fresh checksum).  `type` is an h3c_type, `mem` an h3c_mem. */
typedef struct h3c_desc {
  const void *ptr;
  uint64_t len;
  uint32_t start_raw;
  uint8_t type;
  uint8_t mem;
  uint16_t reserved;
} h3c_desc;

/* ---- scalar host arithmetic (combine is O(log n) GF(2) work, no payload) ---- */

/* folly::crc32c_combine (Common.h:191): shift(c1, len2) ^ c2. */
uint32_t h3c_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2);
/* folly::crc32_combine (Common.h:195), IEEE polynomial. */
uint32_t h3c_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2);
/* register advanced over `nbytes` zero bytes: crc * x^(8*nbytes) mod P. */
uint32_t h3c_crc32c_shift(uint32_t crc, uint64_t nbytes);

/* folly::crc32c(data, n, start) / folly::crc32(...) (Common.h:158,161) for one buffer, on
 * the GPU: device memory is read in place, host memory is staged (the kind is detected
 * with hipPointerGetAttributes).  *out_raw receives the raw register (no final XOR).
 * Synchronous; for many buffers use h3c_batch_create. */
int h3c_crc32c(const void *data, size_t n, uint32_t start_raw, uint32_t *out_raw, void *stream);
int h3c_crc32(const void *data, size_t n, uint32_t start_raw, uint32_t *out_raw, void *stream);
/* The same with folly's own signature and return convention, for a call site that is switched
 * by editing only the function name: folly::crc32c(const uint8_t* data, size_t nbytes,
 * uint32_t startingChecksum = ~0U) (folly/hash/Checksum.h; called at Common.h:158) and
 * folly::crc32(...) (Common.h:161).  The result is the raw register (no final XOR), as folly's.
 * folly's signature has no error channel: an engine failure (no device, a HIP error) prints
 * h3c_last_error() to stderr and aborts rather than return a wrong checksum.  Synchronous, on the
 * default stream; a call costs a GPU round trip, so per-IO host buffers belong on the CPU
 *  and this entry is for GPU-resident buffers at folly call sites.  Graph captures:
 * HIP fails legacy-stream launches while any stream of the process captures; these entries (and every
 * synchronous entry called with stream == NULL) wait while the engine itself captures an UpdateIO graph
 * (H3C_UPD_GRAPHS), so they never abort on the engine's own captures.  A caller that captures graphs
 * of its own must not call them meanwhile. */
uint32_t h3c_folly_crc32c(const uint8_t *data, size_t nbytes, uint32_t startingChecksum);
uint32_t h3c_folly_crc32(const uint8_t *data, size_t nbytes, uint32_t startingChecksum);

/* ---- engine lifetime ---- */

int h3c_device_count(void);
/* Builds the per-device constant tables.  Idempotent, thread-safe.  Every
 * other GPU entry point calls it implicitly for the current device. */
int h3c_init(int device);
const char *h3c_last_error(void); /* thread-local text of the last failure */

/* ---- synchronous batch API (ChecksumInfo semantics, host result arrays) ---- */

/* ChecksumInfo::create for each descriptor (Common.h:146-177):
 * NONE -> {NONE,0}; len==0 -> {type,start_raw}; ptr==NULL && len>0 -> {NONE,0}.
 * Device-memory payloads are read in place; host payloads are staged.
 * Blocks until results are in out_type/out_raw (host arrays, n entries). */
int h3c_batch_create(const h3c_desc *d, size_t n, uint8_t *out_type, uint32_t *out_raw, void *stream);

/* Recompute and compare against expected_raw (ChunkReplica.cc:193-207,
 * BatchReadJob.cc:43-54): ok[i] = (create(d[i]) == {d[i].type, expected_raw[i]}).
 * *n_mismatch receives the count of ok==0.  Returns H3C_OK even when some
 * chunks mismatch; per-chunk status is in ok[]. */
int h3c_batch_verify(const h3c_desc *d, const uint32_t *expected_raw, size_t n, uint32_t *out_raw, uint8_t *ok,
                     uint64_t *n_mismatch, void *stream);

/* Coalescing of concurrent synchronous calls (h3c_batch_create / h3c_batch_verify /
 * h3c_crc32c / h3c_crc32 on the default stream, stream == NULL): callers queue per device and
 * one of them runs everything queued as a single batch -- one staging copy, one launch, one
 * synchronisation -- for the reference's pattern of one ChecksumInfo::create per IO from many
 * AIO / update threads (BatchReadJob.cc:34, ChunkReplica.cc:194).  Results are identical; off
 * by default. */
int h3c_set_coalescing(int on);

/* ---- asynchronous plan API (device-resident descriptors and results) ---- */

typedef struct h3c_plan h3c_plan;

/* Upload descriptors (all H3C_MEM_DEVICE, on `device`) once; reuse the plan
 * for repeated create/verify of the same chunk set (scrub / resync). */
int h3c_plan_create(const h3c_desc *d, size_t n, int device, h3c_plan **out);
/* Enqueue on `stream`: out_raw_dev[i] (device, n u32).  When expected_raw_dev
 * is non-NULL also ok_dev[i] (device, n u8) and *mismatch_dev (device u32,
 * incremented, caller zeroes).  Nothing is synchronised. */
int h3c_plan_run(h3c_plan *p, const uint32_t *expected_raw_dev, uint32_t *out_raw_dev, uint8_t *ok_dev,
                 uint32_t *mismatch_dev, void *stream);
uint64_t h3c_plan_bytes(const h3c_plan *p);
void h3c_plan_destroy(h3c_plan *p);

/* ---- batched combine on device (folly::crc32c_combine per element) ---- */
/* out[i] = combine(c1[i], c2[i], len2[i]); all arrays device-resident. */
int h3c_batch_combine(uint8_t type, const uint32_t *c1_dev, const uint32_t *c2_dev, const uint64_t *len2_dev,
                      size_t n, uint32_t *out_dev, void *stream);

/* ---- batched partial updates (ChunkReplica::update + updateChecksum) ---- */

/* Apply `n_blocks` block-aligned overwrites, in sequence order, to device-resident
 * chunks and maintain their checksums, replacing the per-write prefix/suffix re-read
 * + two crc32c_combine()s of ChunkReplica::updateChecksum case (iv)
 * (src/storage/store/ChunkReplica.cc:356-390) with an O(write) GF(2) delta.
 *   chunk_base_dev[c]      device address of chunk c (chunk_len bytes, fully written)
 *   chunk_raw_in_dev[c]    its current raw checksum (ChunkMetadata.checksumValue)
 *   block write i          overwrites block blk_index_dev[i] (block_bytes at offset
 *                          blk_index*block_bytes) of chunk blk_chunk_dev[i] with
 *                          payload_dev + i*block_bytes
 *   out_raw_dev[i]         the chunk's raw checksum right after write i (what
 *                          updateChecksum stores), chunk_raw_out_dev[c] the final one.
 * block_bytes is a multiple of 1024 (3FS writes are 4 KiB-aligned, kAIOAlignSize).
 * A multi-block write is expanded by the caller into consecutive block writes; its
 * checksum is out_raw of its last block.  Out-of-range entries have no effect,
 * out_raw 0, and are counted in *n_invalid_dev (optional).  Chunks no write reaches keep
 * chunk_raw_in.  The chunk bytes are updated in place.  All arrays are device memory;
 * nothing is synchronised.  The stored checksums are trusted; h3c_update_blocks_ex
 * (below) has the exact mode and the case counters.
 * *n_invalid_dev == UINT32_MAX (counters.invalid == UINT64_MAX) reports a void batch: the
 * one-launch path chains its workgroups' per-chunk sums, and a workgroup that waited past its
 * bound (> 0.25 s, i.e. starved of its CU by other work) gave up.  The chunk bytes are right;
 * out_raw / chunk_raw_out of that call are not -- recompute them (h3c_plan_run over the chunks).
 * The one-launch path (4 KiB blocks, <= 128 chunks) keeps its hash heads, control words and
 * look-back state in a library-owned scratch per (device, stream) -- about 1 MiB plus 4 bytes
 * per write rounded up to a power of two, never cleared between batches (epoch-tagged) -- rather
 * than in the workspace; calls on one stream from several threads enqueue one at a time.  A call
 * made while the stream is being captured into a graph uses the workspace instead.  Up to 64 such scratches
 * live at once; past that the least recently used idle one is freed (after a device synchronisation) and
 * reused.  A stream that ran h3c_update_blocks batches is released with h3c_stream_release before it is
 * destroyed: a new stream may come back with the same handle value and must not inherit the scratch. */
int h3c_stream_release(void *stream);
size_t h3c_update_workspace_bytes(uint32_t n_blocks, uint32_t nchunks, uint64_t chunk_len, uint32_t block_bytes);
int h3c_update_blocks(uint8_t type, const uint64_t *chunk_base_dev, uint32_t nchunks, uint64_t chunk_len,
                      uint32_t block_bytes, const uint32_t *chunk_raw_in_dev, const uint32_t *blk_chunk_dev,
                      const uint32_t *blk_index_dev, const void *payload_dev, uint32_t n_blocks,
                      uint32_t *out_raw_dev, uint32_t *chunk_raw_out_dev, void *workspace_dev,
                      size_t workspace_bytes, uint32_t *n_invalid_dev, void *stream);

/* ---- general batched updates: every UpdateIO case of ChunkReplica::update ---- */

/* UpdateType (src/fbs/storage/Common.h:51-58).  REMOVE must carry offset 0, length 0 and a
 * NONE checksum (the form StorageOperator::doRemove builds, StorageOperator.cc:808-815); it
 * runs updateChecksum's case (i) and stores {NONE, 0} (Rust engine: leaves the checksum).
 * COMMIT (ChunkReplica::commit, ChunkReplica.cc:397-467) touches no byte and no checksum;
 * its result is {NONE, 0}.  Both pass through so an UpdateWorker queue can be drained into
 * one batch without filtering. */
enum h3c_update_kind {
  H3C_UPD_WRITE = 1,
  H3C_UPD_REMOVE = 2,
  H3C_UPD_TRUNCATE = 4,
  H3C_UPD_EXTEND = 8,
  H3C_UPD_COMMIT = 16
};

/* ChunkMetadata fields on the path (Common.h:662-676) plus where the bytes live. */
typedef struct h3c_chunk_state {
  uint64_t base;       /* device address of the chunk bytes, capacity chunk_size */
  uint32_t chunk_size; /* innerFileId.chunkSize: the write bound */
  uint32_t size;       /* meta.size            (in / out) */
  uint32_t value;      /* meta.checksumValue   (in / out; raw, std with H3C_UPD_STD_DOMAIN) */
  uint8_t type;        /* meta.checksumType    (in / out) */
  uint8_t reserved[3];
} h3c_chunk_state;

/* per-op flags (h3c_update_io.flags) */
#define H3C_IO_SYNCING 1u /* UpdateOptions.isSyncing: the resync successor's full-chunk replace
                             (ChunkReplica.cc:211-215, 289; chunk.rs:112, 166-170): WRITE at
                             offset 0 only (ReliableForwarding.cc:203-207), else kInvalidArg */

#define H3C_IO_CHUNK_SIZE 2u /* `chunk_size` carries UpdateIO.chunkSize (raw domain): the range check uses it
                                (ChunkReplica.cc:141-145, kInvalidArg) and a value other than the chunk's
                                innerFileId.chunkSize (the table's chunk_size) fails the op with
                                H3C_ERR_CHUNK_SIZE_MISMATCH (:171-180).  Without the flag the table's
                                chunk_size stands in for it.  The Rust engine path (H3C_UPD_STD_DOMAIN) has
                                no such check (ChunkEngine.cc:32-52) and ignores it. */

/* UpdateIO fields on the path (Common.h:326-345). */
typedef struct h3c_update_io {
  uint64_t payload;        /* device address of `length` bytes (WRITE) */
  uint32_t chunk;          /* index into the chunk table */
  uint32_t offset;
  uint32_t length;         /* WRITE: bytes; TRUNCATE / EXTEND: the new chunk length */
  uint32_t checksum_value; /* the client's ChecksumInfo of the payload */
  uint8_t checksum_type;
  uint8_t kind;            /* h3c_update_kind */
  uint8_t flags;           /* H3C_IO_* */
  uint8_t reserved;
  uint32_t chunk_size;     /* UpdateIO.chunkSize, read with H3C_IO_CHUNK_SIZE */
} h3c_update_io;

typedef struct h3c_update_result {
  uint32_t status; /* H3C_OK, H3C_ERR_INVALID_ARG (range, :140-145), H3C_ERR_CHUNK_SIZE_MISMATCH (:176-180),
                      H3C_ERR_CHECKSUM_MISMATCH (:193-207) */
  uint32_t size;   /* meta.size after the op */
  uint32_t value;  /* result.checksum after the op (meta.checksum(), ChunkReplica.cc:311; std domain:
                      the engine's out_checksum, 0 after a checksum mismatch, engine.rs:303,324) */
  uint8_t type;
  uint8_t reserved[3];
} h3c_update_result;

/* The reference's checksum case counters for one batch.
 *   ChunkReplica (raw domain): storage.chunk_update.checksum_{none,reuse,combine,read_chunk}
 *     (ChunkReplica.cc:25-28, incremented at :336,339,355,389) and the update path's
 *     storage.update.checksum_mismatch (StorageTarget.cc:331-332).
 *   Rust chunk engine (std domain): checksum_{reuse,combine,recalculate} (metrics.rs:12-14,
 *     chunk.rs:153,156,188,217,233,273); combine counts the aligned path's zero pad and append
 *     separately, as chunk.rs does (the pad/append split uses the payload's device address
 *     for is_aligned_buf, aligned.rs:47-49).
 *   stale_chunks (H3C_UPD_EXACT only): chunks whose stored checksum of the batch polynomial
 *     disagreed with their bytes -- the input the trusted mode would have carried forward. */
typedef struct h3c_update_counters {
  uint64_t none, reuse, combine, read_chunk; /* raw domain */
  uint64_t recalculate;                      /* std domain (reuse / combine shared) */
  uint64_t checksum_mismatch;                /* A6 failures (status 4080) */
  uint64_t invalid;                          /* status kInvalidArg */
  uint64_t stale_chunks;                     /* H3C_UPD_EXACT */
} h3c_update_counters;

/* flags */
#define H3C_UPD_STD_DOMAIN 1u /* Rust chunk engine (chunk_engine/src/alloc/chunk.rs:89-281): values are
                                 std-domain crc32c, Engine::update_chunk / copy_on_write / safe_write */
#define H3C_UPD_EXACT 2u      /* do not trust stored checksums: every chunk in the table with bytes is
                                 CRC'd once before the batch (see below) */
#define H3C_UPD_GRAPHS 4u     /* h3c_update_ios*: a batch shape this thread repeats on the same buffers
                                 runs its ~30-launch pipeline as one captured HIP graph.  The caller
                                 promises that no thread of the process launches onto the legacy
                                 default stream while the call runs (HIP fails such launches during
                                 a capture and voids the capture).  Off: plain launches. */

/* Apply `n` UpdateIOs in sequence order to device-resident chunks, replacing
 * ChunkReplica::update's per-op payload verify (ChunkReplica.cc:193-207), zero fill,
 * write / truncate / extend / remove (:256-294) and updateChecksum (:319-394, all four cases)
 * -- or, with H3C_UPD_STD_DOMAIN, Engine::update_chunk's verify and Chunk::copy_on_write /
 * safe_write's checksum (engine.rs:288-429, chunk.rs:89-281).  Arbitrary offsets and lengths;
 * writes to the same bytes are ordered.  Every op's result and every chunk's final state equal
 * the reference's replay of the same ops in sequence order, with one documented exception:
 *
 *   Stored checksums.  The reference's prefix / suffix case (iv) re-reads the chunk bytes, so
 *   its result does not depend on meta.checksumValue; its append case (iii) combines with it
 *   (and a TRUNCATE / EXTEND at offset == size keeps it).  By default (trusted mode) a stored
 *   checksum of `poly_type` is taken as the CRC of the chunk's bytes, and every op costs
 *   O(its own bytes): results are bit-exact whenever stored checksums are consistent with the
 *   bytes; on a chunk whose stored value is off by e (bit rot, a torn write), the reference
 *   heals e at its next case-(ii)/(iv) op while the trusted mode carries it, shifted with the
 *   chunk's length, until a full overwrite.  H3C_UPD_EXACT CRCs each chunk's bytes once
 *   first (O(chunk) per chunk per batch, not per op) and then reproduces the reference
 *   exactly, stale values included; counters->stale_chunks reports how many disagreed.
 *
 * A chunk whose stored checksum is not of `poly_type` (e.g. NONE) is CRC'd once either way.
 * Client checksums must be NONE or `poly_type` (the client's chunk_checksum_type), else the
 * op fails with H3C_ERR_INVALID_ARG; so does a TRUNCATE / EXTEND of a chunk whose stored
 * checksum at the start of the batch is of the other polynomial (raw domain).  `chunks` and
 * `results` are host arrays (pinned memory avoids a staging copy); chunk bytes are updated in
 * place on device.  All per-op and per-chunk work runs on the device; the host issues the
 * launches and copies and reads one count back at the end.  Synchronous on `stream`.  A chunk
 * whose size exceeds its chunk_size fails the whole call with H3C_ERR_INVALID_ARG, before any
 * work. */
int h3c_update_ios(uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios, uint32_t n,
                   h3c_update_result *results, uint32_t flags, void *stream);
/* The same, also returning the batch's case counters (counters may be NULL). */
int h3c_update_ios_ex(uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks, const h3c_update_io *ios,
                      uint32_t n, h3c_update_result *results, uint32_t flags, h3c_update_counters *counters,
                      void *stream);
/* The same with every array in device memory (chunk table in / out, ops, results, counters -- the
 * latter may be NULL): for callers whose op tables already live in HBM; no PCIe traffic.  A chunk
 * whose size exceeds its chunk_size fails its ops with H3C_ERR_INVALID_ARG.  Returns once the
 * batch's outcome is known (the host reads its outcome words back once, at the end): every output
 * is then complete for work ordered after the batch on `stream`; work on another stream orders
 * itself with an event recorded on `stream`.  (On the fast branch the call returns when the last
 * kernel has written its outputs and its outcome, without waiting for the stream's completion
 * signal; other paths synchronise the stream.) */
int h3c_update_ios_dev(uint8_t poly_type, h3c_chunk_state *chunks_dev, uint32_t nchunks, const h3c_update_io *ios_dev,
                       uint32_t n, h3c_update_result *results_dev, uint32_t flags, h3c_update_counters *counters_dev,
                       void *stream);

/* h3c_update_blocks with flags and counters.  flags: H3C_UPD_EXACT recomputes each chunk's
 * checksum from its bytes before the writes (one create pass over the chunk set), so every
 * out_raw / chunk_raw_out equals what updateChecksum case (iv) computes by re-reading the
 * chunk (ChunkReplica.cc:356-390) even where chunk_raw_in disagrees with the bytes; chunks no
 * write reaches keep chunk_raw_in, as the reference leaves their metadata alone.  Without it the
 * stored checksums are trusted (r' = r ^ delta; a stale r stays stale by its own error).
 * H3C_UPD_STD_DOMAIN is not accepted (the block path is raw).  counters_dev (device, may be
 * NULL) receives the batch's case counts: read_chunk per valid block write (reuse when a block
 * is the whole chunk), invalid entries, and with H3C_UPD_EXACT the stale chunks.
 * Asynchronous like h3c_update_blocks. */
int h3c_update_blocks_ex(uint8_t type, const uint64_t *chunk_base_dev, uint32_t nchunks, uint64_t chunk_len,
                         uint32_t block_bytes, const uint32_t *chunk_raw_in_dev, const uint32_t *blk_chunk_dev,
                         const uint32_t *blk_index_dev, const void *payload_dev, uint32_t n_blocks,
                         uint32_t *out_raw_dev, uint32_t *chunk_raw_out_dev, void *workspace_dev,
                         size_t workspace_bytes, uint32_t *n_invalid_dev, uint32_t flags,
                         h3c_update_counters *counters_dev, void *stream);

/* ---- adjacent formats on the same kernels ---- */

/* RPC message checksum, Checksum::calcSerde (src/common/net/MessageHeader.h:32-37):
 * folly::crc32c(data, size, 0) with its low 8 bits replaced by 0x86 | compressed. */
uint32_t h3c_serde_checksum_mark(uint32_t crc0, int compressed);
int h3c_batch_serde_checksum(const h3c_desc *d, size_t n, const uint8_t *compressed /* NULL = none */,
                             uint32_t *out, void *stream);
/* Processor::unpackSerdeMsg's check (src/common/net/Processor.h:113-117): ok[i] = the
 * recomputed calcSerde (compressed flag = bit 0 of received[i]) equals received[i]. */
int h3c_batch_serde_verify(const h3c_desc *d, size_t n, const uint32_t *received, uint8_t *ok, uint64_t *n_bad,
                           void *stream);

/* Rust crc32c crate 0.6.8 as the chunk engine uses it (std domain, std = ~raw;
 * chunk_engine/src/alloc/chunk.rs:152-269, core/engine.rs:297-312):
 * crc32c::crc32c_combine, and crc32c::crc32c (append_to == NULL) /
 * crc32c::crc32c_append(append_to[i], data) per descriptor (type is ignored). */
uint32_t h3c_std_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
int h3c_batch_std_crc32c(const h3c_desc *d, size_t n, const uint32_t *append_to, uint32_t *out_std, void *stream);

/* ChecksumInfo::combine (src/fbs/storage/Common.h:179-198) on a {type, value} pair:
 * H3C_ERR_CHECKSUM_MISMATCH (4080) on a type mismatch, no-op for length 0, a NONE
 * receiver copies o. */
int h3c_checksum_combine(uint8_t *type, uint32_t *value, uint8_t o_type, uint32_t o_value, uint64_t length);
/* The client's fold of split-read results (src/client/storage/StorageClientImpl.cc:1607-1633):
 * group g = pieces [group_begin[g], group_begin[g+1]); the first piece's checksum,
 * then combine(piece_k, lens[k]) for the rest.  status[g] = 0 or the combine error. */
int h3c_combine_fold(const uint8_t *types, const uint32_t *values, const uint64_t *lens, const uint64_t *group_begin,
                     size_t ngroups, uint8_t *out_type, uint32_t *out_value, uint32_t *status);

/* ---- read path: AioReadJob::setResult (src/storage/aio/BatchReadJob.cc:24-55) ---- */

/* One completed read job. */
typedef struct h3c_read_job {
  const void *data;     /* the bytes read (localbuf + headLength) */
  uint64_t length;      /* *lengthInfo */
  uint64_t chunk_len;   /* state.chunkLen */
  uint32_t offset;      /* readIO.offset */
  uint32_t chunk_value; /* state.chunkChecksum.value */
  uint8_t chunk_type;   /* state.chunkChecksum.type */
  uint8_t mem;          /* h3c_mem of data */
  uint8_t recalculate;  /* batch.recalculateChecksum() (resync reads, ReliableForwarding.cc:179-180) */
  uint8_t reserved[5];
} h3c_read_job;

/* result.checksum per job: {NONE,0} for a NONE batch; the stored chunk checksum when the
 * whole chunk is read with its own type; else create(batch_type, data, length).  With
 * `recalculate`, a whole-chunk read is re-checksummed with the stored type and a
 * difference sets status[i] = H3C_ERR_CHECKSUM_MISMATCH (4080). */
int h3c_batch_read_result(uint8_t batch_type, const h3c_read_job *jobs, size_t n, uint8_t *out_type,
                          uint32_t *out_value, uint32_t *status, void *stream);
/* The same, also counting the recalculation mismatches (the reference's
 * storage.aio.checksum_mismatch counter, BatchReadJob.cc:14, :46) into *n_checksum_mismatch
 * (may be NULL). */
int h3c_batch_read_result_ex(uint8_t batch_type, const h3c_read_job *jobs, size_t n, uint8_t *out_type,
                             uint32_t *out_value, uint32_t *status, uint64_t *n_checksum_mismatch, void *stream);

/* ---- host-fed pipeline (payloads in host memory, BASELINE config 5) ---- */

/* A reusable pipeline: two HBM staging windows of `window_bytes` and a copy stream.
 * h3c_hostfed_run streams the host payloads of `d` (pinned memory recommended:
 * hipHostMalloc / hipHostRegister'd RDMA buffers) through the windows, overlapping
 * H2D copies with the CRC kernels, and returns ChecksumInfo::create values (and, with
 * `expected`, verify flags) in host arrays.  Blocks until done.  One polynomial per
 * run.  A pipeline object must not be used by two threads at once. */
typedef struct h3c_hostfed h3c_hostfed;
int h3c_hostfed_create(int device, uint64_t window_bytes, h3c_hostfed **out);
/* Pinned host memory on the NUMA node of `device`'s PCIe root (NUMA-local
 * pinned buffers per GPU for config 5), the host-fed analogue of the storage service's
 * RDMA BufferPool (src/storage/service/StorageOperator.cc:546-558): anonymous pages bound
 * with mbind(MPOL_PREFERRED), faulted in, then hipHostRegister'd.  *node receives the
 * node, or -1 when it is unknown (the memory is then pinned without a binding).  Release
 * with h3c_host_free. */
int h3c_host_alloc(int device, uint64_t bytes, void **out, int *node);
int h3c_host_free(void *p);
int h3c_device_numa_node(int device); /* -1: unknown */
int h3c_hostfed_run(h3c_hostfed *h, const h3c_desc *d, size_t n, const uint32_t *expected_raw, uint32_t *out_raw,
                    uint8_t *ok, uint64_t *n_mismatch, void *stream);
void h3c_hostfed_destroy(h3c_hostfed *h);

/* ---- several GPUs of one process (3fs_amd/csrc/h3c_multi.hip) ---- */

/* The storage service is one process per node whose checksum callers are its AIO and update threads
 * (src/storage/aio/AioReadWorker.h:26, src/storage/update/UpdateWorker.h:15); the resync scrub is one
 * caller per target (src/storage/service/ReliableForwarding.cc:158-182 -> BatchReadJob.cc:43-54).  An
 * h3c_multi drives a list of devices from that one process: one host worker thread per entry (hipSetDevice
 * once, its own stream and host-fed pipeline with NUMA-local windows), each batch split across them and
 * run at once, results written into disjoint slices of the caller's host arrays.  No collective.  A device
 * may be listed twice (two workers on one GPU).  Calls on one object run one at a time; the entries are
 * synchronous.
 *
 * Partition: contiguous index ranges balanced by payload bytes (NONE / null descriptors weigh 0); cut k is
 * the first index whose byte prefix sum reaches k/world of the total (float64 arithmetic, identical to
 * 3fs_amd/shard.py::partition).  cuts[world + 1] receives the range bounds.  A device-resident payload is
 * read where it lives: a descriptor whose memory belongs to another listed device than its range's worker
 * goes to the least-loaded worker on that device; memory on a device the object does not drive fails the
 * call with H3C_ERR_INVALID_ARG before any work.  Place shard k of a resident chunk set on devices[k]
 * (h3c_multi_partition over the chunk lengths) and every descriptor stays in its range. */
typedef struct h3c_multi h3c_multi;
int h3c_multi_partition(const uint64_t *lengths, size_t n, int world, uint64_t *cuts);
/* hostfed_window: bytes per H2D staging window of each worker's pipeline (0: 64 MiB). */
int h3c_multi_create(const int *devices, int ndev, uint64_t hostfed_window, h3c_multi **out);
void h3c_multi_destroy(h3c_multi *m);
int h3c_multi_workers(const h3c_multi *m);
/* h3c_batch_create / h3c_batch_verify semantics per descriptor (ChecksumInfo::create, Common.h:146-177;
 * ChunkReplica.cc:193-207, BatchReadJob.cc:43-54).  Pinned host payloads (8 MiB or more per worker, one
 * polynomial) stream through the worker's double-buffered pipeline (h3c_hostfed_run); the rest through
 * h3c_batch_* on the worker's stream. */
int h3c_multi_batch_create(h3c_multi *m, const h3c_desc *d, size_t n, uint8_t *out_type, uint32_t *out_raw);
int h3c_multi_verify(h3c_multi *m, const h3c_desc *d, size_t n, const uint32_t *expected_raw, uint32_t *out_raw,
                     uint8_t *ok, uint64_t *n_mismatch);
/* h3c_update_ios_ex over several devices: chunks split byte-balanced by chunk_size (then moved to the worker
 * on the device holding their bytes), every op to its chunk's worker in sequence order, so each op's result
 * and each chunk's final state equal one h3c_update_ios_ex call over the whole batch.  An op naming no chunk
 * of the table fails with kInvalidArg as there; a WRITE whose payload lives on another device than its chunk
 * fails the call with H3C_ERR_INVALID_ARG before any work.  counters: the sum over workers. */
int h3c_multi_update_ios(h3c_multi *m, uint8_t poly_type, h3c_chunk_state *chunks, uint32_t nchunks,
                         const h3c_update_io *ios, uint32_t n, h3c_update_result *results, uint32_t flags,
                         h3c_update_counters *counters);
/* A resident chunk set verified repeatedly (scrub / resync): each worker keeps an h3c_plan of its share and
 * its result buffers; a run moves only the expected values and the results across PCIe. */
typedef struct h3c_multi_plan h3c_multi_plan;
int h3c_multi_plan_create(h3c_multi *m, const h3c_desc *d, size_t n, h3c_multi_plan **out);
int h3c_multi_plan_verify(h3c_multi_plan *p, const uint32_t *expected_raw, uint32_t *out_raw, uint8_t *ok,
                          uint64_t *n_mismatch);
void h3c_multi_plan_destroy(h3c_multi_plan *p);
/* The last call's share per worker (arrays of h3c_multi_workers entries, any may be NULL): descriptors or
 * ops, algorithmic bytes, and the worker's wall time in ms. */
int h3c_multi_last_stats(const h3c_multi *m, uint64_t *units, uint64_t *bytes, double *ms);

/* ---- utilities for benches/tests (not on the reference path) ---- */

/* chunk i at base + i*stride gets u64 words splitmix64(seed ^ ((first_chunk+i)<<40) ^ k). */
int h3c_fill_splitmix(void *base_dev, uint64_t chunk_len, uint64_t nchunks, uint64_t stride, uint64_t seed,
                      uint64_t first_chunk, void *stream);

/* Benchmark driver for the synchronous surface: `threads` host threads each call
 * h3c_batch_verify (api 0) or h3c_batch_create (api 1) `calls` times on their own `bytes`-byte
 * pinned host buffer (one descriptor per call, the default stream); lat_us[t * calls + k]
 * receives each call's latency in microseconds, *wall_s the span of the timed calls. */
int h3c_diag_sync_bench(int threads, uint64_t bytes, int calls, int api, double *lat_us, double *wall_s);

/* When enabled, the engine brackets its hot launches with HIP events on the
 * launch stream.  h3c_profile_read(kind) synchronises those events and returns the
 * summed time, launch count and algorithmic bytes of that kind. */
enum h3c_prof_kind {
  H3C_PROF_SEG = 0,     /* seg_crc_kernel: payload bytes read */
  H3C_PROF_UPDATE = 1,  /* upd_delta_kernel: 3 x block bytes per block write */
  H3C_PROF_HOSTFED = 2, /* whole host-fed pipeline (H2D + CRC): payload bytes */
  H3C_PROF_UPDIO = 3    /* h3c_update_ios's block kernel: 12 KiB per fragment (block in + out + new) */
};
void h3c_profile_enable(int on);
int h3c_profile_read(int kind, double *ms, uint64_t *launches, uint64_t *bytes, int reset);

/* Test hooks: force internal paths so tests can cover each one.  The environment variables
 * of the same names set the initial values once, when the library loads; no entry point reads
 * the environment per call.  value 0 restores the default. */
enum h3c_hook {
  H3C_HOOK_SEG_BYTES = 1,   /* segment size of the create / verify kernels (multiple of 1 KiB) */
  H3C_HOOK_DEBUG_FLAGS = 2, /* bit0: no pipelined row loop; bit1: no small-chunk kernel; bit2: no uniform kernel */
  H3C_HOOK_UPD_SCAN = 3,    /* h3c_update_blocks: 1 fused, 2 dense tiles, 3 sort + scan_by_key */
  H3C_HOOK_UPD_GRAPHS = 4,  /* h3c_update_ios: 1 never replays its pipeline as HIP graphs, even with
                               H3C_UPD_GRAPHS; 2 captures them without the flag; 3 as 2, with the first
                               device lease left out of the pointer audit's buffers (every capture is refused:
                               the audit's refusal path, for tests) */
  H3C_HOOK_UPD_LOOKBACK = 5, /* h3c_update_blocks fused path: 1 makes the workgroup with ticket 1 give up
                               its look-back at once, as a starved wait would (the void-batch report:
                               *n_invalid = UINT32_MAX, counters.invalid = UINT64_MAX) */
  H3C_HOOK_UPD_FRONT = 6,    /* h3c_update_ios, bit mask: 1 runs the sizes / cases / fragments as the
                               scan-based stage (~10 launches) instead of the one-pass front kernel; 2 runs
                               phase B (t / s scans, results) as 5 launches instead of one */
  H3C_HOOK_UPD_FAST = 7,     /* h3c_update_ios: 1 never tries the fast branch (every batch takes the general
                               pipeline); 2 tries it first on every batch, whatever the last outcome of the
                               batch shape was (default 0: tried first unless this thread's last batch of the
                               same shape and tables did not qualify) */
  H3C_HOOK_UPD_GIVEUP = 8,   /* h3c_update_ios, bit mask: a starved wait forced (spin limit 0) in the tile or
                               workgroup with ticket 1 of -- 1: uio_front_kernel (the pass is void and redone on
                               the scan-based stage), 2: uio_phaseb_kernel (phase B rerun the scan-based way),
                               4: uio_fast_kernel's look-back (results recomputed by the recovery kernel),
                               8: the aligned sub-branch's look-back in its workgroup with ticket 1 (the pass is void:
                               uio_afix_kernel recomputes the results) */
  H3C_HOOK_FAST_POLL_US = 9, /* h3c_update_ios fast branch: the most microseconds the calling thread spins on the
                               batch's outcome word before a blocking wait (0: adaptive, twice the last batch of
                               the same shape + 50 us, within [100, 2000]) */
  H3C_HOOK_UPD_ALIGNED = 10  /* h3c_update_ios: 1 never tries the aligned sub-branch of the fast branch (full
                               block-aligned 4 KiB WRITEs in two launches); 2 tries it first on every batch that
                               may take the fast branch (default 0: unless this thread's last batch of the same
                               shape and tables had an op it does not take) */
};
int h3c_test_hook(int key, uint64_t value);
/* Engine-internal counters (process-wide, monotonic) for tests and benches:
 *   0 h3c_update_ios pipeline graph replays, 1 graph captures, 2 capture failures,
 *   3 general-pipeline batches redone because a front tile gave up waiting (a void pass),
 *   4 phase B reruns because a phase-B tile gave up waiting,
 *   5 batches redone because a speculative A6 check failed (non-fold payloads),
 *   6 batches redone because the fragment count exceeded its guess,
 *   7 batches run by the fast branch (uio_fast_kernel),
 *   8 fast-branch attempts abandoned because an op did not qualify (the general pipeline ran),
 *   9 fast-branch batches whose results were recomputed after a workgroup gave up waiting,
 *   10 captured graphs refused by the topology check (a memset / memcpy node, or a kernel node not
 *      ordered after the graph's root) and run as plain launches instead,
 *   11 captured graphs refused by the pointer audit (a kernel argument pointing outside every buffer
 *      the graph cache's key names, or a kernel with no registered argument layout) and run as plain
 *      launches instead,
 *   12 batches run by the fast branch's aligned sub-branch (uio_afused_kernel; also counted in 7),
 *   13 aligned attempts abandoned because an op was not a full block-aligned 4 KiB typed WRITE (the
 *      chain-based fast branch or the general pipeline ran),
 *   14 aligned passes whose results were recomputed by uio_afix_kernel (an A6 failure, a block whose last
 *      write failed its check, or a look-back that gave up). */
uint64_t h3c_diag_counter(int which);
/* The shape of the last graph this thread captured for h3c_update_ios (tests): out7 = {nodes, root
 * nodes, memset + memcpy nodes, kernel nodes, nodes reachable from the first root, edges, the largest
 * out-degree}.  A graph is instantiated only when it is one chain of kernel nodes (one root, every
 * node reachable, no memset / memcpy node); else the shape runs as plain launches (counter 10). */
int h3c_diag_last_graph(uint64_t *out7);
/* The pointer audit of the last graph this thread captured for h3c_update_ios (tests): out4 = {kernel
 * nodes audited, pointer arguments checked, pointers outside the key's buffers, kernel nodes whose
 * arguments could not be read}.  A graph is instantiated only when the last two are 0. */
int h3c_diag_last_graph_audit(uint64_t *out4);
/* Host-time trace of this thread's h3c_update_ios_dev calls (bench diagnostics): out6 = summed nanoseconds of
 * {the previous call's return to this call's entry, entry to the first kernel launch, the launches, the last
 * launch to the outcome word seen, the outcome to the return} and the number of calls; reset != 0 clears. */
int h3c_diag_host_trace(uint64_t *out6, int reset);

#ifdef __cplusplus
}
#endif
#endif /* H3C_CRC_H */
