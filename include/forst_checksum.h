/* include/forst_checksum.h -- C ABI of the MI355X (gfx950) block-checksum engine.
 *
 * Drop-in device boundary for ForSt's built-in checksum hot path.  Each entry
 * point replaces a per-block (or per-record) CPU call of the reference with one
 * batched, stream-ordered GPU launch over thousands of independent blocks:
 *
 *   forst_block_checksum_batch  <- ComputeBuiltinChecksumWithLastByte +
 *                                  ChecksumModifierForContext
 *                                  (table/format.h:309, table/format.h:119),
 *                                  as called by BlockBasedTableBuilder::
 *                                  WriteMaybeCompressedBlock
 *                                  (table/block_based/block_based_table_builder.cc:1340-1345)
 *   forst_block_trailer_batch   <- the same + EncodeFixed32 of the 5-byte
 *                                  trailer [type][LE32 checksum]
 *                                  (block_based_table_builder.cc:1340-1360)
 *   forst_block_verify_batch    <- VerifyBlockChecksum
 *                                  (table/block_based/reader_common.h:33,
 *                                  reader_common.cc:26-62) as called by
 *                                  BlockFetcher::ProcessTrailerIfPresent
 *                                  (table/block_fetcher.cc:32) and the batch
 *                                  sites BlockBasedTable::VerifyChecksumInBlocks
 *                                  (block_based_table_reader.cc:2491) and
 *                                  RetrieveMultipleBlocks
 *                                  (block_based_table_reader_sync_and_async.h:225)
 *   forst_crc32c_batch          <- crc32c::Extend / crc32c::Value
 *                                  (util/crc32c.h:25, :35)
 *   forst_xxh3_64_batch         <- XXH3_64bits (util/xxhash.h:933/:5311)
 *   forst_crc32c_buffer         <- crc32c::Extend over one large buffer, as
 *                                  FileChecksumGenCrc32c::Update
 *                                  (util/file_checksum_helper.h:22) and the
 *                                  WritableFileWriter handoff CRC
 *                                  (file/writable_file_writer.cc:100-212)
 *   forst_crc32c_combine[_batch]<- crc32c::Crc32cCombine (util/crc32c.h:32,
 *                                  crc32c.cc:1279)
 *   forst_wal_verify_batch      <- log::Reader::ReadPhysicalRecord CRC check
 *                                  (db/log_reader.cc:450-531) of every 32 KiB
 *                                  log block
 *   forst_wal_record_crc_batch  <- log::Writer::EmitPhysicalRecord CRC
 *                                  (db/log_writer.cc:228-263)
 *   forst_wal_record_xxh3_batch <- log::Reader::ReadRecord record checksum
 *                                  XXH3 (db/log_reader.cc:95-165)
 *   forst_hash64_batch          <- Hash64 / NPHash64 (util/hash.cc:81-88)
 *   forst_kv_protect_batch      <- ProtectionInfo64 ProtectKV[O][S|C]
 *                                  (db/kv_checksum.h:296-460)
 *   forst_kv_verify_batch       <- ProtectionInfo<T>::Verify
 *                                  (db/kv_checksum.h:117-133)
 *   forst_memtable_verify_batch <- MemTable::VerifyEntryChecksum
 *                                  (db/memtable.cc:273-307)
 *   forst_memtable_protect_batch<- MemTable::UpdateEntryChecksum
 *                                  (db/memtable.cc:676-693)
 *
 * Conventions
 *  - All array/buffer pointers are DEVICE pointers (hipMalloc'd, or host
 *    memory registered/mapped so the GPU can read it).  The caller owns every
 *    buffer.  `stream` is a hipStream_t (NULL = default stream).  Calls are
 *    asynchronous and stream-ordered.  Scratch (work-feed counters, WAL
 *    record descriptors, chunk CRCs) comes from an engine-owned per-device
 *    memory pool with stream-ordered alloc/free and is zeroed with
 *    hipMemsetAsync.  No call copies to the host or synchronises except
 *    forst_wal_verify_batch, forst_wal_record_xxh3_batch and
 *    forst_wal_recover_batch, which read counts back (1, 2 and 4 stream
 *    synchronisations per call: record total; logical records + gathered
 *    bytes; items, tokens, emitted counts, gathered bytes), and the
 *    explicitly synchronous host-memory / SST-file / table-writer entry
 *    points below.
 *  - `base` must be 4-byte aligned; blocks live at base + offsets[i] and may
 *    start at any byte (SST blocks are packed back-to-back with 5-byte
 *    trailers, so starts are unaligned).  base_len bounds every access: a
 *    descriptor that reaches past base_len is reported as a failure
 *    (ok[i] = 0, counted in *mismatches) instead of being read.
 *  - Per-block checksum mismatch is data, not an error.  Return values are
 *    FORST_OK or a negative FORST_E* code for invalid arguments / HIP errors.
 *  - Thread safety: every entry point is reentrant; concurrent calls on
 *    different streams are independent.  Shared state: the immutable
 *    per-device table cache set up by forst_init_device() and the per-device
 *    stream-ordered scratch pool (hipMemPool, thread-safe); error messages
 *    are thread-local.
 */
#ifndef FORST_CHECKSUM_H_
#define FORST_CHECKSUM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ChecksumType values -- include/rocksdb/table.h:54-60 (on-disk footer byte). */
enum forst_checksum_type {
  FORST_kNoChecksum = 0,
  FORST_kCRC32c = 1,
  FORST_kxxHash = 2,
  FORST_kxxHash64 = 3,
  FORST_kXXH3 = 4
};

/* return codes */
#define FORST_OK 0
#define FORST_EINVAL (-1)        /* bad pointer / size / alignment */
#define FORST_EUNSUPPORTED (-2)  /* reserved: ChecksumType not handled (all 5 are) */
#define FORST_EHIP (-3)          /* HIP runtime error (see forst_last_error) */
#define FORST_ENODEV (-4)        /* no gfx950 device / code object not loadable */
#define FORST_ECORRUPT (-5)      /* corrupt file structure (SST footer / block format);
                                    message in forst_sst_last_error() */

/* WAL per-log-block status (forst_wal_verify_batch) -- mirrors the reader's
 * outcomes of ReadPhysicalRecord (db/log_reader.h kBadRecord*, kEof). */
#define FORST_WAL_OK 0           /* all records good up to padding / block end */
#define FORST_WAL_BAD_CHECKSUM 1 /* kBadRecordChecksum: rest of block dropped */
#define FORST_WAL_BAD_LENGTH 2   /* kBadRecordLen: header+length past block end */
#define FORST_WAL_ZERO_RECORD 3  /* kZeroType && length==0 (preallocated space) */
#define FORST_WAL_OLD_RECORD 4   /* recyclable header with another log number */

/* Library / device management. */
const char* forst_version(void);
const char* forst_last_error(void); /* thread-local message of the last failure */
/* Optional eager init of the current device (loads code object, caches the
 * CU count).  Every entry point does this lazily; call it up front to keep
 * first-call latency out of a timed region. */
int forst_init_device(void);

/* Write side (a7 + a8): out[i] = ComputeBuiltinChecksumWithLastByte(type,
 *   base+offsets[i], sizes[i], last) + modifiers[i]
 * where last = last_bytes ? last_bytes[i] : base[offsets[i] + sizes[i]] and
 * modifiers may be NULL (format_version <= 5). */
int forst_block_checksum_batch(int checksum_type, const uint8_t* base,
                               uint64_t base_len, const uint64_t* offsets,
                               const uint32_t* sizes, const uint8_t* last_bytes,
                               const uint32_t* modifiers, uint32_t* out,
                               uint64_t n_blocks, void* stream);

/* Write side with the trailer materialised in place: for every block writes
 * base[off+size] = last_bytes[i] and base[off+size+1 .. +5) = LE32(checksum)
 * (the bytes WriteMaybeCompressedBlock appends).  `out` may be NULL. */
int forst_block_trailer_batch(int checksum_type, uint8_t* base,
                              uint64_t base_len, const uint64_t* offsets,
                              const uint32_t* sizes, const uint8_t* last_bytes,
                              const uint32_t* modifiers, uint32_t* out,
                              uint64_t n_blocks, void* stream);

/* Read side (a9): for every block (serialized size sizes[i] + 5 at
 * base+offsets[i]): computed = ComputeBuiltinChecksum(type, data, size+1);
 * stored = DecodeFixed32(data+size+1) - modifiers[i]; ok = stored==computed.
 * computed / stored / ok may be NULL.  *mismatches (device counter, may be
 * NULL) is INCREMENTED by the number of failing blocks. */
int forst_block_verify_batch(int checksum_type, const uint8_t* base,
                             uint64_t base_len, const uint64_t* offsets,
                             const uint32_t* sizes, const uint32_t* modifiers,
                             uint32_t* computed, uint32_t* stored, uint8_t* ok,
                             unsigned long long* mismatches, uint64_t n_blocks,
                             void* stream);

/* out[i] = crc32c::Extend(init_crcs ? init_crcs[i] : 0, base+offsets[i],
 * lengths[i])  (unmasked, as util/crc32c.h returns it). */
int forst_crc32c_batch(const uint8_t* base, uint64_t base_len,
                       const uint64_t* offsets, const uint32_t* lengths,
                       const uint32_t* init_crcs, uint32_t* out,
                       uint64_t n_buffers, void* stream);

/* *out (device) = crc32c::Extend(init, base, len): one buffer of any size,
 * checksummed in 64 KiB chunks at streaming rate and folded with the combine
 * identity crc(A||B) = x^(8|B|) * crc(A) ^ crc(B).  init = 0 gives
 * crc32c::Value. */
int forst_crc32c_buffer(const uint8_t* base, uint64_t len, uint32_t init, uint32_t* out,
                        void* stream);

/* out[i] = crc32c::Crc32cCombine(crc1[i], crc2[i], len2[i]) (device arrays). */
int forst_crc32c_combine_batch(const uint32_t* crc1, const uint32_t* crc2,
                               const uint64_t* len2, uint32_t* out, uint64_t n, void* stream);

/* Host utility (no GPU call): crc32c::Crc32cCombine(crc1, crc2, len2), the
 * CRC of A||B from crc(A), crc(B) and |B|. */
uint32_t forst_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* out[i] = XXH3_64bits(base+offsets[i], lengths[i])  (xxHash 0.8.1, seed 0). */
int forst_xxh3_64_batch(const uint8_t* base, uint64_t base_len,
                        const uint64_t* offsets, const uint32_t* lengths,
                        uint64_t* out, uint64_t n_buffers, void* stream);

/* WAL replay (a13): log blocks [first_block, first_block + n_blocks) of the
 * log image `log` (log_len bytes; the last block may be short).  Checks
 * physical records only (ReadPhysicalRecord: header chain, length, old
 * record, zero type, CRC); fragment order and record types are the caller's
 * (or forst_wal_recover_batch's).  One entry
 * per log block: status_out (FORST_WAL_*), nrec_out = physical records whose
 * CRC verified before the first failure, fail_off_out = byte offset in the
 * block of the failing header (or of the end of parsing).  Any out may be
 * NULL.  *bad_blocks (device counter, may be NULL) += blocks with status !=
 * FORST_WAL_OK && != FORST_WAL_ZERO_RECORD. */
int forst_wal_verify_batch(const uint8_t* log, uint64_t log_len,
                           uint64_t first_block, uint64_t n_blocks,
                           uint32_t log_number, uint8_t* status_out,
                           uint32_t* nrec_out, uint32_t* fail_off_out,
                           unsigned long long* bad_blocks, void* stream);

/* WAL write side (a12): masked record CRC for physical records whose header
 * (7 or 11 bytes, type already in byte 6, log number in 7..10 when
 * recyclable) starts at log + header_offsets[i] and whose payload follows
 * it; writes the CRC into header bytes 0..3 when write_in_place != 0 and to
 * crc_out[i] when crc_out != NULL. */
int forst_wal_record_crc_batch(uint8_t* log, uint64_t log_len,
                               const uint64_t* header_offsets,
                               uint64_t n_records, int write_in_place,
                               uint32_t* crc_out, void* stream);
/* The same with the payload lengths the writer laid out (forst_wal_layout[_at]
 * rec_lengths; they must equal the headers' length fields) and the header size
 * (recyclable: 11 bytes, else 7): the CRC kernel takes its descriptors from
 * these arrays and stores the masked CRCs in place itself, so no pass reads
 * the headers first -- log::Writer::EmitPhysicalRecord knows every length it
 * emits (log_writer.cc:228-263).  Headers that do not fit in the log get
 * crc_out 0 and are not written. */
int forst_wal_record_crc_lengths(uint8_t* log, uint64_t log_len,
                                 const uint64_t* header_offsets,
                                 const uint32_t* payload_lengths, uint64_t n_records,
                                 int recyclable, int write_in_place, uint32_t* crc_out,
                                 void* stream);

/* XXH3_64bits of every logical record (log::Reader::ReadRecord record
 * checksum, db/log_reader.cc:95-165, compared by WriteBatchInternal::
 * UpdateProtectionInfo, db/write_batch.cc:3164-3181).  header_offsets = the
 * physical records in log order (e.g. from forst_wal_layout); a logical
 * record is a kFullType fragment or kFirstType + kMiddleType* + kLastType
 * (recyclable types alike), hashed as the concatenation of its payloads.
 * hashes[j] / first_phys[j] (device, capacity n_phys; first_phys nullable)
 * for j < *n_logical (host).  Synchronises the stream once.  Defined for the
 * fragment sequences log::Writer emits.  Fragment-order and record-type
 * validation (ReadRecord's "missing start of fragmented record", "unknown
 * record type" ...) is NOT done here: forst_wal_recover_batch does the whole
 * reader. */
int forst_wal_record_xxh3_batch(const uint8_t* log, uint64_t log_len,
                                const uint64_t* header_offsets, uint64_t n_phys,
                                uint64_t* hashes, uint64_t* first_phys, uint64_t* n_logical,
                                void* stream);

/* ---- Fused WAL recovery (§8f-2): log::Reader::ReadRecord over a whole log ---
 * (db/log_reader.cc:69-320, ReadPhysicalRecord :450-531, ReadMore :404-448)
 * as DBImpl::RecoverLogFiles (db/db_impl/db_impl_open.cc:1210) drives it, with
 * every record boundary found on the device: the header walk, the CRC of
 * every physical record, the fragment state machine and the XXH3_64bits
 * record checksum of every logical record (:95-165), in one call, without
 * header offsets from the host.  Output = what the reader returns, in order:
 * the logical records (Reader::LastRecordOffset, length, XXH3, fragments) and
 * the reporter's Corruption(bytes, reason) calls (reader position, bytes,
 * reason, record type for "unknown record type %u").  wal_recovery_mode =
 * WALRecoveryMode (include/rocksdb/options.h): 0 kTolerateCorruptedTailRecords,
 * 1 kAbsoluteConsistency, 2 kPointInTimeRecovery, 3 kSkipAnyCorruptedRecords
 * -- it decides which conditions are reported and whether old records end
 * reading, exactly as in ReadRecord; stopping recovery on a report is the
 * caller's (RecoverLogFiles') decision.  Output arrays are DEVICE arrays of
 * the given capacities (any member may be NULL); *result (host) has the
 * counts -- if a count exceeds its capacity, result->truncated is set and
 * only the first `capacity` entries are written.  Reader behaviour is the
 * reference's to the letter, pinned to its compiled log::Reader
 * (tests/golden/wal_reader.json.gz): type bytes >= 0x80 sign-extend
 * (log_reader.cc:469); types 12..17 with a valid CRC act as the reader's own
 * results kEof..kBadRecordChecksum (log_reader.h:173-186); the record
 * checksum of a fragmented record covers every fragment fed to the XXH3 state
 * since its last reset (:73-79, :119-124), aborted ones included;
 * kSetCompressionType and user-defined-timestamp-size records (types 9-11,
 * :167-213) are handled, except a kSetCompressionType record naming kZSTD
 * (a compressed WAL): result->unsupported, FORST_EUNSUPPORTED.  Synchronises
 * the stream (record counts; two more syncs when the log holds type 9-11
 * records, whose reports depend on reader state kept across the log). */
enum forst_wal_report_reason {
  FORST_WAL_PARTIAL_RECORD_1 = 1,   /* "partial record without end(1)" */
  FORST_WAL_PARTIAL_RECORD_2 = 2,   /* "partial record without end(2)" */
  FORST_WAL_MISSING_START_1 = 3,    /* "missing start of fragmented record(1)" */
  FORST_WAL_MISSING_START_2 = 4,    /* "missing start of fragmented record(2)" */
  FORST_WAL_ERROR_IN_MIDDLE = 5,    /* "error in middle of record" */
  FORST_WAL_CHECKSUM_MISMATCH = 6,  /* "checksum mismatch" */
  FORST_WAL_BAD_RECORD_LENGTH = 7,  /* "bad record length" */
  FORST_WAL_TRUNCATED_HEADER = 8,   /* "truncated header" */
  FORST_WAL_TRAILING_DATA = 9,      /* "error reading trailing data" */
  FORST_WAL_TRUNCATED_BODY = 10,    /* "truncated record body" */
  FORST_WAL_UNKNOWN_TYPE = 11,      /* "unknown record type %u" (type as the
                                       reader's unsigned int: 0xFF -> 4294967295) */
  FORST_WAL_MULTIPLE_COMPRESSION = 12,  /* "read multiple SetCompressionType records" */
  FORST_WAL_COMPRESSION_NOT_FIRST = 13, /* "SetCompressionType not the first record" */
  FORST_WAL_COMPRESSION_DECODE = 14,    /* "could not decode SetCompressionType record" */
  FORST_WAL_TS_INTERSPERSED = 15,   /* "user-defined timestamp size record interspersed
                                       partial record" */
  FORST_WAL_TS_DECODE = 16,         /* "could not decode user-defined timestamp size record" */
  FORST_WAL_TS_ZERO = 17,           /* "User-defined timestamp size record contains zero
                                       timestamp size." */
  FORST_WAL_TS_DUPLICATE = 18       /* "User-defined timestamp size record contains update
                                       to recorded column family." */
};
enum forst_wal_stop_reason {
  FORST_WAL_STOP_EOF = 0,              /* kEof */
  FORST_WAL_STOP_OLD_RECORD = 1,       /* kOldRecord (recycled log) */
  FORST_WAL_STOP_TRUNCATED_HEADER = 2, /* kBadHeader at EOF */
  FORST_WAL_STOP_TRUNCATED_BODY = 3,   /* kBadRecordLen at EOF */
  FORST_WAL_STOP_RECYCLED_TAIL = 4     /* corrupt tail of a recycled log, tolerated */
};
typedef struct forst_wal_records {
  uint64_t* offset;       /* Reader::LastRecordOffset of the record */
  uint64_t* length;       /* logical record bytes */
  uint64_t* hash;         /* XXH3_64bits(record) */
  uint32_t* n_fragments;  /* physical records */
} forst_wal_records;
typedef struct forst_wal_reports {
  uint64_t* offset;  /* reader position of the physical record / event */
  uint64_t* bytes;   /* bytes dropped, as passed to Reporter::Corruption */
  uint32_t* reason;  /* forst_wal_report_reason */
  uint32_t* type;    /* record type (FORST_WAL_UNKNOWN_TYPE) */
} forst_wal_reports;
typedef struct forst_wal_recover_result {
  uint64_t n_records, n_reports;
  uint64_t n_physical;   /* physical records parsed by the walk */
  uint64_t stop_offset;  /* reader position where reading ended */
  uint32_t stop_reason;  /* forst_wal_stop_reason */
  uint32_t truncated;    /* a count exceeded its capacity */
  uint32_t unsupported;  /* a kSetCompressionType record names kZSTD (FORST_EUNSUPPORTED) */
  uint32_t reserved;
} forst_wal_recover_result;
int forst_wal_recover_batch(const uint8_t* log, uint64_t log_len, uint32_t log_number,
                            int wal_recovery_mode, forst_wal_records records,
                            uint64_t record_capacity, forst_wal_reports reports,
                            uint64_t report_capacity, forst_wal_recover_result* result,
                            void* stream);

/* Host utility (no GPU call): the physical-record layout log::Writer::AddRecord
 * produces for logical records of the given lengths (db/log_writer.cc:65-160,
 * no compression): header offset, payload length and RecordType of every
 * physical record, the zero-padded block tails, and the image size.  Pass NULL
 * arrays (capacity 0) to count first.  FORST_EINVAL if a capacity is short. */
int forst_wal_layout(const uint32_t* lengths, uint64_t n_records, int recyclable,
                     uint64_t* rec_offsets, uint32_t* rec_lengths, uint8_t* rec_types,
                     uint64_t capacity, uint64_t* pad_offsets, uint32_t* pad_lengths,
                     uint64_t pad_capacity, uint64_t* n_phys, uint64_t* n_pads,
                     uint64_t* total_bytes);
/* The same from a writer that already stands at `block_offset` in its current
 * 32 KiB block (log::Writer::block_offset_, db/log_writer.h): offsets count from
 * the append position, *end_block_offset = block_offset_ after the last record
 * -- a write group framed at once, appended with one WritableFileWriter::Append.
 * forst_wal_layout == forst_wal_layout_at(..., block_offset = 0, ...). */
int forst_wal_layout_at(const uint32_t* lengths, uint64_t n_records, int recyclable,
                        uint32_t block_offset, uint64_t* rec_offsets, uint32_t* rec_lengths,
                        uint8_t* rec_types, uint64_t capacity, uint64_t* pad_offsets,
                        uint32_t* pad_lengths, uint64_t pad_capacity, uint64_t* n_phys,
                        uint64_t* n_pads, uint64_t* total_bytes, uint32_t* end_block_offset);

/* NPHash64 / Hash64 (util/hash.h:45-62, util/hash.cc:81 ->
 * XXPH3_64bits_withSeed, util/xxph3.h:1733; xxHash 0.7.2 preview):
 * out[i] = Hash64(base + offsets[i], lengths[i], seeds ? seeds[i] : seed).
 * Out-of-range buffers give 0. */
int forst_hash64_batch(const uint8_t* base, uint64_t base_len, const uint64_t* offsets,
                       const uint32_t* lengths, const uint64_t* seeds, uint64_t seed,
                       uint64_t* out, uint64_t n, void* stream);

/* Per-KV protection info (a15, db/kv_checksum.h): out[i] =
 *   ProtectionInfo64().ProtectKV(key_i, value_i)               (op_types == NULL)
 *   ProtectionInfo64().ProtectKVO(key_i, value_i, op_types[i])  (kv_checksum.h:296)
 *   [.ProtectS(seqnos[i])]  if seqnos != NULL                   (kv_checksum.h:453)
 *   [.ProtectC(cf_ids[i])]  if cf_ids != NULL                   (kv_checksum.h:420)
 * i.e. the XOR of NPHash64 of each field with its seed (kv_checksum.h:84-88).
 * key_i = base[key_offsets[i] .. + key_sizes[i]), value_i likewise.  The
 * WriteBatch / memtable / block callers (write_batch.cc:824+,
 * memtable.cc:273-307, block.h:271) Encode() the low 1/2/4/8 bytes. */
int forst_kv_protect_batch(const uint8_t* base, uint64_t base_len,
                           const uint64_t* key_offsets, const uint32_t* key_sizes,
                           const uint64_t* value_offsets, const uint32_t* value_sizes,
                           const uint8_t* op_types, const uint64_t* seqnos,
                           const uint32_t* cf_ids, uint64_t* out, uint64_t n, void* stream);

/* ProtectionInfo<T>::Verify(protection_bytes, checksum_ptr)
 * (kv_checksum.h:117-133) per entry, as MemTable::VerifyEntryChecksum
 * (memtable.cc:273-307) and the block kv checksums do it: the low
 * protection_bytes (1, 2, 4, 8) bytes of the protection value against the LE
 * bytes at base + checksum_offsets[i].  computed / ok may be NULL;
 * *mismatches (device counter, may be NULL) += failing entries (entries whose
 * fields reach past base_len fail). */
int forst_kv_verify_batch(const uint8_t* base, uint64_t base_len,
                          const uint64_t* key_offsets, const uint32_t* key_sizes,
                          const uint64_t* value_offsets, const uint32_t* value_sizes,
                          const uint8_t* op_types, const uint64_t* seqnos,
                          const uint32_t* cf_ids, uint32_t protection_bytes,
                          const uint64_t* checksum_offsets, uint64_t* computed, uint8_t* ok,
                          unsigned long long* mismatches, uint64_t n, void* stream);

/* Encoded MemTable entries (a15 at its memtable call site).  Entry i starts at
 * base + entry_offsets[i] in MemTable::Add's layout (db/memtable.cc:696-732):
 *   varint32 internal_key_len | user_key | LE64 (seq << 8 | type) |
 *   varint32 value_len | value | protection_bytes checksum
 * and is decoded on the device (klen, tag split into seq and type, vlen).
 *
 * forst_memtable_verify_batch <- MemTable::VerifyEntryChecksum
 *   (db/memtable.cc:273-307): ProtectKVO(user_key, value, type).ProtectS(seq)
 *   .Verify(protection_bytes, checksum).  status[i] (nullable) =
 *     0 OK
 *     1 "Unable to parse internal key length"
 *     2 "Memtable entry internal key length too short."
 *     3 "Unable to parse internal key value"
 *     4 "Corrupted memtable entry, per key-value checksum verification failed."
 *     5 the entry reaches past base_len (the reference would read on)
 *   computed[i] (nullable) = the 64-bit protection value (0 unless parsed);
 *   *mismatches (device counter, nullable) += entries with status != 0.
 * forst_memtable_protect_batch <- MemTable::UpdateEntryChecksum
 *   (db/memtable.cc:676-693, kv_prot_info == nullptr): the same value, written
 *   as Encode(protection_bytes) at the entry's checksum bytes when
 *   write_in_place; out / status nullable (status 0, 1, 2, 3 or 5). */
int forst_memtable_verify_batch(const uint8_t* base, uint64_t base_len,
                                const uint64_t* entry_offsets, uint64_t n,
                                uint32_t protection_bytes, uint64_t* computed, uint8_t* status,
                                unsigned long long* mismatches, void* stream);
int forst_memtable_protect_batch(uint8_t* base, uint64_t base_len, const uint64_t* entry_offsets,
                                 uint64_t n, uint32_t protection_bytes, int write_in_place,
                                 uint64_t* out, uint8_t* status, void* stream);

/* WriteBatch reps (a15 at its WriteBatch call site) <-
 * WriteBatchInternal::UpdateProtectionInfo(wb, 8) (db/write_batch.cc:3164-3181):
 * for every rep b = base[rep_offsets[b] .. + rep_sizes[b]) (e.g. the logical
 * records forst_wal_recover_batch emits), WriteBatch::Iterate's parse
 * (write_batch.cc:361-716) on the device and, per data record in order,
 * ProtectionInfoUpdater's ProtectKVO(key, value, op).ProtectC(cf)
 * (write_batch.cc:3016-3080; CF variants hash as their base op; Delete /
 * SingleDelete with an empty value).  Rep b's values land at
 * prot[first_entry[b] .. first_entry[b+1]) (first_entry: n_reps + 1 device
 * u64, from the reps' header counts); slots no record filled hold 0.
 * status[b] (nullable): 0 OK, 1 "malformed WriteBatch (too small)",
 * 2 "bad WriteBatch Put", 3 "bad WriteBatch Delete", 4 "bad WriteBatch
 * DeleteRange", 5 "bad WriteBatch Merge", 6 "bad WriteBatch BlobIndex",
 * 7 "bad WriteBatch Blob", 8 "bad EndPrepare XID", 9 "bad commit timestamp",
 * 10 "bad Commit XID", 11 "bad Rollback XID", 12 "bad WriteBatch PutEntity",
 * 13 "unknown WriteBatch tag", 14 "WriteBatch has wrong count", 15 the rep
 * reaches past base_len.  n_protected[b] (nullable) = slots filled.
 * Synchronous: *n_total (host) = first_entry[n_reps]; FORST_EINVAL when it
 * exceeds capacity (call again with capacity >= *n_total). */
int forst_write_batch_protect_batch(const uint8_t* base, uint64_t base_len,
                                    const uint64_t* rep_offsets, const uint32_t* rep_sizes,
                                    uint64_t n_reps, uint64_t* first_entry, uint64_t* prot,
                                    uint64_t capacity, uint8_t* status, uint32_t* n_protected,
                                    uint64_t* n_total, void* stream);

/* Block protection (a15 at its block-load call site) <-
 * Block::InitializeDataBlockProtectionInfo / InitializeIndexBlockProtectionInfo
 * / InitializeMetaIndexBlockProtectionInfo (table/block_based/block.cc:1113-1235,
 * option block_protection_bytes_per_key, include/rocksdb/advanced_options.h:1227):
 * for every uncompressed block b = base[block_offsets[b] .. + block_sizes[b])
 * (no trailer), its entries are decoded on the device as the block iterators
 * decode them -- restart array / data-block hash index geometry, shared /
 * non-shared key prefixes (each full key rebuilt in scratch), index values
 * delta-encoded or full -- and per entry, in order,
 * ProtectionInfo64().ProtectKV(key, value).Encode(protection_bytes) (block.h:
 * 271-274 GenerateKVChecksum) is written: block b's kv_checksum_ is
 * kv_checksums[first_key[b] * protection_bytes .. first_key[b+1] * protection_bytes)
 * (first_key: n_blocks + 1 device u64); prot (nullable, capacity u64) gets the
 * full 64-bit values.  kinds[b]: 0 data, 1 index, 2 metaindex, | 4 index values
 * not delta-encoded (value_is_full), | 8 index values carry the first key
 * (kBinarySearchWithFirstKey).  status[b] (nullable): 0 OK, 1 bad block
 * contents (the reference's size_ = 0 error marker), 2 "bad entry in block",
 * 3 the block reaches past base_len; a failing block gets no keys.
 * Synchronous: *n_total (host) = the key total; FORST_EINVAL when it exceeds
 * capacity (call again with capacity >= *n_total). */
int forst_block_kv_checksum_batch(const uint8_t* base, uint64_t base_len,
                                  const uint64_t* block_offsets, const uint32_t* block_sizes,
                                  const uint8_t* kinds, uint64_t n_blocks,
                                  uint32_t protection_bytes, uint64_t* first_key,
                                  uint8_t* kv_checksums, uint64_t* prot, uint64_t capacity,
                                  uint8_t* status, uint64_t* n_total, void* stream);

/* Bench/test utility: fill dev[0 .. n) with bytes [start, start+n) of the
 * splitmix64 stream `seed` (SURVEY.md §8d synthetic inputs). */
int forst_fill_stream(uint8_t* dev, uint64_t start, uint64_t n, uint64_t seed,
                      void* stream);

/* Kernel timing hooks for bench.py: name of the kernel launched by the last
 * call on this thread and the launch configuration used. */
const char* forst_last_kernel(void);

/* ---- Host-memory batches over the GPUs of one process ------
 * ForSt is one process (DB::VerifyChecksum, db/db_impl/db_impl.cc:6254, walks
 * every file in it); its blocks start in host memory (table builder buffers,
 * FilePrefetchBuffer, mmap'd SST pages -- env/io_posix.cc:958).  These calls
 * take HOST arrays, cut the blocks into contiguous byte-balanced ranges, one
 * per entry of devices[] (forst_partition_bytes), and give every device its
 * own host thread, HIP stream and pinned staging: the range streams through
 * two 64 MiB device windows (the copy of the next window overlaps the kernel
 * on this one) and 4-5 result bytes per block come back.  Pinned or
 * registered host memory (forst_host_register) is copied by DMA in place;
 * pageable memory goes through the thread's pinned staging.  No data moves
 * between devices.  Synchronous; errors via forst_host_last_error().  A
 * device may appear more than once (several threads/streams on one GPU). */

/* cuts[0..parts]: part p = blocks [cuts[p], cuts[p+1]), part p starting at the
 * first block whose payload-byte prefix reaches p/parts of the total. */
int forst_partition_bytes(const uint32_t* sizes, uint64_t n, uint32_t parts, uint64_t* cuts);
/* forst_block_verify_batch over host memory (host arrays; computed / stored /
 * ok / mismatches may be NULL; *mismatches = failing blocks). */
int forst_block_verify_host(int checksum_type, const uint8_t* host_base, uint64_t base_len,
                            const uint64_t* offsets, const uint32_t* sizes,
                            const uint32_t* modifiers, uint32_t* computed, uint32_t* stored,
                            uint8_t* ok, uint64_t* mismatches, uint64_t n_blocks,
                            const int* devices, int n_devices);
/* forst_block_checksum_batch over host memory (write side: the caller's
 * table writer appends the trailers, see forst_trailer_writer_*). */
int forst_block_checksum_host(int checksum_type, const uint8_t* host_base, uint64_t base_len,
                              const uint64_t* offsets, const uint32_t* sizes,
                              const uint8_t* last_bytes, const uint32_t* modifiers, uint32_t* out,
                              uint64_t n_blocks, const int* devices, int n_devices);
/* forst_wal_verify_batch over a log in host memory (the reader's file
 * buffer, or a forst_host_register'ed mmap of the log file), spread over
 * several devices: the log blocks split into equal contiguous ranges, one per
 * device, each streamed through that device's host context in 64 MiB windows
 * (db/log_reader.cc:450-531 checks every 32 KiB log block on its own,
 * log_writer.cc:86-102).  Host outputs (each may be NULL), one entry per log
 * block as forst_wal_verify_batch gives them; *bad_blocks = blocks with a
 * failing status other than FORST_WAL_ZERO_RECORD. */
int forst_wal_verify_host(const uint8_t* host_log, uint64_t log_len, uint32_t log_number,
                          uint8_t* status_out, uint32_t* nrec_out, uint32_t* fail_off_out,
                          uint64_t* bad_blocks, const int* devices, int n_devices);
/* hipHostRegister / hipHostUnregister of a host range (e.g. an mmap'd SST
 * file) so the host-memory calls read it by DMA without staging.  A batch is
 * DMA'd in place only when ONE registration (or one pinned allocation) covers
 * all of it; otherwise it is staged. */
int forst_host_register(void* p, uint64_t len);
int forst_host_unregister(void* p);
const char* forst_host_last_error(void);
/* The host-memory calls keep one context per device and caller -- worker
 * thread, HIP stream, two device windows, pinned mirrors and staging --
 * created on first use and reused by every later call (buffers only grow).
 * forst_host_context_stats reports how many contexts exist and the device /
 * pinned bytes they hold; forst_host_context_trim gives the buffers of every
 * context not in use back to the driver (*released_bytes, nullable), e.g.
 * after a burst of concurrent callers.  What a context keeps for the life of
 * the process (trim does not end them): the first copy of >= 4 MiB through it
 * starts 3 detached helper threads of its copier (host_batch.cc Copier), and
 * its WAL copy stream with its per-window copied[] events stays created; so
 * threads and streams grow with the PEAK number of concurrent contexts per
 * device, not with the number of calls.  Contexts are never freed. */
int forst_host_context_stats(uint32_t* contexts, uint64_t* device_bytes,
                             uint64_t* pinned_bytes);
int forst_host_context_trim(uint64_t* released_bytes);
/* The WAL calls (forst_wal_record_xxh3_batch, forst_wal_recover_batch) run a
 * side branch on a second stream of the caller's device, taken from a
 * per-device pool for the duration of the call: the pool never holds more
 * streams than there were such calls in flight at once, whatever the number
 * of host threads that made them.  *live = streams created and not destroyed,
 * *idle = those not in use; forst_host_context_trim destroys the idle ones. */
int forst_aux_stream_stats(uint32_t* live, uint32_t* idle);
/* BlockFetcher's decompression of one block (table/block_fetcher.cc:333-345,
 * UncompressSerializedBlock, table/format.cc:637-700), host only: the
 * structural blocks the whole-file verify decodes.  compression_type =
 * CompressionType (0 none, 1 Snappy, 2 Zlib, 3 BZip2, 4 LZ4, 5 LZ4HC, 7 ZSTD;
 * zlib is linked, Snappy is decoded here from its published block format, the
 * others are opened from the system's runtime libraries; 6 XPRESS:
 * FORST_EUNSUPPORTED).  format_version >= 2 blocks carry a varint32 size in
 * front (compress_format_version 2; Snappy keeps its own length prefix in
 * both).  FORST_ECORRUPT / FORST_EUNSUPPORTED set *err to the reference's
 * message ("Corrupted compressed block contents: Zlib", "Unsupported
 * compression method for this build: Xpress"); FORST_EINVAL if capacity is
 * short (*out_len = size). */
int forst_block_uncompress(uint8_t compression_type, uint32_t format_version,
                           const uint8_t* in, uint64_t n, uint8_t* out, uint64_t capacity,
                           uint64_t* out_len, const char** err);

/* ---- Write side of flush / compaction with deferred trailers (§8f-3) --------
 * BlockBasedTableBuilder::WriteMaybeCompressedBlock
 * (table/block_based/block_based_table_builder.cc:1311-1360) as a batched
 * writer: forst_trailer_writer_add places each block at its final offset
 * (handle returned at once), the trailers of a window of blocks are computed
 * in one GPU launch, and the finished bytes go to `sink` (WritableFileWriter::
 * Append) in file order.  `sink` returns 0 on success.  block_align = 0 or the
 * alignment for BlockBasedTableOptions::block_align padding of data blocks;
 * window_bytes = 0 for the default (32 MiB). */
typedef int (*forst_sink_fn)(void* arg, const uint8_t* data, uint64_t n);
typedef struct forst_trailer_writer forst_trailer_writer;
int forst_trailer_writer_open(int checksum_type, uint32_t base_context_checksum,
                              uint64_t start_offset, uint32_t block_align, uint64_t window_bytes,
                              forst_sink_fn sink, void* sink_arg, void* stream,
                              forst_trailer_writer** out);
int forst_trailer_writer_add(forst_trailer_writer* w, const uint8_t* block, uint64_t size,
                             uint8_t compression_type, int is_data_block,
                             uint64_t* handle_offset, uint64_t* handle_size);
int forst_trailer_writer_flush(forst_trailer_writer* w);
/* flush, then append the footer (forst_sst_footer_build at the current offset) */
int forst_trailer_writer_footer(forst_trailer_writer* w, uint32_t format_version,
                                uint64_t metaindex_offset, uint64_t metaindex_size,
                                uint64_t index_offset, uint64_t index_size);
uint64_t forst_trailer_writer_offset(const forst_trailer_writer* w);
int forst_trailer_writer_close(forst_trailer_writer* w); /* flushes, frees */
const char* forst_trailer_writer_last_error(void);

/* FooterBuilder::Build (table/format.cc:231-330) of the block-based table:
 * out (>= 53 bytes) / *out_len = 48 (fv 0) or 53.  For format_version >= 6
 * the footer checksum is computed on the GPU (synchronises `stream`); fv < 6
 * makes no GPU call. */
int forst_sst_footer_build(uint32_t format_version, int checksum_type, uint64_t footer_offset,
                           uint32_t base_context_checksum, uint64_t metaindex_offset,
                           uint64_t metaindex_size, uint64_t index_offset, uint64_t index_size,
                           uint8_t* out, uint32_t* out_len, void* stream);

/* ---- SST files (BlockBasedTable::VerifyChecksum, ----------------------------
 * table/block_based/block_based_table_reader.cc:2457-2574) ----------------- */

/* Footer::DecodeFrom (table/format.cc:355-463): every footer version of the
 * block-based table (legacy magic = format_version 0, 1..6).  For
 * format_version >= 6 the footer checksum is ComputeBuiltinChecksum(type,
 * footer_zeroed, 53) + footer_checksum_modifier and must equal
 * stored_footer_checksum (the verify entry point below checks it on the GPU). */
typedef struct forst_sst_footer {
  uint64_t table_magic_number;
  uint64_t footer_offset;
  uint64_t metaindex_offset, metaindex_size;
  uint64_t index_offset, index_size; /* 0, 0 when in the metaindex (fv >= 6) */
  uint32_t format_version;
  int32_t checksum_type;
  uint32_t base_context_checksum;
  uint32_t stored_footer_checksum;
  uint32_t footer_checksum_modifier;
  uint32_t block_trailer_size;
  uint32_t footer_len;
  uint8_t footer_zeroed[53];
  /* fv >= 6: the 8 checked reserved bytes are non-zero.  The reference
   * (format.cc:440-448) reports NotSupported("File uses a future feature not
   * supported in this version") only AFTER the footer checksum matched, so
   * this is a flag, not an error of forst_sst_footer_decode. */
  uint32_t future_feature;
} forst_sst_footer;

/* Table properties the checksum walk needs (table/meta_blocks.cc:81-140,
 * block_based_table_reader.cc:948-972). index_type: 0 kBinarySearch,
 * 1 kHashSearch, 2 kTwoLevelIndexSearch, 3 kBinarySearchWithFirstKey. */
typedef struct forst_sst_properties {
  uint32_t index_type;
  uint64_t index_value_is_delta_encoded;
  uint64_t index_key_is_user_key;
  uint64_t num_data_blocks;
  uint64_t index_partitions;
  uint64_t format_version;
  uint64_t data_size;
  /* offset of the 8-byte "rocksdb.external_sst_file.global_seqno" value
   * inside the properties block, 0 when absent (meta_blocks.cc:346-348):
   * ingestion may rewrite it after the block checksum was taken, so the
   * properties checksum is retried with it zeroed (meta_blocks.cc:401-417) */
  uint64_t global_seqno_value_offset;
} forst_sst_properties;

typedef struct forst_sst_verify_result {
  int32_t status; /* forst_gpu::Status::Code (= the reference Status::Code): 0 OK, 2 Corruption, 3 NotSupported, ... */
  uint32_t format_version;
  int32_t checksum_type;
  uint32_t index_type;
  uint64_t blocks_verified; /* block checksums computed on the GPU */
  uint64_t data_blocks, meta_blocks, index_partitions;
  uint64_t n_failed;
  char message[512]; /* Status::ToString(), the reference's Corruption text */
} forst_sst_verify_result;

/* Host utilities (no GPU call). tail = the last tail_len (<= 53) bytes of a
 * file of file_size bytes. */
int forst_sst_footer_decode(const uint8_t* tail, uint64_t tail_len, uint64_t file_size,
                            forst_sst_footer* out);
/* Block handles of an index block / index partition (IndexValue,
 * table/format.cc:105-148; value delta encoding, optional first key). */
int forst_sst_index_handles(const uint8_t* block, uint64_t block_size, int value_delta_encoded,
                            int has_first_key, uint64_t* offsets, uint64_t* sizes,
                            uint64_t capacity, uint64_t* n);
int forst_sst_properties_decode(const uint8_t* block, uint64_t block_size,
                                forst_sst_properties* out);
const char* forst_sst_last_error(void);

/* Whole-file verify: host_file = the file bytes in host memory (structure is
 * decoded there), dev_file = the same bytes in device memory (every checksum
 * -- footer, metaindex, properties, index, partitions, all meta and data
 * blocks -- is computed on the GPU).  The result carries the reference's
 * Status for the first failure in VerifyChecksum's order. Synchronous. */
int forst_sst_verify_file(const uint8_t* host_file, uint64_t file_size, const uint8_t* dev_file,
                          const char* file_name, forst_sst_verify_result* out, void* stream);

/* DB::VerifyChecksum (db/db_impl/db_impl.cc:6254 -> convenience.cc:57 per
 * file) over n_files SST files: file i is host_files[i] (file_sizes[i] bytes)
 * in host memory and dev_arena[dev_offsets[i] ..] in device memory (each
 * dev_offsets[i] 4-byte aligned, as device buffers are: a file at an
 * unaligned offset gets InvalidArgument in out[i]).  Each
 * file's structural blocks are checked as in forst_sst_verify_file; the meta
 * and data blocks of ALL files are then verified in one launch per checksum
 * type.  out[i] = exactly what forst_sst_verify_file returns for file i.
 * Synchronous. */
int forst_sst_verify_files(const uint8_t* const* host_files, const uint64_t* file_sizes,
                           const uint64_t* dev_offsets, const uint8_t* dev_arena,
                           uint64_t arena_len, const char* const* file_names, uint64_t n_files,
                           forst_sst_verify_result* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FORST_CHECKSUM_H_ */
