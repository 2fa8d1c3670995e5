/* oracle/oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ForSt's block-checksum hot path (the parity oracle and the
 * "port" CPU baseline).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  The product path (forst_amd/) never
 * links it and has no CPU fallback.
 *
 * Every function cites the reference file:line whose behaviour it restates
 * (paths relative to the ForSt tree, RocksDB 8.10.0 fork).
 */
#ifndef FORST_ORACLE_H
#define FORST_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* include/rocksdb/table.h:54-60 */
enum { OR_kNoChecksum = 0, OR_kCRC32c = 1, OR_kxxHash = 2, OR_kxxHash64 = 3,
       OR_kXXH3 = 4 };

/* ---- CRC32C (util/crc32c.h, util/crc32c.cc) ---- */
uint32_t oracle_crc32c_extend(uint32_t crc, const void* p, size_t n);   /* portable slicing-by-8 */
uint32_t oracle_crc32c_extend_fast(uint32_t crc, const void* p, size_t n); /* SSE4.2 3-way */
uint32_t oracle_crc32c_value(const void* p, size_t n);
uint32_t oracle_crc32c_combine(uint32_t crc1, uint32_t crc2, size_t len2);
uint32_t oracle_crc32c_mask(uint32_t crc);
uint32_t oracle_crc32c_unmask(uint32_t masked);
/* x^(8*nbytes) shift of a raw CRC state (GF(2)); used to derive GPU tables. */
uint32_t oracle_crc32c_shift(uint32_t state, uint64_t nbytes);

/* ---- xxHash v0.8.1 (util/xxhash.h) ---- */
uint64_t oracle_xxh3_64(const void* p, size_t n);
uint32_t oracle_xxh32(const void* p, size_t n, uint32_t seed);
uint64_t oracle_xxh64(const void* p, size_t n, uint64_t seed);

/* ---- XXPH3 (xxHash 0.7.2 preview, util/xxph3.h): Hash64 / NPHash64 ---- */
uint64_t oracle_hash64(const void* p, size_t n, uint64_t seed); /* util/hash.cc:81 */
/* db/kv_checksum.h ProtectionInfo64: ProtectKV (op_type < 0) / ProtectKVO,
 * then ProtectS if has_seq, ProtectC if has_cf */
uint64_t oracle_kv_protect(const void* key, size_t klen, const void* value, size_t vlen,
                           int op_type, int has_seq, uint64_t seq, int has_cf, uint32_t cf);
/* ProtectionInfo<T>::Verify (kv_checksum.h:117-133); 1 if the low len bytes match */
int oracle_kv_verify(uint64_t prot, uint32_t len, const void* stored);
int oracle_memtable_verify(const uint8_t* p, size_t avail, uint32_t prot_bytes,
                           uint64_t* computed);
void oracle_memtable_verify_batch(const uint8_t* base, size_t base_len, const uint64_t* offsets,
                                  size_t n, uint32_t prot_bytes, uint64_t* computed,
                                  uint8_t* status);
/* batch forms matching forst_hash64_batch / forst_kv_{protect,verify}_batch */
void oracle_hash64_batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint64_t* seeds, uint64_t seed, uint64_t* out, size_t n);
void oracle_kv_protect_batch(const uint8_t* base, const uint64_t* key_offsets,
                             const uint32_t* key_sizes, const uint64_t* value_offsets,
                             const uint32_t* value_sizes, const uint8_t* op_types,
                             const uint64_t* seqnos, const uint32_t* cf_ids, uint64_t* out,
                             size_t n);

/* ---- block checksum dispatcher (table/format.cc, table/format.h) ---- */
uint32_t oracle_compute_builtin_checksum(int type, const void* p, size_t n);
uint32_t oracle_compute_builtin_checksum_with_last_byte(int type, const void* p,
                                                        size_t n, uint8_t last);
uint32_t oracle_checksum_modifier_for_context(uint32_t base, uint64_t offset);
/* table/block_based/reader_common.cc:26.  Returns 1 if OK.  *computed and
 * *stored receive the values the reference would report (unmasked for CRC,
 * stored with context removed). */
int oracle_verify_block_checksum(int type, const void* data, size_t block_size,
                                 uint32_t modifier, uint32_t* computed,
                                 uint32_t* stored);

/* ---- batch forms (same layout as the C-ABI in include/forst_checksum.h) ---- */
/* compute (write side, a7 + a8): out[i] = ComputeBuiltinChecksumWithLastByte(
 *   type, base+off[i], size[i], last ? last[i] : base[off[i]+size[i]]) + mod[i] */
void oracle_block_checksum_batch(int type, const uint8_t* base,
                                 const uint64_t* offsets, const uint32_t* sizes,
                                 const uint8_t* last_bytes,
                                 const uint32_t* modifiers, uint32_t* out,
                                 size_t n, int nthreads);
/* verify (read side, a9); returns number of mismatches */
uint64_t oracle_block_verify_batch(int type, const uint8_t* base,
                                   const uint64_t* offsets,
                                   const uint32_t* sizes,
                                   const uint32_t* modifiers,
                                   uint32_t* computed, uint8_t* ok, size_t n,
                                   int nthreads);
void oracle_crc32c_batch(const uint8_t* base, const uint64_t* offsets,
                         const uint32_t* lengths, uint32_t* out, size_t n,
                         int nthreads);
void oracle_xxh3_batch(const uint8_t* base, const uint64_t* offsets,
                       const uint32_t* lengths, uint64_t* out, size_t n,
                       int nthreads);

/* XXH3_64bits of logical WAL records as log::Reader::ReadRecord computes its
 * record checksum (db/log_reader.cc:95-165): record j is the payloads of the
 * physical records [first[j], first[j+1]) (the last: up to n_phys) back to
 * back; physical record q has its hs-byte header at phys_offsets[q] and
 * phys_lengths[q] payload bytes after it. */
void oracle_wal_record_xxh3_batch(const uint8_t* log, const uint64_t* phys_offsets,
                                  const uint32_t* phys_lengths, uint64_t n_phys, uint32_t hs,
                                  const uint64_t* first, uint64_t* out, size_t n, int nthreads);

/* ---- WAL (db/log_format.h, db/log_writer.cc, db/log_reader.cc) ---- */
/* masked record CRC as EmitPhysicalRecord writes it (db/log_writer.cc:228) */
uint32_t oracle_wal_record_crc(int type, uint32_t log_number,
                               const void* payload, size_t n);
/* Frame `n` logical records into log blocks the way log::Writer::AddRecord
 * does (db/log_writer.cc:65-160, no compression).  `dst` must hold
 * oracle_wal_framed_size(...) bytes.  Returns bytes written.  Physical record
 * headers are recorded in rec_offsets/rec_lengths (may be NULL) -- offset of
 * the header and the payload length of each physical record. */
uint64_t oracle_wal_framed_size(const uint32_t* lengths, size_t n,
                                int recyclable);
uint64_t oracle_wal_frame(const uint8_t* payloads, const uint32_t* lengths,
                          size_t n, int recyclable, uint32_t log_number,
                          uint8_t* dst, uint64_t* rec_offsets,
                          uint32_t* rec_lengths, uint64_t* n_phys);
/* Verify every physical record CRC of log blocks [0, nbytes) the way
 * log::Reader::ReadPhysicalRecord checks it (db/log_reader.cc:450-531),
 * per 32 KiB log block.  Walks headers; status per physical record written
 * to ok[] in order (1 = CRC ok).  Returns number of physical records seen;
 * *bad receives the count of CRC mismatches. */
uint64_t oracle_wal_verify(const uint8_t* buf, uint64_t nbytes, uint8_t* ok,
                           uint64_t ok_cap, uint64_t* bad, int nthreads);

/* The same check per log block, with forst_wal_verify_batch's outputs:
 * status[b] (0 ok, 1 checksum mismatch, 2 bad length, 3 zero record, 4 old
 * record: a recyclable header whose log number is not log_number), nrec[b] =
 * records verified before the first failure, fail_off[b] = offset in the
 * block of the failing header or of the end of parsing. */
void oracle_wal_verify_blocks(const uint8_t* buf, uint64_t nbytes, uint32_t log_number,
                              uint8_t* status, uint32_t* nrec, uint32_t* fail_off, int nthreads);

/* ---- synthetic data ---- */
uint64_t oracle_splitmix64(uint64_t x);
/* byte i of the stream = byte (i & 7) of splitmix64(seed + (i>>3 + 1)*gamma) */
void oracle_fill_stream(uint8_t* dst, uint64_t start, uint64_t nbytes,
                        uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
