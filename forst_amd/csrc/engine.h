// forst_amd/csrc/engine.h -- host-side launch interface between the C ABI
// (capi.hip) and the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/forst_checksum.h"

namespace forst {

// What a block launch does with each descriptor.
enum BlockMode : int {
  kModeCompute = 0,  // out = checksum(data, size, last) + modifier
  kModeTrailer = 1,  // compute + write [last][LE32] at data+size
  kModeVerify = 2,   // computed vs stored trailer (reader_common.cc:26)
  kModeRaw = 3,      // crc32c::Extend(init, data, len) / XXH3_64bits
};

// The fragment XXH3 kernel (xxh3.hip xxh3_frag_kernel) walks a record in
// windows of 256 K bytes per 16-lane row and step: lane t holds the K
// 16-byte chunks at window offsets 16 t + 256 k.  K = FORST_FRAG_K for the
// XXH3-only kernel (a14 and the recovery's remainder) and FORST_FRAG_CRC_K
// for the fused recovery kernel, whose E / Z constants (wal_recover.hip
// rw_cand_kernel) are taken at the same window ends.  A/B on one box
// (profiles/ab_r05/frag_2k_windows_k8_C5.log): K = 8 took a14 from
// 9.66-9.83 to 9.48-9.54 ms, but the fused kernel at K = 8 needs 211 VGPRs
// (2 waves per SIMD) and the recovery went from 18.3 to 20.7 ms.
#ifndef FORST_FRAG_K
#define FORST_FRAG_K 8
#endif
#ifndef FORST_FRAG_CRC_K
#define FORST_FRAG_CRC_K 4
#endif
constexpr uint32_t kFragKA14 = FORST_FRAG_K, kFragKFused = FORST_FRAG_CRC_K;
static_assert((kFragKA14 == 4 || kFragKA14 == 8) && (kFragKFused == 4 || kFragKFused == 8),
              "4 or 8 chunks per lane");
constexpr uint32_t kFragWinFused = 256 * kFragKFused;
constexpr uint32_t kFragWinFusedShift = kFragKFused == 8 ? 11 : 10;
// The kernel loads whole windows of a long record: records whose last byte
// lies within kFragTail bytes of the log end are hashed from a gathered copy
// instead (wal_hash.h, and the fused recovery's candidates, wal_recover.hip)
constexpr uint64_t kFragTail = 256 * (kFragKA14 > kFragKFused ? kFragKA14 : kFragKFused) + 64;

struct BlockArgs {
  const uint8_t* base;
  uint8_t* base_w;          // same buffer, writable (trailer mode)
  uint64_t base_len;
  const uint64_t* offsets;
  const uint32_t* sizes;
  const uint8_t* last_bytes;   // nullable
  const uint32_t* modifiers;   // nullable
  const uint32_t* init_crcs;   // nullable (raw CRC mode)
  uint32_t* out32;             // nullable
  uint64_t* out64;             // nullable (raw XXH3 mode)
  uint32_t* stored_out;        // nullable (verify)
  uint8_t* ok_out;             // nullable (verify)
  unsigned long long* mismatches;  // nullable (verify)
  uint64_t n;
  // rows kernels' work feed (stream_common.h): a static first share of
  // share1 descriptors per wave, then 64-descriptor chunks claimed from
  // *ticket (zeroed per launch) or, without one, dealt round-robin
  unsigned long long* ticket;
  uint64_t share1;
  int kernel_hint;  // CRC: 0 by mean block size, 1 rows kernel, 2 v2 kernel; XXH3: 3 v1 kernel
  // fused WAL-recovery CRC (launch_xxh3_frag_crc): per physical record, the
  // constants (E | Z << 32) and the CRC verdict; modifiers = the record's
  // first physical record index
  const uint64_t* crc_ez;
  uint8_t* crc_ok;
  // WAL writer mode of the raw CRC rows kernel (forst_wal_record_crc_lengths):
  // wal_hs = the header size (7, or 11 recyclable) when offsets[] are header
  // offsets and sizes[] payload lengths -- each record's CRC covers
  // header[6..hs) + payload (log_writer.cc:240-263) and out32 gets it masked
  // (util/crc32c.h:33)
  uint32_t wal_hs;
  // raw CRC mode: expected values; out32[i] is written only where the CRC
  // differs (the caller pre-fills out32 with them), so a clean verify stores
  // nothing from the streaming loop (stores share vmcnt with its loads)
  const uint32_t* expect;
  // workgroup feed (stream_common.h wg_range): bytes each descriptor weighs
  // on top of its own in the byte-balanced workgroup ranges (set by the
  // launcher)
  uint32_t wg_cost;
};

struct WalArgs {
  const uint8_t* log;
  uint8_t* log_w;
  uint64_t log_len;
  uint64_t first_block;
  uint64_t n_blocks;
  uint32_t log_number;
  uint8_t* status_out;
  uint32_t* nrec_out;
  uint32_t* fail_off_out;
  unsigned long long* bad_blocks;
  // writer side
  const uint64_t* header_offsets;
  uint64_t n_records;
  int write_in_place;
  uint32_t* crc_out;
  const uint32_t* payload_lengths;  // nullable: forst_wal_record_crc_lengths
  int recyclable;
};

// Per-KV protection / Hash64 batches (kv_protect.hip).
enum KvMode : int {
  kKvHash = 0,     // out[i] = Hash64(key_i, seeds ? seeds[i] : seed)
  kKvProtect = 1,  // out[i] = ProtectionInfo64 of (key, value[, op][, seq][, cf])
  kKvVerify = 2,   // ... compared with prot_bytes LE bytes at chk_off[i]
  // encoded memtable entries (db/memtable.cc:273-307, :696-732): key_off[i] =
  // the entry; klen / tag / vlen decoded on the device
  kKvMemVerify = 3,   // MemTable::VerifyEntryChecksum -> status[i]
  kKvMemProtect = 4,  // MemTable::UpdateEntryChecksum (written in place if asked)
};

// per-entry status of the memtable modes (MemTable::VerifyEntryChecksum's
// Corruption reasons, memtable.cc:280-306)
enum KvMemStatus : uint8_t {
  kMemOk = 0,
  kMemBadKeyLength = 1,  // "Unable to parse internal key length"
  kMemKeyTooShort = 2,   // "Memtable entry internal key length too short."
  kMemBadValue = 3,      // "Unable to parse internal key value"
  kMemMismatch = 4,      // "Corrupted memtable entry, per key-value checksum ..."
  kMemOutOfRange = 5,    // the entry reaches past the buffer (no reference twin)
};

struct KvArgs {
  const uint8_t* base;
  uint64_t base_len;
  const uint64_t* key_off;  // (buffers in Hash64 mode)
  const uint32_t* key_len;
  const uint64_t* val_off;
  const uint32_t* val_len;
  const uint8_t* ops;        // nullable: ProtectKV instead of ProtectKVO
  const uint64_t* seqs;      // nullable: no ProtectS
  const uint32_t* cfs;       // nullable: no ProtectC
  const uint64_t* seeds;     // Hash64 mode, nullable
  uint64_t seed;
  const uint64_t* chk_off;   // verify
  uint32_t prot_bytes;       // verify: 1, 2, 4 or 8
  uint64_t* out;             // nullable in verify mode
  uint8_t* ok;               // verify, nullable
  unsigned long long* mismatches;  // verify, nullable
  uint64_t n;
  uint8_t* status;           // memtable modes: KvMemStatus per entry, nullable
  int write_in_place;        // kKvMemProtect: Encode(prot_bytes) at the checksum
  const uint8_t* key_base;   // nullable: keys live in this buffer instead of base
  uint64_t key_base_len;
  uint8_t* enc_out;          // kKvProtect, nullable: Encode(prot_bytes) of entry i
                             // at enc_out + i * prot_bytes (a block's kv_checksum_)
};

// Block protection (kv_sites.hip): block kinds and per-block status
enum BlkKind : uint8_t {
  kBlkData = 0,            // InitializeDataBlockProtectionInfo (block.cc:1113)
  kBlkIndex = 1,           // InitializeIndexBlockProtectionInfo (block.cc:1162)
  kBlkMeta = 2,            // InitializeMetaIndexBlockProtectionInfo (block.cc:1205)
  kBlkValueIsFull = 4,     // index: values not delta-encoded
  kBlkHasFirstKey = 8,     // index: kBinarySearchWithFirstKey values
};
enum BlkStatus : uint8_t {
  kBlkOk = 0,
  kBlkBadContents = 1,  // Block's size_ = 0 error marker / "bad block contents"
  kBlkBadEntry = 2,     // "bad entry in block" (the iterator's CorruptionError)
  kBlkOutOfRange = 3,   // the block reaches past the buffer
};
struct BlkArgs {
  const uint8_t* base;
  uint64_t base_len;
  const uint64_t* offsets;  // block b = base[offsets[b] .. + sizes[b]) (no trailer)
  const uint32_t* sizes;
  const uint8_t* kinds;     // BlkKind | flags per block
  uint64_t n;
  uint32_t prot_bytes;
  uint64_t* first_key;      // out, n + 1
  uint8_t* kv_checksums;    // out, capacity * prot_bytes bytes
  uint64_t* prot;           // out, nullable: the full values, capacity
  uint64_t capacity;
  uint8_t* status;          // out, nullable
};
hipError_t launch_block_kv_checksum(const BlkArgs& a, hipStream_t st, uint64_t* total,
                                    const char** kernel_name);

// WriteBatch reps (kv_sites.hip): per-rep status, the Corruption texts of
// ReadRecordFromWriteBatch / WriteBatch::Iterate (db/write_batch.cc:361-716)
enum WbStatus : uint8_t {
  kWbOk = 0,
  kWbTooSmall = 1,          // "malformed WriteBatch (too small)"
  kWbBadPut = 2,            // "bad WriteBatch Put"
  kWbBadDelete = 3,         // "bad WriteBatch Delete"
  kWbBadDeleteRange = 4,    // "bad WriteBatch DeleteRange"
  kWbBadMerge = 5,          // "bad WriteBatch Merge"
  kWbBadBlobIndex = 6,      // "bad WriteBatch BlobIndex"
  kWbBadBlob = 7,           // "bad WriteBatch Blob"
  kWbBadEndPrepareXid = 8,  // "bad EndPrepare XID"
  kWbBadCommitTs = 9,       // "bad commit timestamp"
  kWbBadCommitXid = 10,     // "bad Commit XID"
  kWbBadRollbackXid = 11,   // "bad Rollback XID"
  kWbBadPutEntity = 12,     // "bad WriteBatch PutEntity"
  kWbUnknownTag = 13,       // "unknown WriteBatch tag"
  kWbWrongCount = 14,       // "WriteBatch has wrong count"
  kWbOutOfRange = 15,       // the rep reaches past the buffer (no reference twin)
};

struct WbArgs {
  const uint8_t* base;
  uint64_t base_len;
  const uint64_t* offsets;  // rep b = base[offsets[b] .. + sizes[b])
  const uint32_t* sizes;
  uint64_t n;
  uint64_t* first_entry;    // out, n + 1: rep b's protections at [first[b], first[b+1])
  uint64_t* prot;           // out, capacity
  uint64_t capacity;
  uint8_t* status;          // out, nullable: WbStatus per rep
  uint32_t* n_protected;    // out, nullable: slots filled per rep
};
// synchronous (reads the protection total back into *total); fails with
// hipErrorInvalidValue when *total > a.capacity
hipError_t launch_write_batch_protect(const WbArgs& a, hipStream_t st, uint64_t* total,
                                      const char** kernel_name);

struct DeviceInfo {
  int device;
  int num_cus;
  bool ok;
};
const DeviceInfo& device_info();  // current device (lazily initialised)

#ifdef FORST_DIAG
// Diagnostics build only (make diag -> lib/libforst_checksum_diag.so): kernel
// variants for A/B runs (tools/ab_bench.py) are selected by environment
// variables read here.  The product library compiles none of the variants and
// reads no environment variable.  Returns "" when unset.
const char* diag_env(const char* name);
#endif

// stream-ordered scratch from a per-device pool that keeps freed memory
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t stream);
hipError_t scratch_free(void* p, hipStream_t stream);
// A second stream with fork / join events on the device of a caller's stream
// (the WAL calls run a side branch on it beside their main kernel).  Taken
// from a per-device pool and given back before the call returns, so the pool
// holds at most as many as there were calls in flight at once; idle ones are
// destroyed by aux_pool_trim (forst_host_context_trim).  nullptr: none could
// be made (the caller then runs everything on its own stream).
struct AuxStream {
  hipStream_t s;
  hipEvent_t fork, join;
  int device;
};
AuxStream* aux_acquire(hipStream_t caller);
void aux_release(AuxStream* a);
void aux_pool_trim();
void aux_pool_stats(uint32_t* live, uint32_t* idle);
// work feed of a rows-kernel launch over nw waves (stream_common.h): sets
// share1 and a zeroed ticket counter that the caller releases with
// scratch_free(a.ticket) after the launch (diagnostics build:
// FORST_FEED=static|rr for the A/B references without a counter)
hipError_t feed_setup(BlockArgs& a, uint64_t nw, hipStream_t stream);

// Launchers (return hipError_t). `kernel_name` receives a static string.
hipError_t launch_crc32c_blocks(int mode, const BlockArgs& a,
                                hipStream_t stream, const char** kernel_name);
hipError_t launch_xxh3_blocks(int mode, const BlockArgs& a,
                              hipStream_t stream, const char** kernel_name);
// XXH3_64bits of WAL logical records read in place across their fragments
// (xxh3.hip xxh3_frag_kernel): offsets = first payload byte, sizes = record
// length, init_crcs = frag_info (hs | j_last << 8); needs base_len >= 4096
hipError_t launch_xxh3_frag(const BlockArgs& a, hipStream_t stream, const char** kernel_name);
// the fragment kernel with every physical record's CRC32C checked from the
// same loads (wal_recover.hip): long records (> 240 B) only
hipError_t launch_xxh3_frag_crc(const BlockArgs& a, hipStream_t stream, const char** kernel_name);
// WAL recovery's short candidates (one fragment, <= 240 B) off the fused
// kernel: their CRC and XXH3 in one pass, a record per 16-lane row
// (launch_wal_short_rows; FORST_REC_SHORT_ROWS=0: launch_crc32c_raw_lanes +
// launch_xxh3_short_rows), ahead of the fused kernel, which is then built
// for records > 240 B only (1); or in the fused kernel's rows (0)
#ifndef FORST_REC_SHORT
#define FORST_REC_SHORT 1
#endif
// ... and the Full records of one fused window (<= kFragWinFused bytes) in a
// fused-kernel launch of their own, ahead of the long records (1): measured
// and not kept (C5 recovery 17.38 -> 17.61 ms, the two launches' fused time
// 13.74 -> 13.80 ms: profiles/ab_r05/recovery_short_candidates.log)
// ... their CRC and XXH3 in one pass over the short list, on 16-lane rows
// (launch_wal_short_rows: 1), or the lane CRC kernel and the XXH3 rows
// kernel apart (0)
#ifndef FORST_REC_SHORT_ROWS
#define FORST_REC_SHORT_ROWS 1
#endif
#ifndef FORST_REC_MED
#define FORST_REC_MED 0
#endif
// XXH3_64bits of inputs of at most 240 bytes, one per 16-lane row: for
// k < n, out[idx ? idx[k] : k] = XXH3(base + off[k], len[k]); a longer or
// out-of-range input gives 0
hipError_t launch_xxh3_short_rows(const uint8_t* base, uint64_t base_len, const uint64_t* off,
                                  const uint32_t* len, uint64_t n, const uint64_t* idx,
                                  uint64_t* out, hipStream_t stream);
// WAL recovery's short candidates, one per 16-lane row: for k < n,
// crc_ok[item[k]] = (crc32c::Value(base + coff[k], clen[k]) ==
// stored[item[k]]) and hash_out[item[k]] = XXH3(base + p0[k], plen[k])
// (clen <= 252, plen <= 240)
hipError_t launch_wal_short_rows(const uint8_t* base, uint64_t base_len, const uint64_t* coff,
                                 const uint32_t* clen, const uint64_t* p0, const uint32_t* plen,
                                 const uint64_t* item, uint64_t n, const uint32_t* stored,
                                 uint8_t* crc_ok, uint64_t* hash_out, hipStream_t stream);
// raw CRC32C (crc32c::Value) of messages all under 256 bytes, one per lane
// (crc32c.hip crc32c_raw_lane_kernel): offsets / sizes / out32 as in raw mode
hipError_t launch_crc32c_raw_lanes(const BlockArgs& a, hipStream_t stream);
hipError_t launch_noop_blocks(int mode, const BlockArgs& a,
                              hipStream_t stream, const char** kernel_name);
// kxxHash (x64 = false, XXH32) / kxxHash64 (x64 = true, Lower32 of XXH64)
hipError_t launch_xxhash_legacy_blocks(bool x64, int mode, const BlockArgs& a,
                                       hipStream_t stream, const char** kernel_name);
hipError_t launch_wal_verify(const WalArgs& a, hipStream_t stream,
                             const char** kernel_name);
hipError_t launch_wal_record_crc(const WalArgs& a, hipStream_t stream,
                                 const char** kernel_name);
hipError_t launch_crc32c_combine_batch(const uint32_t* crc1, const uint32_t* crc2,
                                       const uint64_t* len2, uint32_t* out, uint64_t n,
                                       hipStream_t stream, const char** kernel_name);
hipError_t launch_crc32c_buffer(const uint8_t* base, uint64_t len, uint32_t init, uint32_t* out,
                                hipStream_t stream, const char** kernel_name);
hipError_t launch_wal_record_xxh3(const WalArgs& a, uint64_t* out, uint64_t* out_first,
                                  uint64_t* n_logical_host, hipStream_t stream,
                                  const char** kernel_name);
hipError_t launch_wal_recover(const uint8_t* log, uint64_t log_len, uint32_t log_number, int mode,
                              forst_wal_records recs, uint64_t rec_cap, forst_wal_reports reps,
                              uint64_t rep_cap, forst_wal_recover_result* res, hipStream_t st,
                              const char** name);
hipError_t launch_kv(int mode, const KvArgs& a, hipStream_t stream, const char** kernel_name);
hipError_t launch_fill_stream(uint8_t* dev, uint64_t start, uint64_t n,
                              uint64_t seed, hipStream_t stream);

}  // namespace forst
