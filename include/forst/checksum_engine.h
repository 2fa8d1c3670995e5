// include/forst/checksum_engine.h -- C++ host shim over the C ABI, in the
// reference's vocabulary (ChecksumType, Status with the reference's codes and
// message texts), so a ForSt call site can switch from the per-block CPU
// functions to batched GPU launches.  Its types live in namespace forst_gpu,
// NOT forstdb: the header compiles inside a ForSt translation unit next to
// include/rocksdb/table.h, status.h, table/format.h and util/crc32c.h, and
// forst/forstdb_adapter.h converts forst_gpu::Status / ChecksumType to and
// from ROCKSDB_NAMESPACE's there:
//
//   reference (per block, CPU)                      this shim (per batch, GPU)
//   ComputeBuiltinChecksumWithLastByte + modifier   BlockChecksumEngine::ComputeChecksums
//     (table/format.cc:594, format.h:119)
//   WriteMaybeCompressedBlock trailer               BlockChecksumEngine::WriteTrailers
//     (block_based_table_builder.cc:1340-1360)
//   VerifyBlockChecksum (reader_common.cc:26)       BlockChecksumEngine::VerifyBlocks
//   crc32c::Mask/Unmask (util/crc32c.h:44-53),      forst_gpu::crc32c::Mask/Unmask,
//   ChecksumModifierForContext (format.h:119)       forst_gpu::ChecksumModifierForContext
//     (the shim's own copies for code outside ForSt; ForSt call sites keep
//     the reference's)
//
// Statistics hooks mirror BLOCK_CHECKSUM_COMPUTE_COUNT / _MISMATCH_COUNT
// (include/rocksdb/statistics.h:440,444).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../forst_checksum.h"

namespace forst_gpu {

// include/rocksdb/table.h:54-60
enum ChecksumType : char {
  kNoChecksum = 0x0,
  kCRC32c = 0x1,
  kxxHash = 0x2,
  kxxHash64 = 0x3,
  kXXH3 = 0x4,
};

// Minimal Status with the reference's code names and ToString() format
// ("Corruption: <msg>", include/rocksdb/status.h / util/status.cc).
class Status {
 public:
  enum Code { kOk = 0, kCorruption = 2, kNotSupported = 3, kInvalidArgument = 4,
              kIOError = 5 };
  Status() : code_(kOk) {}
  static Status OK() { return Status(); }
  static Status Corruption(const std::string& m) { return Status(kCorruption, m); }
  static Status NotSupported(const std::string& m) { return Status(kNotSupported, m); }
  static Status InvalidArgument(const std::string& m) { return Status(kInvalidArgument, m); }
  static Status IOError(const std::string& m) { return Status(kIOError, m); }
  bool ok() const { return code_ == kOk; }
  bool IsCorruption() const { return code_ == kCorruption; }
  Code code() const { return code_; }
  const std::string& message() const { return msg_; }
  std::string ToString() const;

 private:
  Status(Code c, std::string m) : code_(c), msg_(std::move(m)) {}
  Code code_;
  std::string msg_;
};

namespace crc32c {
inline uint32_t Mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8ul; }
inline uint32_t Unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8ul;
  return (rot >> 17) | (rot << 15);
}
// util/crc32c.h:32 (host GF(2) arithmetic in the engine library)
inline uint32_t Crc32cCombine(uint32_t crc1, uint32_t crc2, size_t crc2len) {
  return forst_crc32c_combine(crc1, crc2, crc2len);
}
}  // namespace crc32c

// table/format.h:119
inline uint32_t ChecksumModifierForContext(uint32_t base_context_checksum, uint64_t offset) {
  uint32_t all_or_nothing = uint32_t{0} - (base_context_checksum != 0);
  uint32_t modifier =
      base_context_checksum ^ (static_cast<uint32_t>(offset) + static_cast<uint32_t>(offset >> 32));
  return modifier & all_or_nothing;
}

// options/options_helper.h:34 IsSupportedChecksumType
inline bool IsSupportedChecksumType(ChecksumType t) { return t >= kNoChecksum && t <= kXXH3; }
// ... and what the GPU engine implements today
bool GpuSupportsChecksumType(ChecksumType t);

// reader_common.cc:55-60 message, CRC values unmasked by the caller.
std::string BlockChecksumMismatchMessage(ChecksumType type, uint32_t stored, uint32_t computed,
                                         bool context_removed, const std::string& file_name,
                                         uint64_t offset, uint64_t block_size);

struct ChecksumStats {
  uint64_t block_checksum_compute_count = 0;   // BLOCK_CHECKSUM_COMPUTE_COUNT
  uint64_t block_checksum_mismatch_count = 0;  // BLOCK_CHECKSUM_MISMATCH_COUNT
  // PerfContext::block_checksum_time (include/rocksdb/perf_context.h:97):
  // nanoseconds spent verifying block checksums -- the reference times each
  // VerifyBlockChecksum call (PERF_TIMER_GUARD, reader_common.cc:29); here
  // the wall time of each VerifyBlocks batch (launch + wait for its result)
  uint64_t block_checksum_time = 0;
};

// A batch of blocks resident in device memory.  Block i occupies
// base[offsets[i] .. offsets[i] + sizes[i] + 5) (payload, type byte, LE32).
struct DeviceBlockBatch {
  const uint8_t* base = nullptr;      // device
  uint64_t base_len = 0;
  const uint64_t* offsets = nullptr;  // device
  const uint32_t* sizes = nullptr;    // device
  uint64_t n = 0;
};

class BlockChecksumEngine {
 public:
  explicit BlockChecksumEngine(void* hip_stream = nullptr) : stream_(hip_stream) {}
  ~BlockChecksumEngine();
  BlockChecksumEngine(const BlockChecksumEngine&) = delete;
  BlockChecksumEngine& operator=(const BlockChecksumEngine&) = delete;

  // Write side.  last_bytes / modifiers are device arrays (modifiers may be
  // null for format_version <= 5).  out is a device array of n.
  Status ComputeChecksums(ChecksumType type, const DeviceBlockBatch& b, const uint8_t* last_bytes,
                          const uint32_t* modifiers, uint32_t* out);
  Status WriteTrailers(ChecksumType type, const DeviceBlockBatch& b, const uint8_t* last_bytes,
                       const uint32_t* modifiers, uint32_t* out);

  // Read side: VerifyBlockChecksum over the batch.  file_offsets/modifiers
  // describe each block's position in `file_name` (host arrays, used for the
  // context modifier and the error message).  Synchronises the stream.
  // Returns OK, or the exact Corruption status the reference returns for the
  // FIRST failing block; every failing index is appended to *failed.
  Status VerifyBlocks(ChecksumType type, uint32_t base_context_checksum, const DeviceBlockBatch& b,
                      const std::string& file_name, const std::vector<uint64_t>& file_offsets,
                      std::vector<uint64_t>* failed = nullptr);

  const ChecksumStats& stats() const { return stats_; }
  void* stream() const { return stream_; }

 private:
  Status EnsureScratch(uint64_t n);
  void* stream_;
  ChecksumStats stats_;
  // device scratch for verify
  uint32_t* d_computed_ = nullptr;
  uint32_t* d_stored_ = nullptr;
  uint8_t* d_ok_ = nullptr;
  uint32_t* d_mod_ = nullptr;
  unsigned long long* d_bad_ = nullptr;
  uint64_t cap_ = 0;
};

// BlockBasedTable::VerifyChecksum (block_based_table_reader.cc:2457) for one
// SST file: host_file (host memory) is decoded on the host, dev_file (the
// same bytes in device memory) supplies every checksum computed on the GPU.
struct SstVerifyReport {
  uint32_t format_version = 0;
  int checksum_type = 0;
  uint32_t index_type = 0;
  uint64_t blocks_verified = 0;
  uint64_t data_blocks = 0, meta_blocks = 0, index_partitions = 0;
  std::vector<uint64_t> failed;  // indexes into [meta blocks..., data blocks...]
};
Status VerifySstFileChecksums(BlockChecksumEngine& engine, const uint8_t* host_file,
                              uint64_t file_size, const uint8_t* dev_file,
                              const std::string& file_name, SstVerifyReport* report = nullptr);

// DB::VerifyChecksum over many SST files staged in one device arena (file i
// at dev_arena + dev_offset): structural blocks per file, then the meta and
// data blocks of every file in one batch launch per checksum type.  Returns
// one Status per file (the same Status VerifySstFileChecksums returns).
struct SstFileRef {
  const uint8_t* host_file = nullptr;
  uint64_t file_size = 0;
  uint64_t dev_offset = 0;
  std::string file_name;
};
std::vector<Status> VerifySstFilesChecksums(BlockChecksumEngine& engine,
                                            const std::vector<SstFileRef>& files,
                                            const uint8_t* dev_arena, uint64_t arena_len,
                                            std::vector<SstVerifyReport>* reports = nullptr);

// Write-side batching for flush and compaction:
// BlockBasedTableBuilder::WriteMaybeCompressedBlock
// (table/block_based/block_based_table_builder.cc:1311-1360) with the trailer
// deferred.  AddBlock places the block at its final file offset at once
// (handle = (offset, n), as the reference sets it) and writes the type byte;
// the LE32 checksum -- ComputeBuiltinChecksumWithLastByte(block, type) +
// ChecksumModifierForContext(base_context_checksum, offset) -- is filled when
// the block's window comes back from the GPU (one batch launch per window,
// two pinned windows alternating), and windows reach the sink
// (WritableFileWriter::Append) in file order.  block_align pads data blocks
// like :1385-1395; WriteFooter is FooterBuilder::Build (format.cc:231-330).
class GpuTrailerWriter {
 public:
  struct Options {
    ChecksumType checksum = kXXH3;       // BlockBasedTableOptions::checksum (table.h:257)
    uint32_t base_context_checksum = 0;  // format_version >= 6 (builder.cc:615-623)
    uint64_t start_offset = 0;           // file offset of the first block
    bool block_align = false;            // BlockBasedTableOptions::block_align
    uint64_t alignment = 4096;
    uint64_t window_bytes = 32ull << 20;  // blocks per GPU launch (bytes)
  };
  using Sink = std::function<Status(const char* data, size_t n)>;
  GpuTrailerWriter(const Options& opt, Sink sink, void* hip_stream = nullptr);
  ~GpuTrailerWriter();
  GpuTrailerWriter(const GpuTrailerWriter&) = delete;
  GpuTrailerWriter& operator=(const GpuTrailerWriter&) = delete;

  Status AddBlock(const char* data, size_t n, uint8_t compression_type, bool is_data_block,
                  uint64_t* handle_offset, uint64_t* handle_size);
  // every pending trailer computed and every byte handed to the sink
  Status Flush();
  // Flush + the footer for (metaindex, index) handles at the current offset
  Status WriteFooter(uint32_t format_version, uint64_t metaindex_offset, uint64_t metaindex_size,
                     uint64_t index_offset, uint64_t index_size);
  uint64_t offset() const { return offset_; }  // r->get_offset()
  const ChecksumStats& stats() const { return stats_; }

 private:
  struct Window;
  Status Reserve(Window& w, uint64_t bytes, uint64_t blocks);
  Status Launch(Window& w);
  Status Retire(Window& w);
  Options opt_;
  Sink sink_;
  void* stream_;
  uint64_t offset_;
  Window* win_[2];
  int cur_ = 0;
  Status status_;
  ChecksumStats stats_;
};

// ---- WAL ---------------------------------------------
//
// Recovery: DBImpl::RecoverLogFiles (db/db_impl/db_impl_open.cc:1195-1260)
// loops log::Reader::ReadRecord(&record, &scratch, wal_recovery_mode,
// &record_checksum), and the reader calls Reporter::Corruption(bytes,
// Status::Corruption(reason)) as it goes (log_reader.cc:69-320).  WalRecovery
// runs that reader over the whole log image on the GPU
// (forst_wal_recover_batch) and hands the same calls back in the same order:
// Next() yields each record (its bytes, LastRecordOffset, XXH3 record
// checksum) together with the reports ReadRecord made before returning it;
// trailing_reports() are the ones after the last record.
struct WalReport {
  uint64_t offset = 0;  // reader position of the physical record / event
  uint64_t bytes = 0;   // as passed to Reporter::Corruption
  uint32_t reason = 0;  // forst_wal_report_reason
  uint32_t type = 0;    // record type (unknown record type)
  std::string Text() const;  // the reader's reason string (log_reader.cc)
};
struct WalRecord {
  const char* data = nullptr;  // the record: into the host log (one fragment) or
  size_t size = 0;             //   the WalRecovery's scratch (several)
  uint64_t offset = 0;         // Reader::LastRecordOffset
  uint64_t checksum = 0;       // record_checksum (XXH3_64bits of the record)
  uint32_t n_fragments = 0;
  std::vector<WalReport> reports_before;
};
class WalRecovery {
 public:
  explicit WalRecovery(void* hip_stream = nullptr) : stream_(hip_stream) {}
  ~WalRecovery();
  WalRecovery(const WalRecovery&) = delete;
  WalRecovery& operator=(const WalRecovery&) = delete;
  // The log's bytes in device memory (d_log) and the same bytes in host memory
  // (host_log: record bytes are handed out from it).  wal_recovery_mode =
  // WALRecoveryMode (include/rocksdb/options.h).  Synchronises the stream.
  // NotSupported for a compressed WAL (kSetCompressionType naming kZSTD):
  // keep the serial log::Reader for that log.
  Status Recover(const uint8_t* d_log, const uint8_t* host_log, uint64_t log_len,
                 uint32_t log_number, int wal_recovery_mode);
  // false after the last record; status() is then OK unless the record
  // layout could not be followed on the host (NotSupported: fall back)
  bool Next(WalRecord* r);
  const std::vector<WalReport>& trailing_reports() const { return trailing_; }
  const Status& status() const { return status_; }
  const forst_wal_recover_result& result() const { return res_; }

 private:
  Status Grow(uint64_t rec_cap, uint64_t rep_cap);
  void* stream_;
  const uint8_t* host_ = nullptr;
  uint64_t len_ = 0;
  forst_wal_recover_result res_{};
  std::vector<uint64_t> off_, rlen_, hash_;
  std::vector<uint32_t> nfrag_;
  std::vector<WalReport> reports_, trailing_;
  size_t next_rec_ = 0, next_rep_ = 0;
  std::string scratch_;
  Status status_;
  void* dev_ = nullptr;  // device arrays (records, then reports)
  uint64_t rec_cap_ = 0, rep_cap_ = 0;
};

// Write side: log::Writer::AddRecord (db/log_writer.cc:65-160) +
// EmitPhysicalRecord (:228-263) for a whole write group at once.  Frame()
// lays the records out as AddRecord would from the writer's block offset
// (forst_wal_layout_at), assembles the image on the host (zero-padded block
// tails, [len][type][log number] headers, payloads), computes every record
// CRC in one GPU launch (forst_wal_record_crc_batch) and puts them in the
// headers: data()/size() is what AddRecord would have appended, record by
// record, and end_block_offset() the writer's block_offset_ afterwards.
struct ByteRange {
  const char* data;
  size_t size;
};
class WalWriteGroup {
 public:
  WalWriteGroup(bool recyclable, uint32_t log_number, void* hip_stream = nullptr)
      : recyclable_(recyclable), log_number_(log_number), stream_(hip_stream) {}
  ~WalWriteGroup();
  WalWriteGroup(const WalWriteGroup&) = delete;
  WalWriteGroup& operator=(const WalWriteGroup&) = delete;
  Status Frame(const std::vector<ByteRange>& records, uint32_t block_offset);
  const char* data() const { return image_.data(); }
  size_t size() const { return image_.size(); }
  uint32_t end_block_offset() const { return end_bo_; }
  uint64_t physical_records() const { return offs_.size(); }

 private:
  bool recyclable_;
  uint32_t log_number_;
  void* stream_;
  std::string image_;
  std::vector<uint64_t> offs_;
  uint32_t end_bo_ = 0;
  void* dev_ = nullptr;
  uint64_t dev_cap_ = 0;
};


// Per-KV protection (a15) at the reference's three call sites, over HOST
// bytes (copied to the device in one piece per call; synchronous):
//   VerifyMemtableEntries  MemTable::VerifyEntryChecksum (db/memtable.cc:
//     273-307) for entries at offsets[] of one arena buffer: a status code per
//     entry (forst_memtable_verify_batch); for a failing entry the caller
//     returns the reference's own MemTable::VerifyEntryChecksum(entry, ...) --
//     the exact Status text, allow_data_in_errors included
//   BlockKvChecksums       Block::Initialize{Data,Index,MetaIndex}Block-
//     ProtectionInfo (table/block_based/block.cc:1113-1235): each block's
//     kv_checksum_ bytes (forst_block_kv_checksum_batch)
//   WriteBatchProtection   WriteBatchInternal::UpdateProtectionInfo(wb, 8)
//     (db/write_batch.cc:3164-3181): each rep's ProtectionInfoKVOC64 values in
//     record order and its Iterate status (forst_write_batch_protect_batch)
struct KvBytes {
  const char* data;
  size_t size;
};
class KvProtection {
 public:
  explicit KvProtection(void* hip_stream = nullptr) : stream_(hip_stream) {}
  ~KvProtection();
  KvProtection(const KvProtection&) = delete;
  KvProtection& operator=(const KvProtection&) = delete;
  Status VerifyMemtableEntries(const char* arena, uint64_t arena_len,
                               const std::vector<uint64_t>& entry_offsets,
                               uint32_t protection_bytes, std::vector<uint8_t>* status);
  // kinds[i]: forst_block_kv_checksum_batch's block kind | flags
  Status BlockKvChecksums(const std::vector<KvBytes>& blocks, const std::vector<uint8_t>& kinds,
                          uint32_t protection_bytes, std::vector<std::string>* kv_checksums,
                          std::vector<uint8_t>* status);
  Status WriteBatchProtection(const std::vector<KvBytes>& reps,
                              std::vector<std::vector<uint64_t>>* prot,
                              std::vector<Status>* rep_status);
  // the Corruption text of a WriteBatch status code (write_batch.cc:361-716)
  static Status WriteBatchStatus(uint8_t code);

 private:
  Status Stage(const std::vector<KvBytes>& parts, std::vector<uint64_t>* offs);
  uint8_t* Grow(uint64_t bytes);
  void* stream_;
  void* dev_ = nullptr;
  uint64_t cap_ = 0;
  Status grow_status_;
};

}  // namespace forst_gpu
