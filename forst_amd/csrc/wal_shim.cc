// forst_amd/csrc/wal_shim.cc -- the WAL half of the C++ host shim
// (include/forst/checksum_engine.h): WalRecovery hands
// forst_wal_recover_batch's results back the way DBImpl::RecoverLogFiles
// consumes log::Reader::ReadRecord (db/db_impl/db_impl_open.cc:1195-1260),
// WalWriteGroup frames a write group as log::Writer::AddRecord does
// (db/log_writer.cc:65-160, :228-263) with every record CRC from one launch.
#include "../../include/forst/checksum_engine.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

namespace forst_gpu {

namespace {
constexpr uint64_t kBlockSize = 32768;  // db/log_format.h:45
constexpr uint32_t kHeaderSize = 7;     // :48
constexpr uint32_t kRecyclableHeaderSize = 11;  // :52

Status FromRc(int rc) {
  if (rc == FORST_OK) return Status::OK();
  if (rc == FORST_EUNSUPPORTED) return Status::NotSupported(forst_last_error());
  if (rc == FORST_EINVAL) return Status::InvalidArgument(forst_last_error());
  return Status::IOError(forst_last_error());
}
Status FromHip(hipError_t e, const char* what) {
  if (e == hipSuccess) return Status::OK();
  return Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}
bool recyclable_type(uint32_t t) { return (t >= 5 && t <= 8) || t == 11; }  // log_format.h:20-41
uint64_t align8(uint64_t x) { return (x + 7) & ~uint64_t{7}; }
}  // namespace

// the reason strings of log_reader.cc:69-320 (ReportCorruption calls)
std::string WalReport::Text() const {
  switch (reason) {
    case FORST_WAL_PARTIAL_RECORD_1: return "partial record without end(1)";
    case FORST_WAL_PARTIAL_RECORD_2: return "partial record without end(2)";
    case FORST_WAL_MISSING_START_1: return "missing start of fragmented record(1)";
    case FORST_WAL_MISSING_START_2: return "missing start of fragmented record(2)";
    case FORST_WAL_ERROR_IN_MIDDLE: return "error in middle of record";
    case FORST_WAL_CHECKSUM_MISMATCH: return "checksum mismatch";
    case FORST_WAL_BAD_RECORD_LENGTH: return "bad record length";
    case FORST_WAL_TRUNCATED_HEADER: return "truncated header";
    case FORST_WAL_TRAILING_DATA: return "error reading trailing data";
    case FORST_WAL_TRUNCATED_BODY: return "truncated record body";
    case FORST_WAL_UNKNOWN_TYPE: return "unknown record type " + std::to_string(type);
    case FORST_WAL_MULTIPLE_COMPRESSION: return "read multiple SetCompressionType records";
    case FORST_WAL_COMPRESSION_NOT_FIRST: return "SetCompressionType not the first record";
    case FORST_WAL_COMPRESSION_DECODE: return "could not decode SetCompressionType record";
    case FORST_WAL_TS_INTERSPERSED:
      return "user-defined timestamp size record interspersed partial record";
    case FORST_WAL_TS_DECODE: return "could not decode user-defined timestamp size record";
    case FORST_WAL_TS_ZERO:
      return "User-defined timestamp size record contains zero timestamp size.";
    case FORST_WAL_TS_DUPLICATE:
      return "User-defined timestamp size record contains update to recorded column family.";
  }
  return "unknown report reason " + std::to_string(reason);
}

WalRecovery::~WalRecovery() { (void)hipFree(dev_); }

Status WalRecovery::Grow(uint64_t rec_cap, uint64_t rep_cap) {
  if (rec_cap <= rec_cap_ && rep_cap <= rep_cap_ && dev_) return Status::OK();
  rec_cap = rec_cap > rec_cap_ ? rec_cap : rec_cap_;
  rep_cap = rep_cap > rep_cap_ ? rep_cap : rep_cap_;
  (void)hipFree(dev_);
  dev_ = nullptr;
  rec_cap_ = rep_cap_ = 0;
  const uint64_t bytes = align8(rec_cap * 28) + align8(rep_cap * 24);
  Status s = FromHip(hipMalloc(&dev_, bytes ? bytes : 8), "hipMalloc");
  if (s.ok()) {
    rec_cap_ = rec_cap;
    rep_cap_ = rep_cap;
  }
  return s;
}

Status WalRecovery::Recover(const uint8_t* d_log, const uint8_t* host_log, uint64_t log_len,
                            uint32_t log_number, int wal_recovery_mode) {
  host_ = host_log;
  len_ = log_len;
  next_rec_ = next_rep_ = 0;
  off_.clear(), rlen_.clear(), hash_.clear(), nfrag_.clear();
  reports_.clear(), trailing_.clear();
  status_ = Status::OK();
  if (log_len && (!d_log || !host_log)) return status_ = Status::InvalidArgument("null log");
  hipStream_t st = static_cast<hipStream_t>(stream_);
  uint64_t rec_cap = rec_cap_ ? rec_cap_ : (log_len / 1024 > 1024 ? log_len / 1024 : 1024);
  uint64_t rep_cap = rep_cap_ ? rep_cap_ : 1024;
  for (;;) {
    Status s = Grow(rec_cap, rep_cap);
    if (!s.ok()) return status_ = s;
    char* p = static_cast<char*>(dev_);
    forst_wal_records recs{reinterpret_cast<uint64_t*>(p),
                           reinterpret_cast<uint64_t*>(p + 8 * rec_cap_),
                           reinterpret_cast<uint64_t*>(p + 16 * rec_cap_),
                           reinterpret_cast<uint32_t*>(p + 24 * rec_cap_)};
    char* q = p + align8(rec_cap_ * 28);
    forst_wal_reports reps{reinterpret_cast<uint64_t*>(q),
                           reinterpret_cast<uint64_t*>(q + 8 * rep_cap_),
                           reinterpret_cast<uint32_t*>(q + 16 * rep_cap_),
                           reinterpret_cast<uint32_t*>(q + 20 * rep_cap_)};
    s = FromRc(forst_wal_recover_batch(d_log, log_len, log_number, wal_recovery_mode, recs,
                                       rec_cap_, reps, rep_cap_, &res_, stream_));
    if (!s.ok()) return status_ = s;
    if (!res_.truncated) {
      const uint64_t nr = res_.n_records, np = res_.n_reports;
      off_.resize(nr), rlen_.resize(nr), hash_.resize(nr), nfrag_.resize(nr);
      std::vector<uint64_t> ro(np), rb(np);
      std::vector<uint32_t> rr(np), rt(np);
      struct Copy {
        void* dst;
        const void* src;
        size_t n;
      } copies[] = {{off_.data(), recs.offset, nr * 8}, {rlen_.data(), recs.length, nr * 8},
                    {hash_.data(), recs.hash, nr * 8},  {nfrag_.data(), recs.n_fragments, nr * 4},
                    {ro.data(), reps.offset, np * 8},   {rb.data(), reps.bytes, np * 8},
                    {rr.data(), reps.reason, np * 4},   {rt.data(), reps.type, np * 4}};
      for (const Copy& c : copies) {
        if (!c.n) continue;
        s = FromHip(hipMemcpyAsync(c.dst, c.src, c.n, hipMemcpyDeviceToHost, st),
                    "hipMemcpyAsync");
        if (!s.ok()) return status_ = s;
      }
      s = FromHip(hipStreamSynchronize(st), "hipStreamSynchronize");
      if (!s.ok()) return status_ = s;
      reports_.resize(np);
      for (uint64_t i = 0; i < np; ++i) reports_[i] = WalReport{ro[i], rb[i], rr[i], rt[i]};
      return Status::OK();
    }
    rec_cap = res_.n_records > rec_cap_ ? res_.n_records : rec_cap_;
    rep_cap = res_.n_reports > rep_cap_ ? res_.n_reports : rep_cap_;
  }
}

// The record's fragments are consecutive physical records from the reader's
// position at LastRecordOffset (ReadRecord consumes them back to back; a
// < header-size block tail, or a recyclable log's zero-filled one, is skipped
// as ReadPhysicalRecord skips it).  Reports made during this ReadRecord call
// lie before the end of its last fragment.
bool WalRecovery::Next(WalRecord* r) {
  if (!status_.ok()) return false;
  if (next_rec_ >= off_.size()) {
    trailing_.assign(reports_.begin() + static_cast<std::ptrdiff_t>(next_rep_), reports_.end());
    next_rep_ = reports_.size();
    return false;
  }
  const size_t k = next_rec_++;
  uint64_t p = off_[k];
  const uint32_t nf = nfrag_[k];
  scratch_.clear();
  const char* single = nullptr;
  uint64_t got = 0;
  for (uint32_t f = 0; f < nf; ++f) {
    for (;;) {  // block tails the writer padded
      const uint64_t left = kBlockSize - p % kBlockSize;
      if (left < kHeaderSize) {
        p += left;
        continue;
      }
      if (p + kHeaderSize <= len_ && host_[p + 4] == 0 && host_[p + 5] == 0 && host_[p + 6] == 0 &&
          left < kRecyclableHeaderSize) {
        p += left;  // a recyclable writer's 7..10-byte zero tail
        continue;
      }
      break;
    }
    if (p + kHeaderSize > len_) break;
    const uint32_t t = static_cast<uint8_t>(host_[p + 6]);
    const uint32_t hs = recyclable_type(t) ? kRecyclableHeaderSize : kHeaderSize;
    const uint64_t n = static_cast<uint64_t>(host_[p + 4]) | static_cast<uint64_t>(host_[p + 5]) << 8;
    if (p + hs + n > len_) break;
    const char* payload = reinterpret_cast<const char*>(host_ + p + hs);
    if (nf == 1)
      single = payload;
    else
      scratch_.append(payload, n);
    got += n;
    p += hs + n;
  }
  if (got != rlen_[k]) {
    status_ = Status::NotSupported(
        "WAL record layout not followed on the host (offset " + std::to_string(off_[k]) +
        "): use log::Reader for this log");
    return false;
  }
  r->data = nf == 1 ? single : scratch_.data();
  r->size = static_cast<size_t>(got);
  r->offset = off_[k];
  r->checksum = hash_[k];
  r->n_fragments = nf;
  r->reports_before.clear();
  while (next_rep_ < reports_.size() && reports_[next_rep_].offset < p)
    r->reports_before.push_back(reports_[next_rep_++]);
  return true;
}

WalWriteGroup::~WalWriteGroup() { (void)hipFree(dev_); }

Status WalWriteGroup::Frame(const std::vector<ByteRange>& records, uint32_t block_offset) {
  image_.clear();
  offs_.clear();
  const uint64_t n = records.size();
  std::vector<uint32_t> lens(n);
  for (uint64_t i = 0; i < n; ++i) {
    if (records[i].size > 0xffffffffu) return Status::InvalidArgument("record too large");
    lens[i] = static_cast<uint32_t>(records[i].size);
  }
  uint64_t np = 0, npad = 0, total = 0;
  uint32_t end = 0;
  Status s = FromRc(forst_wal_layout_at(lens.data(), n, recyclable_, block_offset, nullptr,
                                        nullptr, nullptr, 0, nullptr, nullptr, 0, &np, &npad,
                                        &total, &end));
  if (!s.ok()) return s;
  std::vector<uint32_t> flen(np);
  std::vector<uint8_t> ftype(np);
  offs_.resize(np);
  s = FromRc(forst_wal_layout_at(lens.data(), n, recyclable_, block_offset, offs_.data(),
                                 flen.data(), ftype.data(), np, nullptr, nullptr, 0, &np, &npad,
                                 &total, &end));
  if (!s.ok()) return s;
  end_bo_ = end;
  image_.assign(total, '\0');  // block-tail pads stay zero (log_writer.cc:91-100)
  const uint32_t hs = recyclable_ ? kRecyclableHeaderSize : kHeaderSize;
  int64_t rec = -1;  // logical record of the fragment, bytes of it placed
  uint64_t used = 0;
  for (uint64_t i = 0; i < np; ++i) {
    const uint8_t t = ftype[i];
    if (t == 1 || t == 2 || t == 5 || t == 6) {  // Full / First: the next record
      ++rec;
      used = 0;
    }
    char* h = &image_[offs_[i]];
    h[4] = static_cast<char>(flen[i] & 0xff);  // EmitPhysicalRecord, :236-258
    h[5] = static_cast<char>(flen[i] >> 8);
    h[6] = static_cast<char>(t);
    if (recyclable_) std::memcpy(h + 7, &log_number_, 4);  // EncodeFixed32 (little endian)
    if (flen[i]) std::memcpy(h + hs, records[static_cast<size_t>(rec)].data + used, flen[i]);
    used += flen[i];
  }
  if (np == 0) return Status::OK();
  // every CRC from one launch: the image in device memory, CRCs (4 B each) back
  hipStream_t st = static_cast<hipStream_t>(stream_);
  const uint64_t need = align8(total) + np * 8 + np * 4 + np * 4;
  if (need > dev_cap_) {
    (void)hipFree(dev_);
    dev_ = nullptr;
    dev_cap_ = 0;
    s = FromHip(hipMalloc(&dev_, need), "hipMalloc");
    if (!s.ok()) return s;
    dev_cap_ = need;
  }
  uint8_t* d_img = static_cast<uint8_t*>(dev_);
  uint64_t* d_off = reinterpret_cast<uint64_t*>(d_img + align8(total));
  uint32_t* d_crc = reinterpret_cast<uint32_t*>(d_off + np);
  uint32_t* d_len = d_crc + np;
  s = FromHip(hipMemcpyAsync(d_img, image_.data(), total, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok())
    s = FromHip(hipMemcpyAsync(d_off, offs_.data(), np * 8, hipMemcpyHostToDevice, st),
                "hipMemcpyAsync");
  if (s.ok())
    s = FromHip(hipMemcpyAsync(d_len, flen.data(), np * 4, hipMemcpyHostToDevice, st),
                "hipMemcpyAsync");
  if (!s.ok()) return s;
  s = FromRc(forst_wal_record_crc_lengths(d_img, total, d_off, d_len, np, recyclable_, 0, d_crc,
                                          stream_));
  if (!s.ok()) return s;
  std::vector<uint32_t> crc(np);
  s = FromHip(hipMemcpyAsync(crc.data(), d_crc, np * 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (!s.ok()) return s;
  for (uint64_t i = 0; i < np; ++i) std::memcpy(&image_[offs_[i]], &crc[i], 4);  // EncodeFixed32
  return Status::OK();
}

}  // namespace forst_gpu

// ---- per-KV protection at its call sites (a15) ------------------------------
namespace forst_gpu {

KvProtection::~KvProtection() { (void)hipFree(dev_); }

uint8_t* KvProtection::Grow(uint64_t bytes) {
  if (bytes > cap_) {
    (void)hipFree(dev_);
    dev_ = nullptr;
    cap_ = 0;
    grow_status_ = FromHip(hipMalloc(&dev_, bytes), "hipMalloc");
    if (!grow_status_.ok()) return nullptr;
    cap_ = bytes;
  }
  grow_status_ = Status::OK();
  return static_cast<uint8_t*>(dev_);
}

Status KvProtection::VerifyMemtableEntries(const char* arena, uint64_t arena_len,
                                           const std::vector<uint64_t>& entry_offsets,
                                           uint32_t protection_bytes,
                                           std::vector<uint8_t>* status) {
  const uint64_t n = entry_offsets.size();
  status->assign(n, 0);
  if (!n) return Status::OK();
  const uint64_t a8 = align8(arena_len);
  uint8_t* d = Grow(a8 + 9 * n);
  if (!d) return grow_status_;
  uint64_t* d_off = reinterpret_cast<uint64_t*>(d + a8);
  uint8_t* d_st = d + a8 + 8 * n;
  hipStream_t st = static_cast<hipStream_t>(stream_);
  Status s = FromHip(hipMemcpyAsync(d, arena, arena_len, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok())
    s = FromHip(hipMemcpyAsync(d_off, entry_offsets.data(), 8 * n, hipMemcpyHostToDevice, st),
                "hipMemcpyAsync");
  if (s.ok())
    s = FromRc(forst_memtable_verify_batch(d, arena_len, d_off, n, protection_bytes, nullptr, d_st,
                                           nullptr, stream_));
  if (s.ok())
    s = FromHip(hipMemcpyAsync(status->data(), d_st, n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipStreamSynchronize(st), "hipStreamSynchronize");
  return s;
}

// the parts back to back (8-byte aligned) in the device buffer: offs[i]
Status KvProtection::Stage(const std::vector<KvBytes>& parts, std::vector<uint64_t>* offs) {
  offs->resize(parts.size());
  uint64_t total = 0;
  for (size_t i = 0; i < parts.size(); ++i) {
    (*offs)[i] = total;
    total = align8(total + parts[i].size);
  }
  std::string img(total + 16, '\0');
  for (size_t i = 0; i < parts.size(); ++i)
    if (parts[i].size) std::memcpy(&img[(*offs)[i]], parts[i].data, parts[i].size);
  uint8_t* d = Grow(img.size());
  if (!d) return grow_status_;
  return FromHip(hipMemcpyAsync(d, img.data(), img.size(), hipMemcpyHostToDevice,
                                static_cast<hipStream_t>(stream_)),
                 "hipMemcpyAsync");
}

Status KvProtection::BlockKvChecksums(const std::vector<KvBytes>& blocks,
                                      const std::vector<uint8_t>& kinds, uint32_t protection_bytes,
                                      std::vector<std::string>* kv_checksums,
                                      std::vector<uint8_t>* status) {
  const uint64_t n = blocks.size();
  kv_checksums->assign(n, std::string());
  status->assign(n, 0);
  if (!n) return Status::OK();
  if (kinds.size() != n) return Status::InvalidArgument("one kind per block");
  std::vector<uint64_t> offs;
  Status s = Stage(blocks, &offs);
  if (!s.ok()) return s;
  const uint64_t img = offs.back() + align8(blocks.back().size) + 16;
  std::vector<uint32_t> sizes(n);
  for (uint64_t i = 0; i < n; ++i) sizes[i] = static_cast<uint32_t>(blocks[i].size);
  // device: image | offsets | sizes | kinds | first_key | status, then the checksums
  void* aux = nullptr;
  s = FromHip(hipMalloc(&aux, 8 * (2 * n + 1) + 4 * n + 2 * n + 64), "hipMalloc");
  if (!s.ok()) return s;
  uint8_t* a = static_cast<uint8_t*>(aux);
  uint64_t* d_off = reinterpret_cast<uint64_t*>(a);
  uint64_t* d_first = d_off + n;
  uint32_t* d_sz = reinterpret_cast<uint32_t*>(d_first + n + 1);
  uint8_t* d_kind = reinterpret_cast<uint8_t*>(d_sz + n);
  uint8_t* d_st = d_kind + n;
  hipStream_t st = static_cast<hipStream_t>(stream_);
  s = FromHip(hipMemcpyAsync(d_off, offs.data(), 8 * n, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipMemcpyAsync(d_sz, sizes.data(), 4 * n, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipMemcpyAsync(d_kind, kinds.data(), n, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  uint64_t total = 0;
  if (s.ok()) {  // the key total first (capacity 0), then the checksums
    const int rc = forst_block_kv_checksum_batch(static_cast<uint8_t*>(dev_), img, d_off, d_sz,
                                                 d_kind, n, protection_bytes, d_first, nullptr,
                                                 nullptr, 0, d_st, &total, stream_);
    if (rc != FORST_OK && !(rc == FORST_EINVAL && total > 0)) s = FromRc(rc);
  }
  void* d_enc = nullptr;
  if (s.ok() && total) s = FromHip(hipMalloc(&d_enc, total * protection_bytes), "hipMalloc");
  if (s.ok() && total)
    s = FromRc(forst_block_kv_checksum_batch(static_cast<uint8_t*>(dev_), img, d_off, d_sz, d_kind,
                                             n, protection_bytes, d_first,
                                             static_cast<uint8_t*>(d_enc), nullptr, total, d_st,
                                             &total, stream_));
  std::vector<uint64_t> first(n + 1, 0);
  std::string enc(total * protection_bytes, '\0');
  if (s.ok())
    s = FromHip(hipMemcpyAsync(first.data(), d_first, 8 * (n + 1), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipMemcpyAsync(status->data(), d_st, n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok() && total)
    s = FromHip(hipMemcpyAsync(&enc[0], d_enc, enc.size(), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipStreamSynchronize(st), "hipStreamSynchronize");
  (void)hipFree(d_enc);
  (void)hipFree(aux);
  if (!s.ok()) return s;
  for (uint64_t i = 0; i < n; ++i)
    (*kv_checksums)[i] = enc.substr(first[i] * protection_bytes,
                                    (first[i + 1] - first[i]) * protection_bytes);
  return Status::OK();
}

Status KvProtection::WriteBatchStatus(uint8_t code) {
  static const char* kText[] = {"",
                                "malformed WriteBatch (too small)",
                                "bad WriteBatch Put",
                                "bad WriteBatch Delete",
                                "bad WriteBatch DeleteRange",
                                "bad WriteBatch Merge",
                                "bad WriteBatch BlobIndex",
                                "bad WriteBatch Blob",
                                "bad EndPrepare XID",
                                "bad commit timestamp",
                                "bad Commit XID",
                                "bad Rollback XID",
                                "bad WriteBatch PutEntity",
                                "unknown WriteBatch tag",
                                "WriteBatch has wrong count"};
  if (code == 0) return Status::OK();
  if (code < sizeof(kText) / sizeof(kText[0])) return Status::Corruption(kText[code]);
  return Status::InvalidArgument("WriteBatch rep outside the staged buffer");
}

Status KvProtection::WriteBatchProtection(const std::vector<KvBytes>& reps,
                                          std::vector<std::vector<uint64_t>>* prot,
                                          std::vector<Status>* rep_status) {
  const uint64_t n = reps.size();
  prot->assign(n, std::vector<uint64_t>());
  rep_status->assign(n, Status::OK());
  if (!n) return Status::OK();
  std::vector<uint64_t> offs;
  Status s = Stage(reps, &offs);
  if (!s.ok()) return s;
  const uint64_t img = offs.back() + align8(reps.back().size) + 16;
  std::vector<uint32_t> sizes(n);
  for (uint64_t i = 0; i < n; ++i) sizes[i] = static_cast<uint32_t>(reps[i].size);
  void* aux = nullptr;
  s = FromHip(hipMalloc(&aux, 8 * (2 * n + 1) + 4 * n + 4 * n + n + 64), "hipMalloc");
  if (!s.ok()) return s;
  uint64_t* d_off = static_cast<uint64_t*>(aux);
  uint64_t* d_first = d_off + n;
  uint32_t* d_sz = reinterpret_cast<uint32_t*>(d_first + n + 1);
  uint32_t* d_np = d_sz + n;
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_np + n);
  hipStream_t st = static_cast<hipStream_t>(stream_);
  s = FromHip(hipMemcpyAsync(d_off, offs.data(), 8 * n, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipMemcpyAsync(d_sz, sizes.data(), 4 * n, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  uint64_t total = 0;
  if (s.ok()) {
    const int rc = forst_write_batch_protect_batch(static_cast<uint8_t*>(dev_), img, d_off, d_sz, n,
                                                   d_first, nullptr, 0, nullptr, nullptr, &total,
                                                   stream_);
    if (rc != FORST_OK && !(rc == FORST_EINVAL && total > 0)) s = FromRc(rc);
  }
  void* d_prot = nullptr;
  if (s.ok()) s = FromHip(hipMalloc(&d_prot, 8 * (total ? total : 1)), "hipMalloc");
  if (s.ok())
    s = FromRc(forst_write_batch_protect_batch(static_cast<uint8_t*>(dev_), img, d_off, d_sz, n,
                                               d_first, static_cast<uint64_t*>(d_prot), total,
                                               d_st, d_np, &total, stream_));
  std::vector<uint64_t> first(n + 1, 0), all(total ? total : 1);
  std::vector<uint32_t> np(n);
  std::vector<uint8_t> code(n);
  if (s.ok()) s = FromHip(hipMemcpyAsync(first.data(), d_first, 8 * (n + 1), hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipMemcpyAsync(np.data(), d_np, 4 * n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipMemcpyAsync(code.data(), d_st, n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok() && total)
    s = FromHip(hipMemcpyAsync(all.data(), d_prot, 8 * total, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = FromHip(hipStreamSynchronize(st), "hipStreamSynchronize");
  (void)hipFree(d_prot);
  (void)hipFree(aux);
  if (!s.ok()) return s;
  for (uint64_t i = 0; i < n; ++i) {
    (*prot)[i].assign(all.begin() + first[i], all.begin() + first[i] + np[i]);
    (*rep_status)[i] = WriteBatchStatus(code[i]);
  }
  return Status::OK();
}

}  // namespace forst_gpu
