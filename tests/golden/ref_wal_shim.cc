// tests/golden/ref_wal_shim.cc -- TEST INFRASTRUCTURE ONLY (fixture veneer).
//
// A C entry point over the REFERENCE's own log::Reader (db/log_reader.cc),
// compiled by tests/golden/gen_wal_golden.py against the reference archive
// (tests/golden/refbuild.py) in a temporary directory and never shipped.
// The log image is fed through an in-memory FSSequentialFile exactly as
// db/log_test.cc:55-120's StringSource does, and ReadRecord(..., &checksum)
// (log_reader.cc:69) is driven to the end as DBImpl::RecoverLogFiles does
// (db/db_impl/db_impl_open.cc:1210).  Output is a text transcript:
//   R <LastRecordOffset> <length> <record_checksum hex>
//   C <bytes> <Status::ToString()>        (Reporter::Corruption, in order)
//   E <LastRecordEnd> <IsEOF>             (after ReadRecord returned false)
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "db/log_reader.h"
#include "file/sequence_file_reader.h"
#include "rocksdb/file_system.h"

using namespace ROCKSDB_NAMESPACE;

namespace {

class MemSource : public FSSequentialFile {
 public:
  MemSource(const char* p, size_t n) : p_(p), n_(n) {}
  IOStatus Read(size_t n, const IOOptions&, Slice* result, char* scratch,
                IODebugContext*) override {
    const size_t k = n < n_ - pos_ ? n : n_ - pos_;
    std::memcpy(scratch, p_ + pos_, k);
    *result = Slice(scratch, k);
    pos_ += k;
    return IOStatus::OK();
  }
  IOStatus Skip(uint64_t n) override {
    pos_ = n > n_ - pos_ ? n_ : pos_ + n;
    return IOStatus::OK();
  }

 private:
  const char* p_;
  size_t n_;
  size_t pos_ = 0;
};

class Transcript : public log::Reader::Reporter {
 public:
  explicit Transcript(std::string* out) : out_(out) {}
  void Corruption(size_t bytes, const Status& s) override {
    char buf[64];
    std::snprintf(buf, sizeof(buf), "C %zu ", bytes);
    *out_ += buf;
    *out_ += s.ToString();
    *out_ += "\n";
  }

 private:
  std::string* out_;
};

}  // namespace

extern "C" __attribute__((visibility("default"))) int ref_wal_read(
    const char* log, size_t len, unsigned long long log_number, int mode, char* out,
    size_t cap, size_t* out_len) {
  std::string t;
  Transcript rep(&t);
  std::unique_ptr<FSSequentialFile> src(new MemSource(log, len));
  std::unique_ptr<SequentialFileReader> file(new SequentialFileReader(std::move(src), "wal"));
  log::Reader reader(nullptr, std::move(file), &rep, /*checksum=*/true, log_number);
  Slice record;
  std::string scratch;
  uint64_t checksum = 0;
  char buf[96];
  while (reader.ReadRecord(&record, &scratch, static_cast<WALRecoveryMode>(mode), &checksum)) {
    std::snprintf(buf, sizeof(buf), "R %llu %zu %016llx\n",
                  static_cast<unsigned long long>(reader.LastRecordOffset()), record.size(),
                  static_cast<unsigned long long>(checksum));
    t += buf;
  }
  std::snprintf(buf, sizeof(buf), "E %llu %d\n",
                static_cast<unsigned long long>(reader.LastRecordEnd()),
                reader.IsEOF() ? 1 : 0);
  t += buf;
  *out_len = t.size();
  if (t.size() > cap) return 1;
  std::memcpy(out, t.data(), t.size());
  return 0;
}
