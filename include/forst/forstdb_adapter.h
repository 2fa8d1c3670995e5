// include/forst/forstdb_adapter.h -- the C++ shim (forst/checksum_engine.h,
// namespace forst_gpu) inside a ForSt translation unit.
//
// The shim keeps its own small ChecksumType / Status in namespace forst_gpu,
// so it compiles next to ForSt's headers without redefining anything of
// namespace forstdb.  At a ForSt call site, include this header AFTER ForSt's
// own headers; it converts between the two vocabularies:
//   forst_gpu::FromForst(ROCKSDB_NAMESPACE::ChecksumType)   selector
//     (include/rocksdb/table.h:54-60; same values, checked below)
//   forst_gpu::ToForst(forst_gpu::Status)  -> ROCKSDB_NAMESPACE::Status
//     (include/rocksdb/status.h:35; same codes and messages, so the returned
//     status is the one the reference returns, e.g. the reader_common.cc:55-60
//     "block checksum mismatch: ..." Corruption)
//   forst_gpu::FromForst(ROCKSDB_NAMESPACE::Status / IOStatus) -> forst_gpu::Status
//     (for GpuTrailerWriter's sink, WritableFileWriter::Append)
// ForSt keeps using its own crc32c::Mask, ChecksumModifierForContext and
// IsSupportedChecksumType (util/crc32c.h, table/format.h, options_helper.h).
// tests/test_integration_cpp.py compiles INTEGRATION.md's call-site snippets
// against the reference headers with this adapter.
#pragma once

#include "rocksdb/status.h"
#include "rocksdb/table.h"

#include "checksum_engine.h"

namespace forst_gpu {

static_assert(static_cast<int>(ROCKSDB_NAMESPACE::kNoChecksum) == kNoChecksum &&
                  static_cast<int>(ROCKSDB_NAMESPACE::kCRC32c) == kCRC32c &&
                  static_cast<int>(ROCKSDB_NAMESPACE::kxxHash) == kxxHash &&
                  static_cast<int>(ROCKSDB_NAMESPACE::kxxHash64) == kxxHash64 &&
                  static_cast<int>(ROCKSDB_NAMESPACE::kXXH3) == kXXH3,
              "ChecksumType values (include/rocksdb/table.h:54-60)");
static_assert(static_cast<int>(ROCKSDB_NAMESPACE::Status::kCorruption) == Status::kCorruption &&
                  static_cast<int>(ROCKSDB_NAMESPACE::Status::kNotSupported) ==
                      Status::kNotSupported &&
                  static_cast<int>(ROCKSDB_NAMESPACE::Status::kInvalidArgument) ==
                      Status::kInvalidArgument &&
                  static_cast<int>(ROCKSDB_NAMESPACE::Status::kIOError) == Status::kIOError,
              "Status::Code values (include/rocksdb/status.h)");

inline ChecksumType FromForst(ROCKSDB_NAMESPACE::ChecksumType t) {
  return static_cast<ChecksumType>(t);
}

inline ROCKSDB_NAMESPACE::Status ToForst(const Status& s) {
  switch (s.code()) {
    case Status::kOk:
      return ROCKSDB_NAMESPACE::Status::OK();
    case Status::kCorruption:
      return ROCKSDB_NAMESPACE::Status::Corruption(s.message());
    case Status::kNotSupported:
      return ROCKSDB_NAMESPACE::Status::NotSupported(s.message());
    case Status::kInvalidArgument:
      return ROCKSDB_NAMESPACE::Status::InvalidArgument(s.message());
    default:
      return ROCKSDB_NAMESPACE::Status::IOError(s.message());
  }
}

inline Status FromForst(const ROCKSDB_NAMESPACE::Status& s) {
  if (s.ok()) return Status::OK();
  const std::string m = s.getState() ? s.getState() : "";
  switch (s.code()) {
    case ROCKSDB_NAMESPACE::Status::kCorruption:
      return Status::Corruption(m);
    case ROCKSDB_NAMESPACE::Status::kNotSupported:
      return Status::NotSupported(m);
    case ROCKSDB_NAMESPACE::Status::kInvalidArgument:
      return Status::InvalidArgument(m);
    default:
      return Status::IOError(s.ToString());
  }
}

}  // namespace forst_gpu
