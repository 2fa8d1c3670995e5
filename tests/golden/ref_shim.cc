// tests/golden/ref_shim.cc -- TEST INFRASTRUCTURE ONLY (fixture generation).
//
// A thin extern "C" veneer over the *reference's own* checksum code, compiled
// from the sources where they lie under /root/reference by gen_golden.py
// into a temporary directory OUTSIDE the repository.  Nothing here re-implements
// the algorithms: every function forwards to the reference symbol named in its
// comment.  Used only to pin the CPU restatement in oracle/oracle.c against
// the real reference by generating the tests/golden fixtures (data only).  The
// compiled library never enters the repository or travels to the GPU box; the
// product (forst_amd/) never links or loads it.

#include <cstdint>
#include <cstring>

#include "rocksdb/table.h"
#include "table/format.h"
#include "util/coding.h"
#include "util/crc32c.h"
#include "util/hash.h"
#include "util/xxhash.h"

using namespace ROCKSDB_NAMESPACE;

#define SHIM_API __attribute__((visibility("default")))

extern "C" {

// util/crc32c.h:25 crc32c::Extend
SHIM_API uint32_t ref_crc32c_extend(uint32_t crc, const char* p, size_t n) {
  return crc32c::Extend(crc, p, n);
}
// util/crc32c.h:35 crc32c::Value
SHIM_API uint32_t ref_crc32c_value(const char* p, size_t n) {
  return crc32c::Value(p, n);
}
// util/crc32c.h:30 crc32c::Crc32cCombine
SHIM_API uint32_t ref_crc32c_combine(uint32_t a, uint32_t b, size_t blen) {
  return crc32c::Crc32cCombine(a, b, blen);
}
// util/crc32c.h:44 / :50
SHIM_API uint32_t ref_crc32c_mask(uint32_t c) { return crc32c::Mask(c); }
SHIM_API uint32_t ref_crc32c_unmask(uint32_t c) { return crc32c::Unmask(c); }

// util/xxhash.h:5311 XXH3_64bits (v0.8.1, ROCKSDB_ prefixed)
SHIM_API uint64_t ref_xxh3_64(const void* p, size_t n) {
  return XXH3_64bits(p, n);
}
SHIM_API uint32_t ref_xxh32(const void* p, size_t n, uint32_t seed) {
  return XXH32(p, n, seed);
}
SHIM_API uint64_t ref_xxh64(const void* p, size_t n, uint64_t seed) {
  return XXH64(p, n, seed);
}

// util/hash.cc:81 Hash64 (XXPH3 preview 0.7.2) -- db/kv_checksum.h NPHash64
SHIM_API uint64_t ref_hash64(const char* p, size_t n, uint64_t seed) {
  return Hash64(p, n, seed);
}

// table/format.cc:568 ComputeBuiltinChecksum
SHIM_API uint32_t ref_compute_builtin_checksum(int type, const char* p,
                                               size_t n) {
  return ComputeBuiltinChecksum(static_cast<ChecksumType>(type), p, n);
}
// table/format.cc:594 ComputeBuiltinChecksumWithLastByte
SHIM_API uint32_t ref_compute_builtin_checksum_with_last_byte(int type,
                                                              const char* p,
                                                              size_t n,
                                                              char last) {
  return ComputeBuiltinChecksumWithLastByte(static_cast<ChecksumType>(type), p,
                                            n, last);
}
// table/format.h:119 ChecksumModifierForContext
SHIM_API uint32_t ref_checksum_modifier_for_context(uint32_t base,
                                                    uint64_t offset) {
  return ChecksumModifierForContext(base, offset);
}

}  // extern "C"
