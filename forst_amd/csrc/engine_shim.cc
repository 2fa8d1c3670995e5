// forst_amd/csrc/engine_shim.cc -- C++ host shim (namespace forst_gpu) over the
// C ABI; see include/forst/checksum_engine.h for the reference mapping.
#include "../../include/forst/checksum_engine.h"

#include <hip/hip_runtime.h>

#include <chrono>
#include <string>
#include <vector>

namespace forst_gpu {

std::string Status::ToString() const {
  switch (code_) {
    case kOk:
      return "OK";
    case kCorruption:
      return "Corruption: " + msg_;
    case kNotSupported:
      return "Not implemented: " + msg_;
    case kInvalidArgument:
      return "Invalid argument: " + msg_;
    case kIOError:
      return "IO error: " + msg_;
  }
  return msg_;
}

bool GpuSupportsChecksumType(ChecksumType t) {
  return t == kNoChecksum || t == kCRC32c || t == kxxHash || t == kxxHash64 || t == kXXH3;
}

// table/block_based/reader_common.cc:55-60
std::string BlockChecksumMismatchMessage(ChecksumType type, uint32_t stored, uint32_t computed,
                                         bool context_removed, const std::string& file_name,
                                         uint64_t offset, uint64_t block_size) {
  return "block checksum mismatch: stored" +
         std::string(context_removed ? "(context removed)" : "") + " = " +
         std::to_string(stored) + ", computed = " + std::to_string(computed) +
         ", type = " + std::to_string(static_cast<int>(type)) + "  in " + file_name + " offset " +
         std::to_string(offset) + " size " + std::to_string(block_size);
}

namespace {
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
}  // namespace

BlockChecksumEngine::~BlockChecksumEngine() {
  (void)hipFree(d_computed_);
  (void)hipFree(d_stored_);
  (void)hipFree(d_ok_);
  (void)hipFree(d_mod_);
  (void)hipFree(d_bad_);
}

Status BlockChecksumEngine::EnsureScratch(uint64_t n) {
  if (!d_bad_) {
    Status s = FromHip(hipMalloc(&d_bad_, sizeof(*d_bad_)), "hipMalloc");
    if (!s.ok()) return s;
  }
  if (n <= cap_) return Status::OK();
  (void)hipFree(d_computed_);
  (void)hipFree(d_stored_);
  (void)hipFree(d_ok_);
  (void)hipFree(d_mod_);
  d_computed_ = d_stored_ = d_mod_ = nullptr;
  d_ok_ = nullptr;
  cap_ = 0;
  Status s = FromHip(hipMalloc(&d_computed_, n * 4), "hipMalloc");
  if (s.ok()) s = FromHip(hipMalloc(&d_stored_, n * 4), "hipMalloc");
  if (s.ok()) s = FromHip(hipMalloc(&d_ok_, n), "hipMalloc");
  if (s.ok()) s = FromHip(hipMalloc(&d_mod_, n * 4), "hipMalloc");
  if (s.ok()) cap_ = n;
  return s;
}

Status BlockChecksumEngine::ComputeChecksums(ChecksumType type, const DeviceBlockBatch& b,
                                             const uint8_t* last_bytes, const uint32_t* modifiers,
                                             uint32_t* out) {
  int rc = forst_block_checksum_batch(type, b.base, b.base_len, b.offsets, b.sizes, last_bytes,
                                      modifiers, out, b.n, stream_);
  if (rc == FORST_OK) stats_.block_checksum_compute_count += b.n;
  return FromRc(rc);
}

Status BlockChecksumEngine::WriteTrailers(ChecksumType type, const DeviceBlockBatch& b,
                                          const uint8_t* last_bytes, const uint32_t* modifiers,
                                          uint32_t* out) {
  int rc = forst_block_trailer_batch(type, const_cast<uint8_t*>(b.base), b.base_len, b.offsets,
                                     b.sizes, last_bytes, modifiers, out, b.n, stream_);
  if (rc == FORST_OK) stats_.block_checksum_compute_count += b.n;
  return FromRc(rc);
}

Status BlockChecksumEngine::VerifyBlocks(ChecksumType type, uint32_t base_context_checksum,
                                         const DeviceBlockBatch& b, const std::string& file_name,
                                         const std::vector<uint64_t>& file_offsets,
                                         std::vector<uint64_t>* failed) {
  if (!IsSupportedChecksumType(type)) {
    // format.cc:385-388 (footer decode rejects unknown types)
    return Status::Corruption("Corrupt or unsupported checksum type: " +
                              std::to_string(static_cast<int>(type)));
  }
  if (b.n == 0) return Status::OK();
  if (file_offsets.size() != b.n) return Status::InvalidArgument("file_offsets.size() != n");
  // PERF_TIMER_GUARD(block_checksum_time) (reader_common.cc:29), per batch
  struct Timer {
    uint64_t* acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~Timer() {
      *acc += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                        std::chrono::steady_clock::now() - t0)
                                        .count());
    }
  } timer{&stats_.block_checksum_time};
  Status s = EnsureScratch(b.n);
  if (!s.ok()) return s;
  hipStream_t st = static_cast<hipStream_t>(stream_);
  const uint32_t* mods = nullptr;
  std::vector<uint32_t> hmods;
  if (base_context_checksum != 0) {  // format_version >= 6
    hmods.resize(b.n);
    for (uint64_t i = 0; i < b.n; ++i)
      hmods[i] = ChecksumModifierForContext(base_context_checksum, file_offsets[i]);
    s = FromHip(hipMemcpyAsync(d_mod_, hmods.data(), b.n * 4, hipMemcpyHostToDevice, st),
                "hipMemcpyAsync");
    if (!s.ok()) return s;
    mods = d_mod_;
  }
  s = FromHip(hipMemsetAsync(d_bad_, 0, sizeof(*d_bad_), st), "hipMemsetAsync");
  if (!s.ok()) return s;
  int rc = forst_block_verify_batch(type, b.base, b.base_len, b.offsets, b.sizes, mods,
                                    d_computed_, d_stored_, d_ok_, d_bad_, b.n, stream_);
  if (rc != FORST_OK) return FromRc(rc);
  unsigned long long bad = 0;
  s = FromHip(hipMemcpyAsync(&bad, d_bad_, sizeof(bad), hipMemcpyDeviceToHost, st), "hipMemcpy");
  if (s.ok()) s = FromHip(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (!s.ok()) return s;
  stats_.block_checksum_compute_count += b.n;
  if (bad == 0) return Status::OK();
  stats_.block_checksum_mismatch_count += bad;
  std::vector<uint8_t> ok(b.n);
  std::vector<uint32_t> computed(b.n), stored(b.n), sizes(b.n);
  s = FromHip(hipMemcpy(ok.data(), d_ok_, b.n, hipMemcpyDeviceToHost), "hipMemcpy");
  if (s.ok()) s = FromHip(hipMemcpy(computed.data(), d_computed_, b.n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
  if (s.ok()) s = FromHip(hipMemcpy(stored.data(), d_stored_, b.n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
  if (s.ok()) s = FromHip(hipMemcpy(sizes.data(), b.sizes, b.n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
  if (!s.ok()) return s;
  Status first = Status::OK();
  for (uint64_t i = 0; i < b.n; ++i) {
    if (ok[i]) continue;
    if (failed) failed->push_back(i);
    if (first.ok()) {
      uint32_t st_v = stored[i], co_v = computed[i];
      if (type == kCRC32c) {  // reader_common.cc:50-54
        st_v = crc32c::Unmask(st_v);
        co_v = crc32c::Unmask(co_v);
      }
      const uint32_t modifier = ChecksumModifierForContext(base_context_checksum, file_offsets[i]);
      first = Status::Corruption(BlockChecksumMismatchMessage(
          type, st_v, co_v, modifier != 0, file_name, file_offsets[i], sizes[i]));
    }
  }
  return first;
}

}  // namespace forst_gpu
