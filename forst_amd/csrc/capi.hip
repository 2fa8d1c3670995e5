// forst_amd/csrc/capi.hip -- the C ABI (include/forst_checksum.h).
//
// Argument validation, per-device info cache and dispatch to the kernel
// launchers.  Scratch comes from a stream-ordered per-device pool
// (hipMallocFromPoolAsync / hipFreeAsync).  The block, raw-hash, combine, KV
// and WAL-writer entry points never copy to the host or synchronise, so they
// can be captured into hipGraphs (cdna_hip_programming.md Guideline 9);
// forst_wal_verify_batch, forst_wal_record_xxh3_batch and forst_wal_recover_batch
// read a record count back (one stream synchronisation each) and cannot be.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/forst_checksum.h"
#include "engine.h"

#define FORST_API extern "C" __attribute__((visibility("default")))

namespace forst {
namespace {

thread_local std::string g_last_error;
thread_local const char* g_last_kernel = "";
thread_local std::string g_last_kernel_buf;

constexpr int kMaxDevices = 64;
DeviceInfo g_info[kMaxDevices];
std::once_flag g_once[kMaxDevices];

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return FORST_OK;
  return set_error(FORST_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

const DeviceInfo& device_info() {
  static DeviceInfo none{-1, 0, false};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices)
    return none;
  std::call_once(g_once[dev], [dev] {
    DeviceInfo& d = g_info[dev];
    d.device = dev;
    d.num_cus = 0;
    d.ok = false;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) {
      d.num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 1;
      d.ok = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    }
  });
  return g_info[dev];
}

namespace {
std::once_flag g_pool_once[kMaxDevices];
hipMemPool_t g_pool[kMaxDevices];
hipError_t g_pool_err[kMaxDevices];
}  // namespace

hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t stream) {
  const int dev = device_info().device;
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::call_once(g_pool_once[dev], [dev] {
    hipMemPoolProps props;
    std::memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    g_pool_err[dev] = hipMemPoolCreate(&g_pool[dev], &props);
    if (g_pool_err[dev] == hipSuccess) {
      uint64_t keep = UINT64_MAX;  // freed blocks stay in the pool for the next call
      g_pool_err[dev] = hipMemPoolSetAttribute(g_pool[dev], hipMemPoolAttrReleaseThreshold, &keep);
    }
  });
  if (g_pool_err[dev] != hipSuccess) return g_pool_err[dev];
  return hipMallocFromPoolAsync(p, bytes ? bytes : 16, g_pool[dev], stream);
}

hipError_t scratch_free(void* p, hipStream_t stream) { return p ? hipFreeAsync(p, stream) : hipSuccess; }

// ---- auxiliary streams (engine.h AuxStream) --------------------------------
// One pool per device, shared by every host thread: a call takes an idle
// entry (or creates one), forks its second branch onto it and gives it back
// before returning, so the number of streams is bounded by the calls in
// flight at once, not by the threads that ever called (ForSt calls from JNI
// and pool threads that come and go).  forst_host_context_trim destroys the
// idle ones.
namespace {
std::mutex g_aux_mu;
std::vector<AuxStream*> g_aux_idle[kMaxDevices];
uint32_t g_aux_live = 0;  // created and not destroyed

int stream_device(hipStream_t st) {
  int dev = -1;
  if (st != nullptr && hipStreamGetDevice(st, &dev) == hipSuccess && dev >= 0) return dev;
  (void)hipGetLastError();
  return hipGetDevice(&dev) == hipSuccess ? dev : -1;
}
}  // namespace

AuxStream* aux_acquire(hipStream_t st) {
  const int dev = stream_device(st);
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  {
    std::lock_guard<std::mutex> g(g_aux_mu);
    auto& idle = g_aux_idle[dev];
    if (!idle.empty()) {
      AuxStream* a = idle.back();
      idle.pop_back();
      return a;
    }
  }
  // created on the stream's device (the caller's current device restored)
  int cur = -1;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  if (have_cur && cur != dev && hipSetDevice(dev) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  AuxStream* a = new AuxStream{nullptr, nullptr, nullptr, dev};
  if (hipStreamCreateWithFlags(&a->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&a->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&a->join, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    if (a->join) (void)hipEventDestroy(a->join);
    if (a->fork) (void)hipEventDestroy(a->fork);
    if (a->s) (void)hipStreamDestroy(a->s);
    delete a;
    a = nullptr;
  }
  if (have_cur && cur != dev) (void)hipSetDevice(cur);
  if (a) {
    std::lock_guard<std::mutex> g(g_aux_mu);
    ++g_aux_live;
  }
  return a;
}

void aux_release(AuxStream* a) {
  if (!a) return;
  std::lock_guard<std::mutex> g(g_aux_mu);
  g_aux_idle[a->device].push_back(a);
}

void aux_pool_trim() {
  std::vector<AuxStream*> gone;
  {
    std::lock_guard<std::mutex> g(g_aux_mu);
    for (auto& idle : g_aux_idle) {
      gone.insert(gone.end(), idle.begin(), idle.end());
      idle.clear();
    }
    g_aux_live -= static_cast<uint32_t>(gone.size());
  }
  for (AuxStream* a : gone) {
    // (work still queued on the stream completes before its resources go)
    (void)hipStreamSynchronize(a->s);
    (void)hipEventDestroy(a->join);
    (void)hipEventDestroy(a->fork);
    (void)hipStreamDestroy(a->s);
    delete a;
  }
  (void)hipGetLastError();
}

void aux_pool_stats(uint32_t* live, uint32_t* idle) {
  std::lock_guard<std::mutex> g(g_aux_mu);
  uint32_t n = 0;
  for (auto& v : g_aux_idle) n += static_cast<uint32_t>(v.size());
  if (live) *live = g_aux_live;
  if (idle) *idle = n;
}

#ifdef FORST_DIAG
const char* diag_env(const char* name) {
  const char* v = std::getenv(name);
  return v ? v : "";
}
#endif

hipError_t feed_setup(BlockArgs& a, uint64_t nw, hipStream_t stream) {
  // half the descriptors as equal static shares (no claims while the
  // machine fills), the rest in claimed 64-descriptor chunks that absorb
  // the byte imbalance of mixed block sizes
  a.ticket = nullptr;
#ifdef FORST_DIAG
  const std::string mode = diag_env("FORST_FEED");
  if (mode == "static") {  // one contiguous share per wave (A/B reference)
    a.share1 = (a.n + 64 * nw - 1) / (64 * nw) * 64;
    if (a.share1 * nw > a.n) a.share1 = a.n / (64 * nw) * 64;
    return hipSuccess;
  }
  if (mode == "rr") {  // round-robin chunks, no counter (A/B reference)
    a.share1 = a.n / (2 * 64 * nw) * 64;
    return hipSuccess;
  }
  if (mode == "rr0") {  // round-robin chunks only: every wave sweeps the buffer in step
    a.share1 = 0;
    return hipSuccess;
  }
#endif
  a.share1 = a.n / (2 * 64 * nw) * 64;
  void* p = nullptr;
  hipError_t e = scratch_alloc(&p, 64 * sizeof(unsigned long long), stream);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(p, 0, sizeof(unsigned long long), stream);
  if (e != hipSuccess) {
    (void)scratch_free(p, stream);
    return e;
  }
  a.ticket = static_cast<unsigned long long*>(p);
  return hipSuccess;
}

namespace {

int check_device() {
  const DeviceInfo& d = device_info();
  if (d.device < 0) return set_error(FORST_ENODEV, "no HIP device");
  if (!d.ok)
    return set_error(FORST_ENODEV,
                     "device is not gfx950 (MI355X); this engine ships gfx950 code only");
  return FORST_OK;
}

bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3) == 0; }

int check_block_args(const uint8_t* base, const uint64_t* offsets, const uint32_t* sizes,
                     uint64_t n) {
  if (n == 0) return FORST_OK;
  if (!base || !offsets || !sizes)
    return set_error(FORST_EINVAL, "base/offsets/sizes must be non-null");
  if (!aligned4(base)) return set_error(FORST_EINVAL, "base must be 4-byte aligned");
  return FORST_OK;
}

// trailer bytes [type][LE32 out] at each block end (split write side: the
// streaming kernel runs in compute mode, the in-place writes come after it)
__global__ void __launch_bounds__(256) trailer_scatter_kernel(BlockArgs a) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t off = a.offsets[i];
  const uint32_t n = a.sizes[i];
  if (off > a.base_len || uint64_t(n) + 5 > a.base_len - off) return;
  uint8_t* p = a.base_w + off + n;
  const uint32_t v = a.out32[i];
  p[0] = a.last_bytes[i];
  p[1] = static_cast<uint8_t>(v);
  p[2] = static_cast<uint8_t>(v >> 8);
  p[3] = static_cast<uint8_t>(v >> 16);
  p[4] = static_cast<uint8_t>(v >> 24);
}

hipError_t launch_blocks(int type, int mode, const BlockArgs& a, hipStream_t s);

int dispatch_blocks(int type, int mode, const BlockArgs& a, void* stream) {
  int rc = check_device();
  if (rc) return rc;
  if (type < FORST_kNoChecksum || type > FORST_kXXH3)  // options_helper.h:34
    return set_error(FORST_EINVAL, "unknown ChecksumType " + std::to_string(type));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // Write side: the 5 trailer bytes per block are partial writes into 64 B
  // memory sectors shared with block data (a read-modify-write below the
  // L2).  Stored by the streaming kernel as rows finish they cost 16 % of
  // the pass (C2, round 1), split off into a second, tiny kernel 8 %.  Since
  // round 4 the rows kernels stage a workgroup's results in LDS and write
  // them after their loop, which beats the split form (C2 write side -1.4 %,
  // NS16X -0.2 %, profiles/ab_r04/trailer_fused_staged.log);
  // FORST_TRAILER_SPLIT=1 builds the split form.
  // (diagnostics build: FORST_TRAILER=fused|split at run time)
#ifndef FORST_TRAILER_SPLIT
#define FORST_TRAILER_SPLIT 0
#endif
  bool split = FORST_TRAILER_SPLIT;
#ifdef FORST_DIAG
  if (*diag_env("FORST_TRAILER")) split = std::string(diag_env("FORST_TRAILER")) != "fused";
#endif
  if (mode == kModeTrailer && split && a.n) {
    BlockArgs c = a;
    void* tmp = nullptr;
    hipError_t e = hipSuccess;
    if (!c.out32) {
      e = scratch_alloc(&tmp, 4 * a.n, s);
      c.out32 = static_cast<uint32_t*>(tmp);
    }
    if (e == hipSuccess) e = launch_blocks(type, kModeCompute, c, s);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(trailer_scatter_kernel, dim3(static_cast<uint32_t>((a.n + 255) / 256)),
                         dim3(256), 0, s, c);
      e = hipGetLastError();
      g_last_kernel_buf = std::string(g_last_kernel) + "+trailer_scatter_kernel";
      g_last_kernel = g_last_kernel_buf.c_str();
    }
    if (tmp) {
      const hipError_t f = scratch_free(tmp, s);
      if (e == hipSuccess) e = f;
    }
    return hip_status(e, "kernel launch");
  }
  return hip_status(launch_blocks(type, mode, a, s), "kernel launch");
}

hipError_t launch_blocks(int type, int mode, const BlockArgs& a, hipStream_t s) {
  hipError_t e;
  switch (type) {
    case FORST_kCRC32c:
      e = launch_crc32c_blocks(mode, a, s, &g_last_kernel);
      break;
    case FORST_kXXH3:
      e = launch_xxh3_blocks(mode, a, s, &g_last_kernel);
      break;
    case FORST_kNoChecksum:
      e = launch_noop_blocks(mode, a, s, &g_last_kernel);
      break;
    case FORST_kxxHash:
    case FORST_kxxHash64:
      e = launch_xxhash_legacy_blocks(type == FORST_kxxHash64, mode, a, s, &g_last_kernel);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return e;
}

}  // namespace
}  // namespace forst

using namespace forst;

FORST_API const char* forst_version(void) { return "forst-mi355x 0.1.0 (gfx950)"; }
FORST_API const char* forst_last_error(void) { return g_last_error.c_str(); }
FORST_API const char* forst_last_kernel(void) { return g_last_kernel; }

FORST_API int forst_init_device(void) { return check_device(); }

FORST_API int forst_aux_stream_stats(uint32_t* live, uint32_t* idle) {
  aux_pool_stats(live, idle);
  return FORST_OK;
}

FORST_API int forst_block_checksum_batch(int checksum_type, const uint8_t* base,
                                         uint64_t base_len, const uint64_t* offsets,
                                         const uint32_t* sizes, const uint8_t* last_bytes,
                                         const uint32_t* modifiers, uint32_t* out,
                                         uint64_t n_blocks, void* stream) {
  int rc = check_block_args(base, offsets, sizes, n_blocks);
  if (rc) return rc;
  if (n_blocks && !out) return set_error(FORST_EINVAL, "out must be non-null");
  BlockArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.offsets = offsets;
  a.sizes = sizes;
  a.last_bytes = last_bytes;
  a.modifiers = modifiers;
  a.out32 = out;
  a.n = n_blocks;
  return dispatch_blocks(checksum_type, kModeCompute, a, stream);
}

FORST_API int forst_block_trailer_batch(int checksum_type, uint8_t* base, uint64_t base_len,
                                        const uint64_t* offsets, const uint32_t* sizes,
                                        const uint8_t* last_bytes, const uint32_t* modifiers,
                                        uint32_t* out, uint64_t n_blocks, void* stream) {
  int rc = check_block_args(base, offsets, sizes, n_blocks);
  if (rc) return rc;
  if (n_blocks && !last_bytes)
    return set_error(FORST_EINVAL, "trailer mode needs last_bytes (compression types)");
  BlockArgs a{};
  a.base = base;
  a.base_w = base;
  a.base_len = base_len;
  a.offsets = offsets;
  a.sizes = sizes;
  a.last_bytes = last_bytes;
  a.modifiers = modifiers;
  a.out32 = out;
  a.n = n_blocks;
  return dispatch_blocks(checksum_type, kModeTrailer, a, stream);
}

FORST_API int forst_block_verify_batch(int checksum_type, const uint8_t* base,
                                       uint64_t base_len, const uint64_t* offsets,
                                       const uint32_t* sizes, const uint32_t* modifiers,
                                       uint32_t* computed, uint32_t* stored, uint8_t* ok,
                                       unsigned long long* mismatches, uint64_t n_blocks,
                                       void* stream) {
  int rc = check_block_args(base, offsets, sizes, n_blocks);
  if (rc) return rc;
  BlockArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.offsets = offsets;
  a.sizes = sizes;
  a.modifiers = modifiers;
  a.out32 = computed;
  a.stored_out = stored;
  a.ok_out = ok;
  a.mismatches = mismatches;
  a.n = n_blocks;
  return dispatch_blocks(checksum_type, kModeVerify, a, stream);
}

FORST_API int forst_crc32c_batch(const uint8_t* base, uint64_t base_len,
                                 const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* init_crcs, uint32_t* out,
                                 uint64_t n_buffers, void* stream) {
  int rc = check_block_args(base, offsets, lengths, n_buffers);
  if (rc) return rc;
  if (n_buffers && !out) return set_error(FORST_EINVAL, "out must be non-null");
  BlockArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.offsets = offsets;
  a.sizes = lengths;
  a.init_crcs = init_crcs;
  a.out32 = out;
  a.n = n_buffers;
  return dispatch_blocks(FORST_kCRC32c, kModeRaw, a, stream);
}

FORST_API int forst_wal_record_xxh3_batch(const uint8_t* log, uint64_t log_len,
                                          const uint64_t* header_offsets, uint64_t n_phys,
                                          uint64_t* hashes, uint64_t* first_phys,
                                          uint64_t* n_logical, void* stream) {
  if (!n_logical) return set_error(FORST_EINVAL, "n_logical must be non-null");
  *n_logical = 0;
  if (n_phys == 0) return FORST_OK;
  if (!log || !aligned4(log) || !header_offsets || !hashes)
    return set_error(FORST_EINVAL, "log/header_offsets/hashes must be non-null, log 4-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  WalArgs a{};
  a.log = log;
  a.log_len = log_len;
  a.header_offsets = header_offsets;
  a.n_records = n_phys;
  return hip_status(launch_wal_record_xxh3(a, hashes, first_phys, n_logical,
                                           static_cast<hipStream_t>(stream), &g_last_kernel),
                    "wal_record_xxh3 launch");
}

FORST_API int forst_wal_recover_batch(const uint8_t* log, uint64_t log_len, uint32_t log_number,
                                     int wal_recovery_mode, forst_wal_records records,
                                     uint64_t record_capacity, forst_wal_reports reports,
                                     uint64_t report_capacity, forst_wal_recover_result* result,
                                     void* stream) {
  if (!result) return set_error(FORST_EINVAL, "result must be non-null");
  std::memset(result, 0, sizeof(*result));
  if (log_len && (!log || !aligned4(log)))
    return set_error(FORST_EINVAL, "log must be non-null, 4-byte aligned");
  if (wal_recovery_mode < 0 || wal_recovery_mode > 3)
    return set_error(FORST_EINVAL, "unknown WALRecoveryMode " + std::to_string(wal_recovery_mode));
  int rc = check_device();
  if (rc) return rc;
  rc = hip_status(launch_wal_recover(log, log_len, log_number, wal_recovery_mode, records,
                                     record_capacity, reports, report_capacity, result,
                                     static_cast<hipStream_t>(stream), &g_last_kernel),
                  "wal_recover launch");
  if (rc == FORST_OK && result->unsupported)
    return set_error(FORST_EUNSUPPORTED,
                     "WAL compression: a kSetCompressionType record names kZSTD");
  return rc;
}

FORST_API int forst_crc32c_buffer(const uint8_t* base, uint64_t len, uint32_t init, uint32_t* out,
                                  void* stream) {
  if (!out || (len && (!base || !aligned4(base))))
    return set_error(FORST_EINVAL, "out must be non-null, base non-null and 4-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  return hip_status(launch_crc32c_buffer(base, len, init, out, static_cast<hipStream_t>(stream),
                                         &g_last_kernel),
                    "crc32c_buffer launch");
}

FORST_API int forst_crc32c_combine_batch(const uint32_t* crc1, const uint32_t* crc2,
                                         const uint64_t* len2, uint32_t* out, uint64_t n,
                                         void* stream) {
  if (n == 0) return FORST_OK;
  if (!crc1 || !crc2 || !len2 || !out)
    return set_error(FORST_EINVAL, "crc1/crc2/len2/out must be non-null");
  int rc = check_device();
  if (rc) return rc;
  return hip_status(launch_crc32c_combine_batch(crc1, crc2, len2, out, n,
                                                static_cast<hipStream_t>(stream), &g_last_kernel),
                    "crc32c_combine launch");
}

FORST_API int forst_xxh3_64_batch(const uint8_t* base, uint64_t base_len,
                                  const uint64_t* offsets, const uint32_t* lengths,
                                  uint64_t* out, uint64_t n_buffers, void* stream) {
  int rc = check_block_args(base, offsets, lengths, n_buffers);
  if (rc) return rc;
  if (n_buffers && !out) return set_error(FORST_EINVAL, "out must be non-null");
  BlockArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.offsets = offsets;
  a.sizes = lengths;
  a.out64 = out;
  a.n = n_buffers;
  return dispatch_blocks(FORST_kXXH3, kModeRaw, a, stream);
}

FORST_API int forst_wal_verify_batch(const uint8_t* log, uint64_t log_len, uint64_t first_block,
                                     uint64_t n_blocks, uint32_t log_number, uint8_t* status_out,
                                     uint32_t* nrec_out, uint32_t* fail_off_out,
                                     unsigned long long* bad_blocks, void* stream) {
  if (n_blocks == 0) return FORST_OK;
  if (!log || !aligned4(log)) return set_error(FORST_EINVAL, "log must be non-null, 4-byte aligned");
  const uint64_t total_blocks = (log_len + 32767) / 32768;
  if (first_block > total_blocks || n_blocks > total_blocks - first_block)
    return set_error(FORST_EINVAL, "log block range outside log_len");
  int rc = check_device();
  if (rc) return rc;
  WalArgs a{};
  a.log = log;
  a.log_len = log_len;
  a.first_block = first_block;
  a.n_blocks = n_blocks;
  a.log_number = log_number;
  a.status_out = status_out;
  a.nrec_out = nrec_out;
  a.fail_off_out = fail_off_out;
  a.bad_blocks = bad_blocks;
  return hip_status(launch_wal_verify(a, static_cast<hipStream_t>(stream), &g_last_kernel),
                    "wal_verify launch");
}

FORST_API int forst_wal_record_crc_batch(uint8_t* log, uint64_t log_len,
                                         const uint64_t* header_offsets, uint64_t n_records,
                                         int write_in_place, uint32_t* crc_out, void* stream) {
  if (n_records == 0) return FORST_OK;
  if (!log || !aligned4(log) || !header_offsets)
    return set_error(FORST_EINVAL, "log/header_offsets must be non-null, log 4-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  WalArgs a{};
  a.log = log;
  a.log_w = log;
  a.log_len = log_len;
  a.header_offsets = header_offsets;
  a.n_records = n_records;
  a.write_in_place = write_in_place;
  a.crc_out = crc_out;
  return hip_status(launch_wal_record_crc(a, static_cast<hipStream_t>(stream), &g_last_kernel),
                    "wal_record_crc launch");
}

FORST_API int forst_wal_record_crc_lengths(uint8_t* log, uint64_t log_len,
                                           const uint64_t* header_offsets,
                                           const uint32_t* payload_lengths, uint64_t n_records,
                                           int recyclable, int write_in_place, uint32_t* crc_out,
                                           void* stream) {
  if (n_records == 0) return FORST_OK;
  if (!log || !aligned4(log) || !header_offsets || !payload_lengths)
    return set_error(FORST_EINVAL,
                     "log/header_offsets/payload_lengths must be non-null, log 4-byte aligned");
  int rc = check_device();
  if (rc) return rc;
  WalArgs a{};
  a.log = log;
  a.log_w = log;
  a.log_len = log_len;
  a.header_offsets = header_offsets;
  a.payload_lengths = payload_lengths;
  a.recyclable = recyclable ? 1 : 0;
  a.n_records = n_records;
  a.write_in_place = write_in_place;
  a.crc_out = crc_out;
  return hip_status(launch_wal_record_crc(a, static_cast<hipStream_t>(stream), &g_last_kernel),
                    "wal_record_crc_lengths launch");
}

namespace forst {
namespace {
int dispatch_kv(int mode, const KvArgs& a, void* stream) {
  if (a.n == 0) return FORST_OK;
  if (!a.base || !a.key_off || !a.key_len)
    return set_error(FORST_EINVAL, "base/offsets/lengths must be non-null");
  int rc = check_device();
  if (rc) return rc;
  return hip_status(launch_kv(mode, a, static_cast<hipStream_t>(stream), &g_last_kernel),
                    "kv launch");
}
}  // namespace
}  // namespace forst

FORST_API int forst_hash64_batch(const uint8_t* base, uint64_t base_len, const uint64_t* offsets,
                                 const uint32_t* lengths, const uint64_t* seeds, uint64_t seed,
                                 uint64_t* out, uint64_t n, void* stream) {
  if (n && !out) return set_error(FORST_EINVAL, "out must be non-null");
  KvArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.key_off = offsets;
  a.key_len = lengths;
  a.seeds = seeds;
  a.seed = seed;
  a.out = out;
  a.n = n;
  return dispatch_kv(kKvHash, a, stream);
}

FORST_API int forst_kv_protect_batch(const uint8_t* base, uint64_t base_len,
                                     const uint64_t* key_offsets, const uint32_t* key_sizes,
                                     const uint64_t* value_offsets, const uint32_t* value_sizes,
                                     const uint8_t* op_types, const uint64_t* seqnos,
                                     const uint32_t* cf_ids, uint64_t* out, uint64_t n,
                                     void* stream) {
  if (n && (!out || !value_offsets || !value_sizes))
    return set_error(FORST_EINVAL, "out/value_offsets/value_sizes must be non-null");
  KvArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.key_off = key_offsets;
  a.key_len = key_sizes;
  a.val_off = value_offsets;
  a.val_len = value_sizes;
  a.ops = op_types;
  a.seqs = seqnos;
  a.cfs = cf_ids;
  a.out = out;
  a.n = n;
  return dispatch_kv(kKvProtect, a, stream);
}

FORST_API int forst_kv_verify_batch(const uint8_t* base, uint64_t base_len,
                                    const uint64_t* key_offsets, const uint32_t* key_sizes,
                                    const uint64_t* value_offsets, const uint32_t* value_sizes,
                                    const uint8_t* op_types, const uint64_t* seqnos,
                                    const uint32_t* cf_ids, uint32_t protection_bytes,
                                    const uint64_t* checksum_offsets, uint64_t* computed,
                                    uint8_t* ok, unsigned long long* mismatches, uint64_t n,
                                    void* stream) {
  if (n && (!value_offsets || !value_sizes || !checksum_offsets))
    return set_error(FORST_EINVAL, "value/checksum arrays must be non-null");
  // kv_checksum.h:97-133 supports 1, 2, 4, 8 (advanced_options.h:1227)
  if (protection_bytes != 1 && protection_bytes != 2 && protection_bytes != 4 &&
      protection_bytes != 8)
    return set_error(FORST_EINVAL, "protection_bytes must be 1, 2, 4 or 8");
  KvArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.key_off = key_offsets;
  a.key_len = key_sizes;
  a.val_off = value_offsets;
  a.val_len = value_sizes;
  a.ops = op_types;
  a.seqs = seqnos;
  a.cfs = cf_ids;
  a.prot_bytes = protection_bytes;
  a.chk_off = checksum_offsets;
  a.out = computed;
  a.ok = ok;
  a.mismatches = mismatches;
  a.n = n;
  return dispatch_kv(kKvVerify, a, stream);
}

namespace {
int mem_args(KvArgs& a, const uint8_t* base, uint64_t base_len, const uint64_t* entry_offsets,
             uint32_t protection_bytes, uint64_t n) {
  if (n && !entry_offsets) return set_error(FORST_EINVAL, "entry_offsets must be non-null");
  if (protection_bytes != 1 && protection_bytes != 2 && protection_bytes != 4 &&
      protection_bytes != 8)
    return set_error(FORST_EINVAL, "protection_bytes must be 1, 2, 4 or 8");
  a.base = base;
  a.base_len = base_len;
  a.key_off = entry_offsets;
  a.prot_bytes = protection_bytes;
  a.n = n;
  return FORST_OK;
}
int dispatch_mem(int mode, const KvArgs& a, void* stream) {
  if (a.n == 0) return FORST_OK;
  if (!a.base) return set_error(FORST_EINVAL, "base must be non-null");
  int rc = check_device();
  if (rc) return rc;
  return hip_status(launch_kv(mode, a, static_cast<hipStream_t>(stream), &g_last_kernel),
                    "memtable kv launch");
}
}  // namespace

FORST_API int forst_memtable_verify_batch(const uint8_t* base, uint64_t base_len,
                                          const uint64_t* entry_offsets, uint64_t n,
                                          uint32_t protection_bytes, uint64_t* computed,
                                          uint8_t* status, unsigned long long* mismatches,
                                          void* stream) {
  KvArgs a{};
  int rc = mem_args(a, base, base_len, entry_offsets, protection_bytes, n);
  if (rc) return rc;
  a.out = computed;
  a.status = status;
  a.mismatches = mismatches;
  return dispatch_mem(kKvMemVerify, a, stream);
}

FORST_API int forst_memtable_protect_batch(uint8_t* base, uint64_t base_len,
                                           const uint64_t* entry_offsets, uint64_t n,
                                           uint32_t protection_bytes, int write_in_place,
                                           uint64_t* out, uint8_t* status, void* stream) {
  KvArgs a{};
  int rc = mem_args(a, base, base_len, entry_offsets, protection_bytes, n);
  if (rc) return rc;
  a.out = out;
  a.status = status;
  a.write_in_place = write_in_place ? 1 : 0;
  return dispatch_mem(kKvMemProtect, a, stream);
}

FORST_API int forst_write_batch_protect_batch(const uint8_t* base, uint64_t base_len,
                                              const uint64_t* rep_offsets,
                                              const uint32_t* rep_sizes, uint64_t n_reps,
                                              uint64_t* first_entry, uint64_t* prot,
                                              uint64_t capacity, uint8_t* status,
                                              uint32_t* n_protected, uint64_t* n_total,
                                              void* stream) {
  if (n_total) *n_total = 0;
  if (!first_entry) return set_error(FORST_EINVAL, "first_entry must be non-null");
  if (n_reps && (!base || !rep_offsets || !rep_sizes))
    return set_error(FORST_EINVAL, "base/rep_offsets/rep_sizes must be non-null");
  if (capacity && !prot) return set_error(FORST_EINVAL, "prot must be non-null");
  int rc = check_device();
  if (rc) return rc;
  WbArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.offsets = rep_offsets;
  a.sizes = rep_sizes;
  a.n = n_reps;
  a.first_entry = first_entry;
  a.prot = prot;
  a.capacity = capacity;
  a.status = status;
  a.n_protected = n_protected;
  uint64_t total = 0;
  const hipError_t e = launch_write_batch_protect(a, static_cast<hipStream_t>(stream), &total,
                                                  &g_last_kernel);
  if (n_total) *n_total = total;
  if (e == hipErrorInvalidValue && total > capacity)
    return set_error(FORST_EINVAL, "capacity " + std::to_string(capacity) + " < " +
                                       std::to_string(total) + " protection slots");
  return hip_status(e, "write_batch_protect");
}

FORST_API int forst_block_kv_checksum_batch(const uint8_t* base, uint64_t base_len,
                                            const uint64_t* block_offsets,
                                            const uint32_t* block_sizes, const uint8_t* kinds,
                                            uint64_t n_blocks, uint32_t protection_bytes,
                                            uint64_t* first_key, uint8_t* kv_checksums,
                                            uint64_t* prot, uint64_t capacity, uint8_t* status,
                                            uint64_t* n_total, void* stream) {
  if (n_total) *n_total = 0;
  if (!first_key) return set_error(FORST_EINVAL, "first_key must be non-null");
  if (n_blocks && (!base || !block_offsets || !block_sizes || !kinds))
    return set_error(FORST_EINVAL, "base/block_offsets/block_sizes/kinds must be non-null");
  if (protection_bytes != 1 && protection_bytes != 2 && protection_bytes != 4 &&
      protection_bytes != 8)
    return set_error(FORST_EINVAL, "protection_bytes must be 1, 2, 4 or 8");
  if (capacity && !kv_checksums)
    return set_error(FORST_EINVAL, "kv_checksums must be non-null");
  int rc = check_device();
  if (rc) return rc;
  BlkArgs a{};
  a.base = base;
  a.base_len = base_len;
  a.offsets = block_offsets;
  a.sizes = block_sizes;
  a.kinds = kinds;
  a.n = n_blocks;
  a.prot_bytes = protection_bytes;
  a.first_key = first_key;
  a.kv_checksums = kv_checksums;
  a.prot = prot;
  a.capacity = capacity;
  a.status = status;
  uint64_t total = 0;
  const hipError_t e =
      launch_block_kv_checksum(a, static_cast<hipStream_t>(stream), &total, &g_last_kernel);
  if (n_total) *n_total = total;
  if (e == hipErrorInvalidValue && total > capacity)
    return set_error(FORST_EINVAL, "capacity " + std::to_string(capacity) + " < " +
                                       std::to_string(total) + " keys");
  return hip_status(e, "block_kv_checksum");
}

FORST_API int forst_fill_stream(uint8_t* dev, uint64_t start, uint64_t n, uint64_t seed,
                                void* stream) {
  if (n == 0) return FORST_OK;
  if (!dev || (reinterpret_cast<uintptr_t>(dev) & 7))
    return set_error(FORST_EINVAL, "fill_stream needs an 8-byte aligned dev pointer");
  int rc = check_device();
  if (rc) return rc;
  return hip_status(launch_fill_stream(dev, start, n, seed, static_cast<hipStream_t>(stream)),
                    "fill_stream launch");
}
