// forst_amd/csrc/host_batch.cc -- host-memory batches over the GPUs of one
// process (SURVEY.md §8e / §8d "end-to-end").
//
// ForSt is one process: DB::VerifyChecksum (db/db_impl/db_impl.cc:6254) walks
// every live SST file, and flush / compaction threads hand blocks that live in
// host memory (the table builder's buffer, a FilePrefetchBuffer, an mmap'd
// file -- env/io_posix.cc:958).  These entry points take such a host batch and
// a device list, cut the blocks into contiguous byte-balanced ranges (one per
// device, forst_partition_bytes) and give every device its own host thread,
// HIP stream and pinned staging: the thread streams its range through two
// device windows (copy of window k+1 overlaps the kernel on window k), runs
// the block kernels on them and brings back 4-5 B per block.  No data crosses
// between devices; the only join is the host threads'.
//
// Host memory that is pinned or registered (hipHostRegister, e.g. an mmap'd
// SST file: forst_host_register) is copied by DMA straight from the caller's
// pages; pageable memory is first memcpy'd into the thread's pinned staging.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/forst_checksum.h"

namespace {

thread_local std::string g_host_err;

int fail(int code, const std::string& m) {
  g_host_err = m;
  return code;
}

constexpr uint64_t kWindowBytes = 64ull << 20;  // device window per copy (two per device)
constexpr uint32_t kTrailer = 5;               // block_based_table_reader.h:75

// [cuts[p], cuts[p+1]) = part p: contiguous, byte-balanced (part p starts at
// the first block whose byte prefix reaches p/parts of the total) -- the same
// rule as forst_amd/shard.py byte_ranges
void partition(const uint32_t* sizes, uint64_t n, uint32_t parts, uint64_t* cuts) {
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) total += sizes[i];
  cuts[0] = 0;
  uint64_t i = 0, prefix = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    const uint64_t target = static_cast<uint64_t>(
        (static_cast<unsigned __int128>(total) * p) / parts);
    while (i < n && prefix < target) prefix += sizes[i++];
    cuts[p] = i;
  }
  cuts[parts] = n;
  for (uint32_t p = 1; p <= parts; ++p) cuts[p] = std::max(cuts[p], cuts[p - 1]);
}

bool is_device_readable_host(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;  // pinned or registered
}

enum class Op { kVerify, kChecksum };

struct HostBatch {
  Op op;
  int type;
  const uint8_t* base;
  uint64_t base_len;
  const uint64_t* offsets;
  const uint32_t* sizes;
  const uint8_t* last_bytes;
  const uint32_t* modifiers;
  uint32_t* out;      // computed (verify) / checksums (compute)
  uint32_t* stored;   // verify, nullable
  uint8_t* ok;        // verify, nullable
};

// One device's share [lo, hi) of the blocks, in windows of at most
// kWindowBytes (a block larger than that gets a window of its own).
struct DeviceRun {
  int device = 0;
  uint64_t lo = 0, hi = 0;
  uint64_t mismatches = 0;
  int rc = FORST_OK;
  std::string err;
};

// bytes a block needs in host memory: payload + trailer (verify), payload +
// type byte (compute without last_bytes), payload (compute with last_bytes)
uint64_t block_end(const HostBatch& b, uint64_t i) {
  const uint32_t extra = b.op == Op::kVerify ? kTrailer : b.last_bytes ? 0 : 1;
  return b.offsets[i] + b.sizes[i] + extra;
}

void run_device(const HostBatch& b, bool direct, DeviceRun& r) {
  auto bail = [&](hipError_t e, const char* what) {
    r.rc = FORST_EHIP;
    r.err = std::string(what) + ": " + hipGetErrorString(e);
  };
  hipError_t e = hipSetDevice(r.device);
  if (e != hipSuccess) return bail(e, "hipSetDevice");
  if (r.hi <= r.lo) return;
  // windows: contiguous block runs whose bytes fit one device window
  std::vector<std::pair<uint64_t, uint64_t>> win;
  uint64_t max_bytes = 0, max_blocks = 0;
  for (uint64_t c0 = r.lo; c0 < r.hi;) {
    const uint64_t base0 = b.offsets[c0] & ~3ull;
    uint64_t c1 = c0 + 1;
    while (c1 < r.hi && block_end(b, c1) - base0 <= kWindowBytes && c1 - c0 < (1u << 20)) ++c1;
    uint64_t end = 0;
    for (uint64_t i = c0; i < c1; ++i) end = std::max(end, block_end(b, i));
    max_bytes = std::max(max_bytes, end - base0);
    max_blocks = std::max(max_blocks, c1 - c0);
    win.emplace_back(c0, c1);
    c0 = c1;
  }
  hipStream_t st;
  if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess)
    return bail(e, "hipStreamCreate");
  const uint64_t dbytes = (max_bytes + 255) & ~255ull;
  // per slot: device window + descriptors + outputs; pinned descriptors,
  // outputs and (pageable input only) the staged window
  struct Slot {
    uint8_t* d = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t *d_size = nullptr, *d_mod = nullptr, *d_out = nullptr, *d_st = nullptr;
    uint8_t *d_last = nullptr, *d_ok = nullptr;
    unsigned long long* d_bad = nullptr;
    uint8_t* h = nullptr;  // pinned staging (pageable input)
    uint64_t* h_off = nullptr;
    uint32_t *h_size = nullptr, *h_mod = nullptr, *h_out = nullptr, *h_st = nullptr;
    uint8_t *h_last = nullptr, *h_ok = nullptr;
    unsigned long long* h_bad = nullptr;
    hipEvent_t done;
    int64_t win = -1;  // window whose results are pending in this slot
  } slot[2];
  const uint64_t m = max_blocks;
  for (Slot& s : slot) {
    void* p = nullptr;
    if ((e = hipMalloc(&p, dbytes + m * 26 + 64)) != hipSuccess) return bail(e, "hipMalloc");
    s.d = static_cast<uint8_t*>(p);
    s.d_off = reinterpret_cast<uint64_t*>(s.d + dbytes);
    s.d_size = reinterpret_cast<uint32_t*>(s.d_off + m);
    s.d_mod = s.d_size + m;
    s.d_out = s.d_mod + m;
    s.d_st = s.d_out + m;
    s.d_bad = reinterpret_cast<unsigned long long*>(s.d_st + m);  // 24 m bytes in: aligned
    s.d_last = reinterpret_cast<uint8_t*>(s.d_bad + 1);
    s.d_ok = s.d_last + m;
    if ((e = hipHostMalloc(&p, m * 26 + 128 + (direct ? 0 : dbytes))) != hipSuccess)
      return bail(e, "hipHostMalloc");
    s.h_off = static_cast<uint64_t*>(p);
    s.h_size = reinterpret_cast<uint32_t*>(s.h_off + m);
    s.h_mod = s.h_size + m;
    s.h_out = s.h_mod + m;
    s.h_st = s.h_out + m;
    s.h_bad = reinterpret_cast<unsigned long long*>(s.h_st + m);
    s.h_last = reinterpret_cast<uint8_t*>(s.h_bad + 1);
    s.h_ok = s.h_last + m;
    s.h = direct ? nullptr : s.h_ok + m + 64 - ((reinterpret_cast<uintptr_t>(s.h_ok + m)) & 63);
    if ((e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
      return bail(e, "hipEventCreate");
  }
  auto collect = [&](Slot& s) -> bool {
    if (s.win < 0) return true;
    hipError_t w = hipEventSynchronize(s.done);
    if (w != hipSuccess) {
      bail(w, "hipEventSynchronize");
      return false;
    }
    const uint64_t c0 = win[s.win].first, c1 = win[s.win].second, k = c1 - c0;
    std::memcpy(b.out + c0, s.h_out, k * 4);
    if (b.op == Op::kVerify) {
      if (b.stored) std::memcpy(b.stored + c0, s.h_st, k * 4);
      if (b.ok) std::memcpy(b.ok + c0, s.h_ok, k);
      r.mismatches += *s.h_bad;
    }
    s.win = -1;
    return true;
  };
  for (uint64_t w = 0; w < win.size() && r.rc == FORST_OK; ++w) {
    Slot& s = slot[w & 1];
    if (!collect(s)) break;  // the slot's previous window is done: reuse it
    const uint64_t c0 = win[w].first, c1 = win[w].second, k = c1 - c0;
    const uint64_t base0 = b.offsets[c0] & ~3ull;
    uint64_t end = 0;
    for (uint64_t i = c0; i < c1; ++i) {
      end = std::max(end, block_end(b, i));
      s.h_off[i - c0] = b.offsets[i] - base0;
      s.h_size[i - c0] = b.sizes[i];
      if (b.modifiers) s.h_mod[i - c0] = b.modifiers[i];
      if (b.last_bytes) s.h_last[i - c0] = b.last_bytes[i];
    }
    const uint64_t nbytes = std::min(end, b.base_len) - base0;
    const uint8_t* src = b.base + base0;
    if (!direct) {
      std::memcpy(s.h, src, nbytes);
      src = s.h;
    }
    bool okc = (e = hipMemcpyAsync(s.d, src, nbytes, hipMemcpyHostToDevice, st)) == hipSuccess;
    okc = okc && (e = hipMemcpyAsync(s.d_off, s.h_off, k * 8, hipMemcpyHostToDevice, st)) == hipSuccess;
    okc = okc && (e = hipMemcpyAsync(s.d_size, s.h_size, k * 4, hipMemcpyHostToDevice, st)) == hipSuccess;
    if (okc && b.modifiers)
      okc = (e = hipMemcpyAsync(s.d_mod, s.h_mod, k * 4, hipMemcpyHostToDevice, st)) == hipSuccess;
    if (okc && b.last_bytes)
      okc = (e = hipMemcpyAsync(s.d_last, s.h_last, k, hipMemcpyHostToDevice, st)) == hipSuccess;
    if (!okc) {
      bail(e, "hipMemcpyAsync");
      break;
    }
    int rc;
    if (b.op == Op::kVerify) {
      okc = (e = hipMemsetAsync(s.d_bad, 0, 8, st)) == hipSuccess;
      rc = forst_block_verify_batch(b.type, s.d, nbytes, s.d_off, s.d_size,
                                    b.modifiers ? s.d_mod : nullptr, s.d_out, s.d_st, s.d_ok,
                                    s.d_bad, k, st);
    } else {
      rc = forst_block_checksum_batch(b.type, s.d, nbytes, s.d_off, s.d_size,
                                      b.last_bytes ? s.d_last : nullptr,
                                      b.modifiers ? s.d_mod : nullptr, s.d_out, k, st);
    }
    if (rc != FORST_OK) {
      r.rc = rc;
      r.err = forst_last_error();
      break;
    }
    okc = (e = hipMemcpyAsync(s.h_out, s.d_out, k * 4, hipMemcpyDeviceToHost, st)) == hipSuccess;
    if (okc && b.op == Op::kVerify) {
      okc = (e = hipMemcpyAsync(s.h_st, s.d_st, k * 4, hipMemcpyDeviceToHost, st)) == hipSuccess &&
            (e = hipMemcpyAsync(s.h_ok, s.d_ok, k, hipMemcpyDeviceToHost, st)) == hipSuccess &&
            (e = hipMemcpyAsync(s.h_bad, s.d_bad, 8, hipMemcpyDeviceToHost, st)) == hipSuccess;
    }
    if (okc) okc = (e = hipEventRecord(s.done, st)) == hipSuccess;
    if (!okc) {
      bail(e, "hipMemcpyAsync");
      break;
    }
    s.win = static_cast<int64_t>(w);
  }
  if (r.rc == FORST_OK) {
    collect(slot[0]);
    if (r.rc == FORST_OK) collect(slot[1]);
  }
  (void)hipStreamSynchronize(st);
  for (Slot& s : slot) {
    (void)hipFree(s.d);
    (void)hipHostFree(s.h_off);
    (void)hipEventDestroy(s.done);
  }
  (void)hipStreamDestroy(st);
}

int run_host_batch(const HostBatch& b, uint64_t n, const int* devices, int n_devices,
                   uint64_t* mismatches) {
  if (mismatches) *mismatches = 0;
  if (n == 0) return FORST_OK;
  if (!b.base || !b.offsets || !b.sizes || !b.out || !devices || n_devices <= 0)
    return fail(FORST_EINVAL, "host batch: null array or no device");
  if (b.type < FORST_kNoChecksum || b.type > FORST_kXXH3)  // options_helper.h:34
    return fail(FORST_EINVAL, "unknown ChecksumType " + std::to_string(b.type));
  for (uint64_t i = 0; i < n; ++i)
    if (b.offsets[i] > b.base_len || block_end(b, i) > b.base_len)
      return fail(FORST_EINVAL, "block " + std::to_string(i) + " reaches past base_len");
  std::vector<uint64_t> cuts(n_devices + 1);
  partition(b.sizes, n, static_cast<uint32_t>(n_devices), cuts.data());
  const bool direct = is_device_readable_host(b.base);
  std::vector<DeviceRun> runs(n_devices);
  std::vector<std::thread> th;
  for (int d = 0; d < n_devices; ++d) {
    runs[d].device = devices[d];
    runs[d].lo = cuts[d];
    runs[d].hi = cuts[d + 1];
    th.emplace_back(run_device, std::cref(b), direct, std::ref(runs[d]));
  }
  for (auto& t : th) t.join();
  uint64_t bad = 0;
  for (const DeviceRun& r : runs) {
    if (r.rc != FORST_OK) return fail(r.rc, "device " + std::to_string(r.device) + ": " + r.err);
    bad += r.mismatches;
  }
  if (mismatches) *mismatches = bad;
  return FORST_OK;
}

}  // namespace

#define FORST_API extern "C" __attribute__((visibility("default")))

FORST_API const char* forst_host_last_error(void) { return g_host_err.c_str(); }

FORST_API int forst_partition_bytes(const uint32_t* sizes, uint64_t n, uint32_t parts,
                                    uint64_t* cuts) {
  if ((!sizes && n) || !cuts || parts == 0) return fail(FORST_EINVAL, "partition: bad arguments");
  partition(sizes, n, parts, cuts);
  return FORST_OK;
}

FORST_API int forst_block_verify_host(int checksum_type, const uint8_t* host_base,
                                      uint64_t base_len, const uint64_t* offsets,
                                      const uint32_t* sizes, const uint32_t* modifiers,
                                      uint32_t* computed, uint32_t* stored, uint8_t* ok,
                                      uint64_t* mismatches, uint64_t n_blocks,
                                      const int* devices, int n_devices) {
  std::vector<uint32_t> scratch;
  if (!computed && n_blocks) {
    scratch.resize(n_blocks);
    computed = scratch.data();
  }
  const HostBatch b{Op::kVerify, checksum_type, host_base, base_len, offsets, sizes, nullptr,
                    modifiers,  computed,      stored,    ok};
  return run_host_batch(b, n_blocks, devices, n_devices, mismatches);
}

FORST_API int forst_block_checksum_host(int checksum_type, const uint8_t* host_base,
                                        uint64_t base_len, const uint64_t* offsets,
                                        const uint32_t* sizes, const uint8_t* last_bytes,
                                        const uint32_t* modifiers, uint32_t* out,
                                        uint64_t n_blocks, const int* devices, int n_devices) {
  const HostBatch b{Op::kChecksum, checksum_type, host_base, base_len, offsets, sizes, last_bytes,
                    modifiers,     out,           nullptr,   nullptr};
  return run_host_batch(b, n_blocks, devices, n_devices, nullptr);
}

FORST_API int forst_host_register(void* p, uint64_t len) {
  if (!p || !len) return fail(FORST_EINVAL, "host_register: null or empty range");
  // a read-only mapping (an SST file mmap'd PROT_READ) can only be pinned
  // read-only; anything else as a normal registration
  hipError_t e = hipHostRegister(p, len, hipHostRegisterReadOnly);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipHostRegister(p, len, hipHostRegisterDefault);
  }
  if (e != hipSuccess) return fail(FORST_EHIP, std::string("hipHostRegister: ") + hipGetErrorString(e));
  return FORST_OK;
}

FORST_API int forst_host_unregister(void* p) {
  const hipError_t e = hipHostUnregister(p);
  if (e != hipSuccess)
    return fail(FORST_EHIP, std::string("hipHostUnregister: ") + hipGetErrorString(e));
  return FORST_OK;
}
