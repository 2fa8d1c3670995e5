// forst_amd/csrc/host_batch.cc -- host-memory batches over the GPUs of one
// process (SURVEY.md §8e / §8d "end-to-end").
//
// ForSt is one process: DB::VerifyChecksum (db/db_impl/db_impl.cc:6254) walks
// every live SST file, and flush / compaction threads hand blocks that live in
// host memory (the table builder's buffer, a FilePrefetchBuffer, an mmap'd
// file -- env/io_posix.cc:958).  These entry points take such a host batch and
// a device list, cut the blocks into contiguous byte-balanced ranges (one per
// device, forst_partition_bytes) and give every device its own worker thread,
// HIP stream and pinned staging: the worker streams its range through two
// device windows (copy of window k+1 overlaps the kernel on window k), runs
// the block kernels on them and brings back 4-5 B per block.  No data crosses
// between devices; the only join is the caller's wait for the workers.
//
// The per-device resources -- worker thread, non-blocking stream, two device
// windows with descriptor / result arrays, their pinned mirrors and staging
// -- live in a context that is created once and reused by every later call
// (a pool per device: concurrent callers each take a free context, so flush,
// compaction and verify threads never share one).  Buffers only grow; nothing
// is allocated or freed on the steady-state path, and an error leaves the
// context intact (nothing to leak).  forst_host_context_stats reports what the
// pool holds.
//
// Host memory that is pinned or registered over the whole batch
// (hipHostRegister, e.g. an mmap'd SST file: forst_host_register) is copied by
// DMA straight from the caller's pages; otherwise it is first memcpy'd into the
// context's pinned staging.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/forst_checksum.h"
#include "engine.h"

namespace {

thread_local std::string g_host_err;

int fail(int code, const std::string& m) {
  g_host_err = m;
  return code;
}

constexpr uint64_t kWindowBytes = 64ull << 20;  // device window per copy (two per device)
constexpr uint64_t kWindowBlocks = 1u << 20;    // descriptors per window
constexpr uint32_t kTrailer = 5;                // block_based_table_reader.h:75
constexpr uint64_t kPerBlock = 26;              // descriptor + result bytes per block

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

// ranges registered through forst_host_register: start -> length
std::mutex g_reg_mu;
std::map<uintptr_t, uint64_t> g_regs;

// DMA straight from the caller's pages only if ONE pinned allocation or
// registration covers the whole range: a forst_host_register'ed range, or a
// hipHostMalloc'ed / otherwise registered allocation whose extent
// (hipMemGetAddressRange) holds it.  Anything else -- two registrations with
// unregistered pages between them, a registration over part of the range, a
// dropped one -- is staged.
bool range_device_readable(const uint8_t* base, uint64_t len) {
  if (!len) return false;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(base);
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_regs.upper_bound(lo);
    if (it != g_regs.begin()) {
      --it;
      if (it->first <= lo && lo + len <= it->first + it->second) return true;
    }
  }
  if (!is_device_readable_host(base)) return false;
  void* pb = nullptr;
  size_t ps = 0;
  if (hipMemGetAddressRange(&pb, &ps, const_cast<uint8_t*>(base)) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t ab = reinterpret_cast<uintptr_t>(pb);
  return ab <= lo && lo + len <= ab + ps;
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

// bytes a block needs in host memory: payload + trailer (verify), payload +
// type byte (compute without last_bytes), payload (compute with last_bytes)
uint64_t block_end(const HostBatch& b, uint64_t i) {
  const uint32_t extra = b.op == Op::kVerify ? kTrailer : b.last_bytes ? 0 : 1;
  return b.offsets[i] + b.sizes[i] + extra;
}

// one device window: device bytes + descriptors + results, and their pinned
// mirrors (+ staging for pageable input)
struct Slot {
  uint64_t dbytes = 0, blocks = 0, hbytes = 0;  // capacities
  uint8_t* d = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t *d_size = nullptr, *d_mod = nullptr, *d_out = nullptr, *d_st = nullptr;
  uint8_t *d_last = nullptr, *d_ok = nullptr;
  unsigned long long* d_bad = nullptr;
  uint8_t* hbase = nullptr;
  uint8_t* h = nullptr;  // pinned staging (pageable input)
  uint64_t* h_off = nullptr;
  uint32_t *h_size = nullptr, *h_mod = nullptr, *h_out = nullptr, *h_st = nullptr;
  uint8_t *h_last = nullptr, *h_ok = nullptr;
  unsigned long long* h_bad = nullptr;
  hipEvent_t done = nullptr;
  int64_t win = -1;  // window whose results are pending in this slot

  void release() {
    (void)hipFree(d);
    (void)hipHostFree(hbase);
    d = nullptr;
    hbase = nullptr;
    dbytes = blocks = hbytes = 0;
  }
  // grow-only: (re)allocate when a call needs more than the slot holds
  hipError_t reserve(uint64_t need_bytes, uint64_t need_blocks, bool staging) {
    const uint64_t nb = (need_bytes + 255) & ~255ull;
    const uint64_t hb = staging ? nb : 0;
    if (nb <= dbytes && need_blocks <= blocks && hb <= hbytes && d) return hipSuccess;
    const uint64_t db = std::max(nb, dbytes), m = std::max(need_blocks, blocks),
                   hs = std::max(hb, hbytes);
    release();
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, db + m * kPerBlock + 64);
    if (e != hipSuccess) return e;
    d = static_cast<uint8_t*>(p);
    d_off = reinterpret_cast<uint64_t*>(d + db);
    d_size = reinterpret_cast<uint32_t*>(d_off + m);
    d_mod = d_size + m;
    d_out = d_mod + m;
    d_st = d_out + m;
    d_bad = reinterpret_cast<unsigned long long*>(d_st + m);  // 24 m bytes in: aligned
    d_last = reinterpret_cast<uint8_t*>(d_bad + 1);
    d_ok = d_last + m;
    if ((e = hipHostMalloc(&p, m * kPerBlock + 128 + hs)) != hipSuccess) {
      (void)hipFree(d);
      d = nullptr;
      return e;
    }
    hbase = static_cast<uint8_t*>(p);
    h_off = reinterpret_cast<uint64_t*>(hbase);
    h_size = reinterpret_cast<uint32_t*>(h_off + m);
    h_mod = h_size + m;
    h_out = h_mod + m;
    h_st = h_out + m;
    h_bad = reinterpret_cast<unsigned long long*>(h_st + m);
    h_last = reinterpret_cast<uint8_t*>(h_bad + 1);
    h_ok = h_last + m;
    h = hs ? h_ok + m + 64 - ((reinterpret_cast<uintptr_t>(h_ok + m)) & 63) : nullptr;
    dbytes = db;
    blocks = m;
    hbytes = hs;
    return hipSuccess;
  }
};

// The staged path's copy into pinned memory, split over the worker and
// kCopyHelpers helper threads: one thread's memcpy from pageable memory (page
// walks, first touch of an mmap'd file) ran at ~19 GiB/s, under the PCIe
// rate the DMA behind it reaches (bench host_memory_verify, round 5).
// Helpers are started on the first large copy and live with the context.
constexpr int kCopyHelpers = 3;
constexpr uint64_t kCopySplitMin = 4ull << 20;  // smaller copies: one thread
struct Copier {
  std::thread th[kCopyHelpers];
  std::mutex mu;
  std::condition_variable go, done;
  uint64_t gen = 0;
  int pending = 0;
  bool started = false;
  uint8_t* dst = nullptr;
  const uint8_t* src = nullptr;
  uint64_t n = 0;

  // slice k of kCopyHelpers + 1, cut at 4 KiB boundaries of the destination
  void slice(int k) const {
    const uint64_t parts = kCopyHelpers + 1;
    const uint64_t lo = (n * k / parts) & ~4095ull;
    const uint64_t hi = k + 1 == static_cast<int>(parts) ? n : (n * (k + 1) / parts) & ~4095ull;
    if (hi > lo) std::memcpy(dst + lo, src + lo, hi - lo);
  }
  void loop(int k) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu);
        go.wait(lk, [&] { return gen != seen; });
        seen = gen;
      }
      slice(k + 1);
      std::lock_guard<std::mutex> lk(mu);
      if (--pending == 0) done.notify_all();
    }
  }
  void copy(uint8_t* d, const uint8_t* s, uint64_t bytes) {
    if (bytes < kCopySplitMin) {
      std::memcpy(d, s, bytes);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      if (!started) {
        started = true;
        for (int k = 0; k < kCopyHelpers; ++k) {
          th[k] = std::thread([this, k] { loop(k); });
          th[k].detach();  // lives with the context (for the whole process)
        }
      }
      dst = d;
      src = s;
      n = bytes;
      pending = kCopyHelpers;
      ++gen;
    }
    go.notify_all();
    slice(0);
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [&] { return pending == 0; });
  }
};

// a per-device context: worker thread + stream + two slots, reused by every
// call that takes it from the pool
struct DeviceCtx {
  int device = 0;
  hipStream_t st = nullptr;
  Slot slot[2];
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool busy = false;
  std::mutex res_mu;  // held while the slots' buffers change (reserve / trim) or are read (stats)
  Copier copier;      // the staged path's copies into pinned memory
  // (WAL path) a second stream for the host-to-device copies: the WAL verify
  // reads a count back (one stream synchronisation per window), so the next
  // window's copy runs on its own stream to overlap it
  hipStream_t cst = nullptr;
  hipEvent_t copied[2] = {nullptr, nullptr};

  explicit DeviceCtx(int dev) : device(dev) {
    worker = std::thread([this] { loop(); });
    worker.detach();  // contexts live for the whole process
  }
  void loop() {
    (void)hipSetDevice(device);
    for (;;) {
      std::function<void()> j;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [this] { return static_cast<bool>(job); });
        j = std::move(job);
      }
      j();
      {
        std::lock_guard<std::mutex> lk(mu);
        busy = false;
      }
      cv.notify_all();
    }
  }
  void run(std::function<void()> j) {
    std::lock_guard<std::mutex> lk(mu);
    busy = true;
    job = std::move(j);
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !busy; });
  }
  // stream and events, once (on the worker's device)
  // (all or nothing: a partial failure destroys what it created, so a later
  // call retries from scratch instead of finding a stream without events)
  hipError_t init() {
    if (st) return hipSuccess;
    hipStream_t s0 = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    for (Slot& s : slot) {
      if ((e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess) {
        for (Slot& u : slot) {
          if (u.done) (void)hipEventDestroy(u.done);
          u.done = nullptr;
        }
        (void)hipStreamDestroy(s0);
        return e;
      }
    }
    st = s0;
    return hipSuccess;
  }
};

std::mutex g_pool_mu;
std::map<int, std::vector<DeviceCtx*>>* g_free = new std::map<int, std::vector<DeviceCtx*>>();
std::vector<DeviceCtx*>* g_all = new std::vector<DeviceCtx*>();  // never destroyed

DeviceCtx* acquire_ctx(int dev) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  auto& v = (*g_free)[dev];
  if (!v.empty()) {
    DeviceCtx* c = v.back();
    v.pop_back();
    return c;
  }
  DeviceCtx* c = new DeviceCtx(dev);
  g_all->push_back(c);
  return c;
}

void release_ctx(DeviceCtx* c) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  (*g_free)[c->device].push_back(c);
}

// One device's share [lo, hi) of the blocks, in windows of at most
// kWindowBytes (a block larger than that gets a window of its own).
struct DeviceRun {
  uint64_t lo = 0, hi = 0;
  uint64_t mismatches = 0;
  int rc = FORST_OK;
  std::string err;
};

struct Window {
  uint64_t c0, c1, base0, end;  // blocks [c0, c1) in host bytes [base0, end)
};

void run_device(const HostBatch& b, bool direct, DeviceCtx& cx, DeviceRun& r) {
  auto bail = [&](hipError_t e, const char* what) {
    r.rc = FORST_EHIP;
    r.err = std::string(what) + ": " + hipGetErrorString(e);
  };
  if (r.hi <= r.lo) return;
  hipError_t e = cx.init();
  if (e != hipSuccess) return bail(e, "hipStreamCreate / hipEventCreate");
  // windows: contiguous block runs whose bytes fit one device window; a
  // window spans [min offset, max end) of its blocks, so descriptors need not
  // ascend
  std::vector<Window> win;
  uint64_t max_bytes = 0, max_blocks = 0;
  for (uint64_t c0 = r.lo; c0 < r.hi;) {
    uint64_t lo = b.offsets[c0], hi = block_end(b, c0), c1 = c0 + 1;
    while (c1 < r.hi && c1 - c0 < kWindowBlocks) {
      const uint64_t nlo = std::min(lo, b.offsets[c1]), nhi = std::max(hi, block_end(b, c1));
      if (nhi - (nlo & ~3ull) > kWindowBytes) break;
      lo = nlo;
      hi = nhi;
      ++c1;
    }
    const uint64_t base0 = lo & ~3ull;
    max_bytes = std::max(max_bytes, hi - base0);
    max_blocks = std::max(max_blocks, c1 - c0);
    win.push_back({c0, c1, base0, hi});
    c0 = c1;
  }
  for (Slot& s : cx.slot) {
    std::unique_lock<std::mutex> rl(cx.res_mu);
    e = s.reserve(max_bytes, max_blocks, !direct);
    rl.unlock();
    if (e != hipSuccess)
      return bail(e, "window allocation");
    s.win = -1;
  }
  hipStream_t st = cx.st;
  auto collect = [&](Slot& s) -> bool {
    if (s.win < 0) return true;
    hipError_t w = hipEventSynchronize(s.done);
    if (w != hipSuccess) {
      bail(w, "hipEventSynchronize");
      s.win = -1;
      return false;
    }
    const Window& wd = win[s.win];
    const uint64_t k = wd.c1 - wd.c0;
    std::memcpy(b.out + wd.c0, s.h_out, k * 4);
    if (b.op == Op::kVerify) {
      if (b.stored) std::memcpy(b.stored + wd.c0, s.h_st, k * 4);
      if (b.ok) std::memcpy(b.ok + wd.c0, s.h_ok, k);
      r.mismatches += *s.h_bad;
    }
    s.win = -1;
    return true;
  };
  for (uint64_t w = 0; w < win.size() && r.rc == FORST_OK; ++w) {
    Slot& s = cx.slot[w & 1];
    if (!collect(s)) break;  // the slot's previous window is done: reuse it
    const Window& wd = win[w];
    const uint64_t k = wd.c1 - wd.c0;
    for (uint64_t i = wd.c0; i < wd.c1; ++i) {
      s.h_off[i - wd.c0] = b.offsets[i] - wd.base0;
      s.h_size[i - wd.c0] = b.sizes[i];
      if (b.modifiers) s.h_mod[i - wd.c0] = b.modifiers[i];
      if (b.last_bytes) s.h_last[i - wd.c0] = b.last_bytes[i];
    }
    const uint64_t nbytes = std::min(wd.end, b.base_len) - wd.base0;
    const uint8_t* src = b.base + wd.base0;
    if (!direct) {
      cx.copier.copy(s.h, src, nbytes);
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
      if ((e = hipMemsetAsync(s.d_bad, 0, 8, st)) != hipSuccess) {
        bail(e, "hipMemsetAsync");
        break;
      }
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
    collect(cx.slot[0]);
    if (r.rc == FORST_OK) collect(cx.slot[1]);
  }
  // the context goes back to the pool idle: nothing of this call in flight
  (void)hipStreamSynchronize(st);
  cx.slot[0].win = cx.slot[1].win = -1;
}

// ---- WAL log blocks from host memory (a13 over several devices) -----------
// db/log_reader.cc:450-531 checks every physical record of a 32 KiB log block
// on its own (records never straddle a block, log_writer.cc:86-102), so a
// log read into host memory (the reader's 32 KiB reads, log_reader.cc:404)
// splits into contiguous block ranges, one per device, each streamed through
// the device's context in windows of kWalWinBlocks blocks:
// forst_wal_verify_batch per window, 9 B of results per block back.
constexpr uint64_t kWalBlockBytes = 32768;  // db/log_format.h:45
constexpr uint64_t kWalWinBlocks = kWindowBytes / kWalBlockBytes;

struct WalHostBatch {
  const uint8_t* log;
  uint64_t log_len;
  uint32_t log_number;
  uint8_t* status;
  uint32_t* nrec;
  uint32_t* fail;
};

void run_wal_device(const WalHostBatch& b, bool direct, DeviceCtx& cx, DeviceRun& r) {
  auto bail = [&](hipError_t e, const char* what) {
    r.rc = FORST_EHIP;
    r.err = std::string(what) + ": " + hipGetErrorString(e);
  };
  if (r.hi <= r.lo) return;
  hipError_t e = cx.init();
  if (e != hipSuccess) return bail(e, "hipStreamCreate / hipEventCreate");
  if (!cx.cst) {
    hipStream_t s1 = nullptr;
    if ((e = hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)) != hipSuccess)
      return bail(e, "hipStreamCreate");
    for (auto& ev : cx.copied)
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
        for (auto& u : cx.copied) {
          if (u) (void)hipEventDestroy(u);
          u = nullptr;
        }
        (void)hipStreamDestroy(s1);
        return bail(e, "hipEventCreate");
      }
    cx.cst = s1;
  }
  const uint64_t nwin = (r.hi - r.lo + kWalWinBlocks - 1) / kWalWinBlocks;
  const uint64_t wblocks = std::min<uint64_t>(r.hi - r.lo, kWalWinBlocks);
  for (Slot& s : cx.slot) {
    std::unique_lock<std::mutex> rl(cx.res_mu);
    // device window: the log bytes; per block 1 + 4 + 4 result bytes in the
    // slot's descriptor area (blocks * kPerBlock >= 9 per block)
    e = s.reserve(wblocks * kWalBlockBytes, wblocks, !direct);
    rl.unlock();
    if (e != hipSuccess) return bail(e, "window allocation");
    s.win = -1;
  }
  const hipStream_t st = cx.st, cs = cx.cst;
  auto win_range = [&](uint64_t w, uint64_t* b0, uint64_t* nb, uint64_t* lo, uint64_t* len) {
    *b0 = r.lo + w * kWalWinBlocks;
    *nb = std::min<uint64_t>(kWalWinBlocks, r.hi - *b0);
    *lo = *b0 * kWalBlockBytes;
    *len = std::min<uint64_t>(b.log_len, (*b0 + *nb) * kWalBlockBytes) - *lo;
  };
  // the copy of window w into slot w & 1 (on the copy stream)
  auto issue_copy = [&](uint64_t w) -> bool {
    uint64_t b0, nb, lo, len;
    win_range(w, &b0, &nb, &lo, &len);
    Slot& s = cx.slot[w & 1];
    const uint8_t* src = b.log + lo;
    if (!direct) {
      // the staging buffer of this slot was last read by the copy of window
      // w - 2, which the verify of w - 2 (done: synchronised) waited for
      cx.copier.copy(s.h, src, len);
      src = s.h;
    }
    if ((e = hipMemcpyAsync(s.d, src, len, hipMemcpyHostToDevice, cs)) != hipSuccess ||
        (e = hipEventRecord(cx.copied[w & 1], cs)) != hipSuccess) {
      bail(e, "hipMemcpyAsync");
      return false;
    }
    return true;
  };
  if (!issue_copy(0)) {
    (void)hipStreamSynchronize(cs);
    return;
  }
  for (uint64_t w = 0; w < nwin && r.rc == FORST_OK; ++w) {
    uint64_t b0, nb, lo, len;
    win_range(w, &b0, &nb, &lo, &len);
    Slot& s = cx.slot[w & 1];
    if ((e = hipStreamWaitEvent(st, cx.copied[w & 1], 0)) != hipSuccess) {
      bail(e, "hipStreamWaitEvent");
      break;
    }
    // the next window's copy overlaps this one's verify (its slot's previous
    // verify, of window w - 1, is complete: forst_wal_verify_batch
    // synchronises st, and the copies of the results below are waited for)
    if (w + 1 < nwin && !issue_copy(w + 1)) break;
    uint8_t* d_st = reinterpret_cast<uint8_t*>(s.d_out);
    uint32_t* d_nr = s.d_st;
    uint32_t* d_fo = s.d_mod;
    if ((e = hipMemsetAsync(s.d_bad, 0, 8, st)) != hipSuccess) {
      bail(e, "hipMemsetAsync");
      break;
    }
    const int rc = forst_wal_verify_batch(s.d, len, 0, nb, b.log_number, d_st, d_nr, d_fo, s.d_bad,
                                          st);
    if (rc != FORST_OK) {
      r.rc = rc;
      r.err = forst_last_error();
      break;
    }
    bool ok = true;
    if (b.status) ok = ok && (e = hipMemcpyAsync(s.h_out, d_st, nb, hipMemcpyDeviceToHost, st)) == hipSuccess;
    if (b.nrec) ok = ok && (e = hipMemcpyAsync(s.h_st, d_nr, 4 * nb, hipMemcpyDeviceToHost, st)) == hipSuccess;
    if (b.fail) ok = ok && (e = hipMemcpyAsync(s.h_mod, d_fo, 4 * nb, hipMemcpyDeviceToHost, st)) == hipSuccess;
    ok = ok && (e = hipMemcpyAsync(s.h_bad, s.d_bad, 8, hipMemcpyDeviceToHost, st)) == hipSuccess;
    ok = ok && (e = hipStreamSynchronize(st)) == hipSuccess;
    if (!ok) {
      bail(e, "hipMemcpyAsync");
      break;
    }
    if (b.status) std::memcpy(b.status + b0, s.h_out, nb);
    if (b.nrec) std::memcpy(b.nrec + b0, s.h_st, 4 * nb);
    if (b.fail) std::memcpy(b.fail + b0, s.h_mod, 4 * nb);
    r.mismatches += *s.h_bad;
  }
  (void)hipStreamSynchronize(cs);
  (void)hipStreamSynchronize(st);
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
  int n_dev_total = 0;
  if (hipGetDeviceCount(&n_dev_total) != hipSuccess) n_dev_total = 0;
  for (int d = 0; d < n_devices; ++d)
    if (devices[d] < 0 || devices[d] >= n_dev_total)
      return fail(FORST_ENODEV, "no HIP device " + std::to_string(devices[d]));
  std::vector<uint64_t> cuts(n_devices + 1);
  partition(b.sizes, n, static_cast<uint32_t>(n_devices), cuts.data());
  const bool direct = range_device_readable(b.base, b.base_len);
  std::vector<DeviceRun> runs(n_devices);
  std::vector<DeviceCtx*> ctx(n_devices);
  for (int d = 0; d < n_devices; ++d) {
    runs[d].lo = cuts[d];
    runs[d].hi = cuts[d + 1];
    ctx[d] = acquire_ctx(devices[d]);
    DeviceCtx* c = ctx[d];
    DeviceRun* r = &runs[d];
    c->run([&b, direct, c, r] { run_device(b, direct, *c, *r); });
  }
  for (DeviceCtx* c : ctx) {
    c->wait();
    release_ctx(c);
  }
  uint64_t bad = 0;
  for (int d = 0; d < n_devices; ++d) {
    if (runs[d].rc != FORST_OK)
      return fail(runs[d].rc, "device " + std::to_string(devices[d]) + ": " + runs[d].err);
    bad += runs[d].mismatches;
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

FORST_API int forst_wal_verify_host(const uint8_t* host_log, uint64_t log_len,
                                    uint32_t log_number, uint8_t* status_out, uint32_t* nrec_out,
                                    uint32_t* fail_off_out, uint64_t* bad_blocks,
                                    const int* devices, int n_devices) {
  if (bad_blocks) *bad_blocks = 0;
  if (log_len == 0) return FORST_OK;
  if (!host_log || !devices || n_devices <= 0)
    return fail(FORST_EINVAL, "wal_verify_host: null log or no device");
  int n_dev_total = 0;
  if (hipGetDeviceCount(&n_dev_total) != hipSuccess) n_dev_total = 0;
  for (int d = 0; d < n_devices; ++d)
    if (devices[d] < 0 || devices[d] >= n_dev_total)
      return fail(FORST_ENODEV, "no HIP device " + std::to_string(devices[d]));
  const uint64_t nb = (log_len + kWalBlockBytes - 1) / kWalBlockBytes;
  const WalHostBatch b{host_log, log_len, log_number, status_out, nrec_out, fail_off_out};
  const bool direct = range_device_readable(host_log, log_len);
  std::vector<DeviceRun> runs(n_devices);
  std::vector<DeviceCtx*> ctx(n_devices);
  for (int d = 0; d < n_devices; ++d) {  // equal contiguous block ranges
    runs[d].lo = nb * d / n_devices;
    runs[d].hi = nb * (d + 1) / n_devices;
    ctx[d] = acquire_ctx(devices[d]);
    DeviceCtx* c = ctx[d];
    DeviceRun* r = &runs[d];
    c->run([&b, direct, c, r] { run_wal_device(b, direct, *c, *r); });
  }
  for (DeviceCtx* c : ctx) {
    c->wait();
    release_ctx(c);
  }
  uint64_t bad = 0;
  for (int d = 0; d < n_devices; ++d) {
    if (runs[d].rc != FORST_OK)
      return fail(runs[d].rc, "device " + std::to_string(devices[d]) + ": " + runs[d].err);
    bad += runs[d].mismatches;
  }
  if (bad_blocks) *bad_blocks = bad;
  return FORST_OK;
}

FORST_API int forst_host_context_stats(uint32_t* contexts, uint64_t* device_bytes,
                                       uint64_t* pinned_bytes) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  uint64_t db = 0, pb = 0;
  for (DeviceCtx* c : *g_all) {
    std::lock_guard<std::mutex> rl(c->res_mu);
    for (const Slot& s : c->slot) {
      if (s.d) db += s.dbytes + s.blocks * kPerBlock + 64;
      if (s.hbase) pb += s.blocks * kPerBlock + 128 + s.hbytes;
    }
  }
  if (contexts) *contexts = static_cast<uint32_t>(g_all->size());
  if (device_bytes) *device_bytes = db;
  if (pinned_bytes) *pinned_bytes = pb;
  return FORST_OK;
}

// the windows and staging of every context not in use right now go back to
// the driver (contexts, threads and streams stay; the next call that takes
// one grows it again)
FORST_API int forst_host_context_trim(uint64_t* released_bytes) {
  // the releases run on the caller's thread: its current device is restored
  // afterwards, so the caller's later HIP (or torch) work keeps its device
  int prev_dev = -1;
  const bool have_prev = hipGetDevice(&prev_dev) == hipSuccess;
  uint64_t freed = 0;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto& kv : *g_free)
      for (DeviceCtx* c : kv.second) {
        std::lock_guard<std::mutex> rl(c->res_mu);
        (void)hipSetDevice(c->device);
        for (Slot& s : c->slot) {
          if (s.d) freed += s.dbytes + s.blocks * kPerBlock + 64;
          if (s.hbase) freed += s.blocks * kPerBlock + 128 + s.hbytes;
          s.release();
          s.win = -1;
        }
      }
  }
  // the WAL calls' idle auxiliary streams and events (engine.h aux_pool_trim)
  forst::aux_pool_trim();
  if (have_prev) (void)hipSetDevice(prev_dev);
  (void)hipGetLastError();
  if (released_bytes) *released_bytes = freed;
  return FORST_OK;
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
  std::lock_guard<std::mutex> g(g_reg_mu);
  g_regs[reinterpret_cast<uintptr_t>(p)] = len;
  return FORST_OK;
}

FORST_API int forst_host_unregister(void* p) {
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    g_regs.erase(reinterpret_cast<uintptr_t>(p));
  }
  const hipError_t e = hipHostUnregister(p);
  if (e != hipSuccess)
    return fail(FORST_EHIP, std::string("hipHostUnregister: ") + hipGetErrorString(e));
  return FORST_OK;
}
