// forst_amd/csrc/wal.hip -- WAL record CRCs, reader and writer side.
//
// Reader (log::Reader::ReadPhysicalRecord, db/log_reader.cc:450-531): a log is
// a run of 32 KiB blocks (db/log_format.h:45); inside a block, physical
// records [crc:4 len:2 type:1 (lognum:4)] payload follow each other, so the
// header chain is serial but every record's CRC is independent.  The verify
// is split into a pipeline on one stream:
//
//   walk    one LANE per log block follows the header chain (4-8 byte reads per
//           record, no payload), applying the structural checks the reader
//           makes before the CRC (bad length, old record, zero type,
//           truncated header); writes the record count per block and a
//           per-256-block tile sum
//   scan    one workgroup turns tile sums into tile prefixes (+ total)
//   fill    re-walks and writes one CRC descriptor per record
//           (offset = header + 6, length = hs + len - 6) at its global index
//   crc     crc32c_rows / stream2 kernel in raw mode over the descriptors --
//           the bulk of the bytes, at the block kernels' streaming rate
//   status  one lane per block compares computed vs stored masked CRCs and
//           reports the first failure exactly as the serial reader would
//
// The record total is needed to size the descriptor array, so the pipeline
// reads it back once (one stream synchronisation per call).  Scratch comes
// from a per-device stream-ordered pool that keeps its memory.
//
// Writer (log::Writer::EmitPhysicalRecord, db/log_writer.cc:228-263): header
// offsets are given, so descriptors are built per record, the same raw CRC
// kernel runs, and a finish kernel masks (util/crc32c.h:33) and stores them.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

#include "device_common.h"
#include "engine.h"

namespace forst {

hipError_t launch_wal_verify_wave(const WalArgs& a, hipStream_t stream, const char** name);
hipError_t launch_wal_record_crc_wave(const WalArgs& a, hipStream_t stream, const char** name);

namespace {

constexpr uint32_t kLogBlock = 32768;  // db/log_format.h:45
constexpr uint32_t kLogHdr = 7;        // db/log_format.h:48
constexpr uint32_t kLogRHdr = 11;      // db/log_format.h:52
constexpr uint32_t kTile = 256;        // log blocks per walk workgroup (one per lane)
constexpr uint32_t kScanThreads = 1024;
constexpr uint32_t kMaskDelta = 0xa282ead8u;  // util/crc32c.h:30

__device__ __forceinline__ bool recyclable_type(uint32_t t) {  // db/log_format.h:20-41
  return (t >= 5 && t <= 8) || t == 11;
}
__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {  // any alignment
  return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
         (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}
__device__ __forceinline__ void st_le32(uint8_t* p, uint32_t v) {
  p[0] = static_cast<uint8_t>(v);
  p[1] = static_cast<uint8_t>(v >> 8);
  p[2] = static_cast<uint8_t>(v >> 16);
  p[3] = static_cast<uint8_t>(v >> 24);
}
__device__ __forceinline__ uint32_t crc_unmask(uint32_t m) {  // util/crc32c.h:39
  const uint32_t r = m - kMaskDelta;
  return (r >> 17) | (r << 15);
}
__device__ __forceinline__ uint32_t crc_mask(uint32_t c) {  // util/crc32c.h:33
  return ((c >> 15) | (c << 17)) + kMaskDelta;
}

struct WalScratch {
  uint32_t* cnt;          // [n_blocks] structurally valid records per block
  uint32_t* stop;         // [n_blocks] status << 24 | stop position in block
  uint64_t* base;         // [n_blocks] global index of the block's first record
  uint32_t* tile_sum;     // [n_tiles]
  uint64_t* tile_prefix;  // [n_tiles + 1], last = total
  uint64_t* desc_off;     // [total]
  uint32_t* desc_len;     // [total]
  uint32_t* computed;     // [total]
};

// The header chain of log block b, as far as the reader can follow it without
// the CRC (log_reader.cc:465-512 in order: truncated header at EOF -> stop,
// length past the block -> kBadRecordLen (2), recycled record of an older log
// -> kOldRecord (4), type 0 / length 0 -> zero padding (3)).  FILL writes a
// descriptor per record at out_base.
template <bool FILL>
__device__ __forceinline__ uint32_t walk_block(const WalArgs& a, uint64_t b, uint32_t* stop,
                                               uint64_t out_base, uint64_t* d_off,
                                               uint32_t* d_len) {
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  uint32_t status = 0, cnt = 0;
  uint64_t pos = start;
  while (start < end && end - pos >= kLogHdr) {
    const uint8_t* h = a.log + pos;
    const uint32_t length = static_cast<uint32_t>(h[4]) | (static_cast<uint32_t>(h[5]) << 8);
    const uint32_t type = h[6];
    const bool recyc = recyclable_type(type);
    const uint32_t hs = recyc ? kLogRHdr : kLogHdr;
    if (end - pos < hs) break;
    if (hs + length > end - pos) {
      status = 2;
      break;
    }
    if (recyc && ld_le32(h + 7) != a.log_number) {
      status = 4;
      break;
    }
    if (type == 0 && length == 0) {
      status = 3;
      break;
    }
    if (FILL) {
      d_off[out_base + cnt] = pos + 6;
      d_len[out_base + cnt] = hs + length - 6;
    }
    ++cnt;
    pos += hs + length;
  }
  *stop = (status << 24) | static_cast<uint32_t>(pos - start);
  return cnt;
}

// exclusive scan of one value per thread over a 256-thread workgroup
__device__ __forceinline__ uint32_t wg_exclusive_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (uint32_t d = 1; d < kTile; d <<= 1) {
    const uint32_t add = t >= d ? sh[t - d] : 0u;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const uint32_t incl = sh[t];
  *total = sh[kTile - 1];
  __syncthreads();
  return incl - v;
}

__global__ void __launch_bounds__(kTile) wal_walk_kernel(WalArgs a, WalScratch s) {
  __shared__ uint32_t sh[kTile];
  const uint64_t bi = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  uint32_t cnt = 0, stop = 0;
  if (bi < a.n_blocks) {
    cnt = walk_block<false>(a, a.first_block + bi, &stop, 0, nullptr, nullptr);
    s.cnt[bi] = cnt;
    s.stop[bi] = stop;
  }
  uint32_t tot;
  wg_exclusive_scan(cnt, sh, &tot);
  if (threadIdx.x == 0) s.tile_sum[blockIdx.x] = tot;
}

// single workgroup: tile_prefix[i] = sum(tile_sum[0..i)), tile_prefix[n] = total
__global__ void __launch_bounds__(kScanThreads) wal_scan_kernel(WalScratch s, uint64_t n_tiles) {
  __shared__ uint64_t sh[kScanThreads];
  const uint32_t t = threadIdx.x;
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < n_tiles; c0 += kScanThreads) {
    const uint64_t i = c0 + t;
    const uint64_t v = i < n_tiles ? s.tile_sum[i] : 0;
    sh[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kScanThreads; d <<= 1) {
      const uint64_t add = t >= d ? sh[t - d] : 0;
      __syncthreads();
      sh[t] += add;
      __syncthreads();
    }
    if (i < n_tiles) s.tile_prefix[i] = carry + sh[t] - v;
    carry += sh[kScanThreads - 1];
    __syncthreads();
  }
  if (t == 0) s.tile_prefix[n_tiles] = carry;
}

__global__ void __launch_bounds__(kTile) wal_fill_kernel(WalArgs a, WalScratch s) {
  __shared__ uint32_t sh[kTile];
  const uint64_t bi = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  const uint32_t cnt = bi < a.n_blocks ? s.cnt[bi] : 0u;
  uint32_t tot;
  const uint64_t base = s.tile_prefix[blockIdx.x] + wg_exclusive_scan(cnt, sh, &tot);
  if (bi < a.n_blocks) {
    s.base[bi] = base;
    uint32_t stop;
    if (cnt) walk_block<true>(a, a.first_block + bi, &stop, base, s.desc_off, s.desc_len);
  }
}

// first failing record of the block in reader order: a CRC mismatch among the
// structurally valid records (kBadRecordChecksum, 1), else the walk's stop
__global__ void __launch_bounds__(kTile) wal_status_kernel(WalArgs a, WalScratch s) {
  const uint64_t bi = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (bi >= a.n_blocks) return;
  const uint32_t cnt = s.cnt[bi];
  const uint64_t base = s.base[bi];
  const uint64_t start = (a.first_block + bi) * kLogBlock;
  uint32_t status = s.stop[bi] >> 24, pos = s.stop[bi] & 0xffffffu, nrec = cnt;
  for (uint32_t j = 0; j < cnt; ++j) {
    const uint64_t off = s.desc_off[base + j] - 6;
    if (crc_unmask(ld_le32(a.log + off)) != s.computed[base + j]) {
      status = 1;
      nrec = j;
      pos = static_cast<uint32_t>(off - start);
      break;
    }
  }
  if (a.status_out) a.status_out[bi] = static_cast<uint8_t>(status);
  if (a.nrec_out) a.nrec_out[bi] = nrec;
  if (a.fail_off_out) a.fail_off_out[bi] = pos;
  if (a.bad_blocks && status != 0 && status != 3) atomicAdd(a.bad_blocks, 1ull);
}

// writer side: descriptor per header offset (length 0 = header out of range)
__global__ void __launch_bounds__(kTile) wal_rec_desc_kernel(WalArgs a, uint64_t* d_off,
                                                             uint32_t* d_len) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i >= a.n_records) return;
  const uint64_t off = a.header_offsets[i];
  uint64_t o = 0;
  uint32_t n = 0;
  if (off <= a.log_len && a.log_len - off >= kLogHdr) {
    const uint8_t* h = a.log + off;
    const uint32_t length = static_cast<uint32_t>(h[4]) | (static_cast<uint32_t>(h[5]) << 8);
    const uint32_t hs = recyclable_type(h[6]) ? kLogRHdr : kLogHdr;
    if (a.log_len - off >= uint64_t(hs) + length) {
      o = off + 6;
      n = hs + length - 6;
    }
  }
  d_off[i] = o;
  d_len[i] = n;
}

__global__ void __launch_bounds__(kTile) wal_rec_finish_kernel(WalArgs a, const uint32_t* d_len,
                                                               const uint32_t* computed) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i >= a.n_records) return;
  const bool valid = d_len[i] != 0;
  const uint32_t c = valid ? crc_mask(computed[i]) : 0u;
  if (valid && a.write_in_place) st_le32(a.log_w + a.header_offsets[i], c);
  if (a.crc_out) a.crc_out[i] = c;
}

size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

bool wave_variant() {
  const char* v = std::getenv("FORST_WAL_VARIANT");
  return v && std::string(v) == "wave";
}

}  // namespace

hipError_t launch_wal_verify(const WalArgs& a, hipStream_t stream, const char** name) {
  if (a.n_blocks == 0) return hipSuccess;
  if (wave_variant()) return launch_wal_verify_wave(a, stream, name);
  const uint64_t n_tiles = (a.n_blocks + kTile - 1) / kTile;
  const size_t nb = a.n_blocks;
  const size_t sz_cnt = up256(4 * nb), sz_stop = up256(4 * nb), sz_base = up256(8 * nb),
               sz_ts = up256(4 * n_tiles), sz_tp = up256(8 * (n_tiles + 1));
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, sz_cnt + sz_stop + sz_base + sz_ts + sz_tp, stream);
  if (e != hipSuccess) return e;
  uint8_t* p = static_cast<uint8_t*>(scratch);
  WalScratch s{};
  s.cnt = reinterpret_cast<uint32_t*>(p);
  s.stop = reinterpret_cast<uint32_t*>(p + sz_cnt);
  s.base = reinterpret_cast<uint64_t*>(p + sz_cnt + sz_stop);
  s.tile_sum = reinterpret_cast<uint32_t*>(p + sz_cnt + sz_stop + sz_base);
  s.tile_prefix = reinterpret_cast<uint64_t*>(p + sz_cnt + sz_stop + sz_base + sz_ts);
  const dim3 grid(static_cast<uint32_t>(n_tiles));
  hipLaunchKernelGGL(wal_walk_kernel, grid, dim3(kTile), 0, stream, a, s);
  hipLaunchKernelGGL(wal_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, s, n_tiles);
  uint64_t total = 0;
  if ((e = hipGetLastError()) != hipSuccess ||
      (e = hipMemcpyAsync(&total, s.tile_prefix + n_tiles, 8, hipMemcpyDeviceToHost, stream)) !=
          hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess) {
    (void)scratch_free(scratch, stream);
    return e;
  }
  void* desc = nullptr;
  const size_t sz_off = up256(8 * total), sz_len = up256(4 * total);
  if ((e = scratch_alloc(&desc, sz_off + 2 * sz_len, stream)) != hipSuccess) {
    (void)scratch_free(scratch, stream);
    return e;
  }
  s.desc_off = static_cast<uint64_t*>(desc);
  s.desc_len = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(desc) + sz_off);
  s.computed = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(desc) + sz_off + sz_len);
  hipLaunchKernelGGL(wal_fill_kernel, grid, dim3(kTile), 0, stream, a, s);
  *name = "wal_walk_kernel";
  if (total) {
    BlockArgs b{};
    b.base = a.log;
    b.base_len = a.log_len;
    b.offsets = s.desc_off;
    b.sizes = s.desc_len;
    b.out32 = s.computed;
    b.n = total;
    e = launch_crc32c_blocks(kModeRaw, b, stream, name);
  }
  hipLaunchKernelGGL(wal_status_kernel, grid, dim3(kTile), 0, stream, a, s);
  if (e == hipSuccess) e = hipGetLastError();
  const hipError_t f1 = scratch_free(desc, stream), f2 = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f1 != hipSuccess ? f1 : f2;
}

hipError_t launch_wal_record_crc(const WalArgs& a, hipStream_t stream, const char** name) {
  if (a.n_records == 0) return hipSuccess;
  if (wave_variant()) return launch_wal_record_crc_wave(a, stream, name);
  const size_t n = a.n_records;
  const size_t sz_off = up256(8 * n), sz_len = up256(4 * n);
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, sz_off + 2 * sz_len, stream);
  if (e != hipSuccess) return e;
  uint64_t* d_off = static_cast<uint64_t*>(scratch);
  uint32_t* d_len = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + sz_off);
  uint32_t* comp = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + sz_off + sz_len);
  const dim3 grid(static_cast<uint32_t>((n + kTile - 1) / kTile));
  hipLaunchKernelGGL(wal_rec_desc_kernel, grid, dim3(kTile), 0, stream, a, d_off, d_len);
  BlockArgs b{};
  b.base = a.log;
  b.base_len = a.log_len;
  b.offsets = d_off;
  b.sizes = d_len;
  b.out32 = comp;
  b.n = n;
  e = launch_crc32c_blocks(kModeRaw, b, stream, name);
  hipLaunchKernelGGL(wal_rec_finish_kernel, grid, dim3(kTile), 0, stream, a, d_len, comp);
  if (e == hipSuccess) e = hipGetLastError();
  const hipError_t f = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f;
}

}  // namespace forst
