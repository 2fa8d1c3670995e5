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
#include "scan_common.h"
#include "wal_hash.h"

namespace forst {

#ifdef FORST_DIAG
hipError_t launch_wal_verify_wave(const WalArgs& a, hipStream_t stream, const char** name);
hipError_t launch_wal_record_crc_wave(const WalArgs& a, hipStream_t stream, const char** name);
#endif

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
  uint32_t* stored;       // [total] unmasked stored CRC (fill, from the header it reads anyway)
};

// The header chain of log block b, as far as the reader can follow it without
// the CRC (log_reader.cc:465-512 in order: truncated header at EOF -> stop,
// length past the block -> kBadRecordLen (2), recycled record of an older log
// -> kOldRecord (4), type 0 / length 0 -> zero padding (3)).  FILL writes a
// descriptor per record at out_base.
template <bool FILL>
__device__ __forceinline__ uint32_t walk_block(const WalArgs& a, uint64_t b, uint32_t* stop,
                                               uint64_t out_base, uint64_t* d_off,
                                               uint32_t* d_len, uint32_t* d_stored) {
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  uint32_t status = 0, cnt = 0;
  uint64_t pos = start;
  while (start < end && end - pos >= kLogHdr) {
    const WalHdr h = load_wal_header(a.log, a.log_len, pos);
    const uint32_t length = h.length;
    const uint32_t type = h.type;
    const bool recyc = recyclable_type(type);
    const uint32_t hs = recyc ? kLogRHdr : kLogHdr;
    if (end - pos < hs) break;
    if (hs + length > end - pos) {
      status = 2;
      break;
    }
    if (recyc && h.lognum != a.log_number) {
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
      d_stored[out_base + cnt] = crc_unmask(h.crc);  // log_reader.cc:522-523
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
    cnt = walk_block<false>(a, a.first_block + bi, &stop, 0, nullptr, nullptr, nullptr);
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

// The records of a tile's 256 log blocks are one contiguous run of the
// descriptor arrays; lane b's records are interleaved with its neighbours'
// in that run, so direct stores are partial-line writes.  When the run fits,
// the lanes write it into LDS and the workgroup stores it coalesced.
constexpr uint32_t kFillCap = 2560;  // records staged per tile (40 KiB of LDS)

__global__ void __launch_bounds__(kTile) wal_fill_kernel(WalArgs a, WalScratch s) {
  __shared__ uint32_t sh[kTile];
  __shared__ uint64_t l_off[kFillCap];
  __shared__ uint32_t l_len[kFillCap], l_st[kFillCap];
  const uint64_t bi = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  const uint32_t cnt = bi < a.n_blocks ? s.cnt[bi] : 0u;
  uint32_t tot;
  const uint32_t excl = wg_exclusive_scan(cnt, sh, &tot);
  const uint64_t wg_base = s.tile_prefix[blockIdx.x];
  const uint64_t base = wg_base + excl;
  const bool staged = tot <= kFillCap;  // workgroup-uniform
  if (bi < a.n_blocks) {
    s.base[bi] = base;
    uint32_t stop;
    if (cnt) {
      if (staged)
        walk_block<true>(a, a.first_block + bi, &stop, excl, l_off, l_len, l_st);
      else {
        walk_block<true>(a, a.first_block + bi, &stop, base, s.desc_off, s.desc_len, s.stored);
        for (uint32_t j = 0; j < cnt; ++j) s.computed[base + j] = s.stored[base + j];
      }
    }
  }
  // computed[] pre-filled with the stored CRCs (crc_records' expect: the CRC
  // kernel overwrites only the records whose CRC differs)
  if (staged) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < tot; i += kTile) {
      s.desc_off[wg_base + i] = l_off[i];
      s.desc_len[wg_base + i] = l_len[i];
      s.stored[wg_base + i] = l_st[i];
      s.computed[wg_base + i] = l_st[i];
    }
  }
}

// first failing record of the block in reader order: a CRC mismatch among the
// structurally valid records (kBadRecordChecksum, 1), else the walk's stop.
// Reads the fill's per-record arrays only (no third walk over the headers).
__global__ void __launch_bounds__(kTile) wal_status_kernel(WalArgs a, WalScratch s) {
  const uint64_t bi = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (bi >= a.n_blocks) return;
  const uint32_t cnt = s.cnt[bi];
  const uint64_t base = s.base[bi];
  const uint64_t start = (a.first_block + bi) * kLogBlock;
  uint32_t status = s.stop[bi] >> 24, pos = s.stop[bi] & 0xffffffu, nrec = cnt;
  for (uint32_t j = 0; j < cnt; ++j) {
    if (s.stored[base + j] != s.computed[base + j]) {
      status = 1;
      nrec = j;
      pos = static_cast<uint32_t>(s.desc_off[base + j] - 6 - start);
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
  if (a.payload_lengths) {  // the writer's lengths (forst_wal_record_crc_lengths)
    const uint32_t hs = a.recyclable ? kLogRHdr : kLogHdr;
    const uint32_t length = a.payload_lengths[i];
    if (off <= a.log_len && a.log_len - off >= uint64_t(hs) + length) {
      o = off + 6;
      n = hs + length - 6;
    }
  } else if (off <= a.log_len && a.log_len - off >= kLogHdr) {
    const WalHdr h = load_wal_header(a.log, a.log_len, off);
    const uint32_t hs = recyclable_type(h.type) ? kLogRHdr : kLogHdr;
    if (a.log_len - off >= uint64_t(hs) + h.length) {
      o = off + 6;
      n = hs + h.length - 6;
    }
  }
  d_off[i] = o;
  d_len[i] = n;
}

// the in-place stores of the lengths path: validity from the arrays (the rows
// kernel's rule, stream_common.h load_batch), the masked CRCs from it
__global__ void __launch_bounds__(kTile) wal_rec_store_kernel(WalArgs a, const uint32_t* crc) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i >= a.n_records) return;
  const uint64_t off = a.header_offsets[i];
  const uint32_t hs = a.recyclable ? kLogRHdr : kLogHdr;
  if (off <= a.log_len && a.log_len - off >= uint64_t(hs) + a.payload_lengths[i])
    st_le32(a.log_w + off, crc[i]);
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

// ---- a14: XXH3 of logical records (log_reader.cc:95-165) --------------------
// A logical record is a kFullType fragment, or kFirstType + kMiddleType* +
// kLastType; the reader hashes it with XXH3_64bits (full) or the streaming API
// over the fragments (= XXH3_64bits of their concatenation).  wal_hash.h hashes
// them in place across the fragment headers (a writer's layout) or from a
// gathered copy (anything else).

__device__ __forceinline__ uint32_t norm_type(uint32_t t) {  // recyclable -> legacy
  return (t >= 5 && t <= 8) ? t - 4 : t;
}

struct FragInfo {
  uint64_t off;  // payload offset in the log
  uint32_t len, type;
  bool ok;
};

__device__ __forceinline__ FragInfo frag_info(const WalArgs& a, uint64_t i) {
  FragInfo f{0, 0, 0, false};
  const uint64_t off = a.header_offsets[i];
  if (off <= a.log_len && a.log_len - off >= kLogHdr) {
    const WalHdr h = load_wal_header(a.log, a.log_len, off);
    const uint32_t hs = recyclable_type(h.type) ? kLogRHdr : kLogHdr;
    if (a.log_len - off >= uint64_t(hs) + h.length) {
      f.off = off + hs;
      f.len = h.length;
      f.type = norm_type(h.type);
      f.ok = f.type >= 1 && f.type <= 4;
    }
  }
  return f;
}

// start flags (kFullType / kFirstType) and each fragment's header fields,
// packed (length | type << 16 | ok << 20 | recyclable << 21): the one pass
// over the headers; the later kernels read the packed word
__global__ void __launch_bounds__(kTile) rec_start_kernel(WalArgs a, uint64_t* start,
                                                          uint32_t* pinfo) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i >= a.n_records) return;
  const FragInfo f = frag_info(a, i);
  start[i] = f.ok && (f.type == 1 || f.type == 2) ? 1 : 0;
  pinfo[i] = f.ok ? (f.len | (f.type << 16) | (1u << 20) |
                     (f.off - a.header_offsets[i] == kLogRHdr ? 1u << 21 : 0u))
                  : 0u;
}

// per logical record: first fragment and kind
__global__ void __launch_bounds__(kTile) rec_owner_kernel(WalArgs a, const uint64_t* start,
                                                          const uint32_t* pinfo,
                                                          const uint64_t* lid_excl,
                                                          uint64_t* first_phys, uint8_t* kind) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i >= a.n_records) return;
  if (start[i]) {
    first_phys[lid_excl[i]] = i;
    kind[lid_excl[i]] = static_cast<uint8_t>((pinfo[i] >> 16) & 15u);
  }
}

// the fragments of logical record j (wal_hash.h accessor): a kFullType
// record is its start fragment; a kFirstType record owns every valid
// fragment up to the next start
struct A14Frags {
  WalArgs a;
  const uint64_t* first;
  const uint8_t* kind;
  const uint32_t* pinfo;
  uint64_t n_logical;
  __device__ uint64_t begin(uint64_t j) const { return first[j]; }
  __device__ uint64_t end(uint64_t j) const {
    if (kind[j] == 1) return first[j] + 1;
    return j + 1 < n_logical ? first[j + 1] : a.n_records;
  }
  __device__ uint64_t header(uint64_t q) const { return a.header_offsets[q]; }
  __device__ uint32_t hs(uint64_t q) const { return (pinfo[q] >> 21) & 1u ? kLogRHdr : kLogHdr; }
  __device__ uint32_t len(uint64_t q) const { return pinfo[q] & 0xffffu; }
  __device__ bool use(uint64_t q) const { return (pinfo[q] >> 20) & 1u; }
};

#ifdef FORST_DIAG
// ---- raw CRC of a record list split by size (A/B variant) -------------------
// WAL records span 7 B .. 32 KiB: with FORST_WAL_SPLIT=1 small ones go to the
// rows kernel (one record per 16-lane row), large ones to the v2 kernel (one
// per wave), results scattered back in record order.  Measured slower than
// one rows launch over all records (C5 0.478 vs 0.499), so not the default.
constexpr uint32_t kSplitBytes = 8192;

__global__ void __launch_bounds__(kTile) split_flag_kernel(const uint32_t* len, uint64_t n,
                                                           uint64_t* flag) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i < n) flag[i] = len[i] < kSplitBytes ? 1 : 0;
}

__global__ void __launch_bounds__(kTile) split_compact_kernel(
    const uint64_t* off, const uint32_t* len, uint64_t n, const uint64_t* flag,
    const uint64_t* pos, uint64_t* s_off, uint32_t* s_len, uint64_t* b_off, uint32_t* b_len) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i >= n) return;
  if (flag[i]) {
    s_off[pos[i]] = off[i];
    s_len[pos[i]] = len[i];
  } else {
    b_off[i - pos[i]] = off[i];
    b_len[i - pos[i]] = len[i];
  }
}

__global__ void __launch_bounds__(kTile) split_scatter_kernel(uint64_t n, const uint64_t* flag,
                                                              const uint64_t* pos,
                                                              const uint32_t* s_out,
                                                              const uint32_t* b_out,
                                                              uint32_t* out) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x;
  if (i < n) out[i] = flag[i] ? s_out[pos[i]] : b_out[i - pos[i]];
}

#endif  // FORST_DIAG

size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

#ifdef FORST_DIAG
// diagnostics build: FORST_WAL_VARIANT=wave selects the one-wave-per-log-block
// kernels (crc32c.hip), the A/B reference of this pipeline
bool wave_variant() { return std::string(diag_env("FORST_WAL_VARIANT")) == "wave"; }
#endif

}  // namespace

namespace {

// out[i] = crc32c::Extend(0, base + off[i], len[i]) for a record list
// (FORST_WAL_SPLIT=1: split by size between the rows and v2 kernels)
#ifndef FORST_WAL_EXPECT
#define FORST_WAL_EXPECT 1
#endif
hipError_t crc_records(const uint8_t* base, uint64_t base_len, const uint64_t* off,
                       const uint32_t* len, uint64_t n, uint32_t* out, hipStream_t stream,
                       const char** name, const uint32_t* expect = nullptr) {
  BlockArgs b{};
  b.base = base;
  b.base_len = base_len;
  b.offsets = off;
  b.sizes = len;
  b.out32 = out;
  b.n = n;
  b.expect = expect;  // (out pre-filled with it)
  // default: one launch (the rows kernel for this size mix); the split is an
  // A/B variant (C5: 0.499 one launch vs 0.478 split, tools/wal_ab.py)
#ifndef FORST_DIAG
  return launch_crc32c_blocks(kModeRaw, b, stream, name);
#else
  if (std::string(diag_env("FORST_WAL_SPLIT")) != "1")
    return launch_crc32c_blocks(kModeRaw, b, stream, name);
  const uint64_t nt = (n + kTile - 1) / kTile;
  const dim3 grid(static_cast<uint32_t>(nt));
  const size_t s8 = up256(8 * n), s4 = up256(4 * n), st = up256(8 * (nt + 1));
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, 4 * s8 + 4 * s4 + st, stream);
  if (e != hipSuccess) return e;
  uint8_t* p = static_cast<uint8_t*>(scratch);
  uint64_t* flag = reinterpret_cast<uint64_t*>(p);
  uint64_t* pos = reinterpret_cast<uint64_t*>(p + s8);
  uint64_t* s_off = reinterpret_cast<uint64_t*>(p + 2 * s8);
  uint64_t* b_off = reinterpret_cast<uint64_t*>(p + 3 * s8);
  uint32_t* s_len = reinterpret_cast<uint32_t*>(p + 4 * s8);
  uint32_t* b_len = reinterpret_cast<uint32_t*>(p + 4 * s8 + s4);
  uint32_t* s_out = reinterpret_cast<uint32_t*>(p + 4 * s8 + 2 * s4);
  uint32_t* b_out = reinterpret_cast<uint32_t*>(p + 4 * s8 + 3 * s4);
  uint64_t* tiles = reinterpret_cast<uint64_t*>(p + 4 * s8 + 4 * s4);
  hipLaunchKernelGGL(split_flag_kernel, grid, dim3(kTile), 0, stream, len, n, flag);
  scan_u64(flag, n, tiles, pos, stream);
  const uint64_t nst = (n + kScanTile - 1) / kScanTile;
  uint64_t n_small = 0;
  if ((e = hipMemcpyAsync(&n_small, tiles + nst, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess) {
    (void)scratch_free(scratch, stream);
    return e;
  }
  hipLaunchKernelGGL(split_compact_kernel, grid, dim3(kTile), 0, stream, off, len, n, flag, pos,
                     s_off, s_len, b_off, b_len);
  if (n_small) {
    BlockArgs bs = b;
    bs.offsets = s_off;
    bs.sizes = s_len;
    bs.out32 = s_out;
    bs.n = n_small;
    bs.kernel_hint = 1;
    e = launch_crc32c_blocks(kModeRaw, bs, stream, name);
  }
  if (e == hipSuccess && n_small < n) {
    BlockArgs bb = b;
    bb.offsets = b_off;
    bb.sizes = b_len;
    bb.out32 = b_out;
    bb.n = n - n_small;
    bb.kernel_hint = 2;
    e = launch_crc32c_blocks(kModeRaw, bb, stream, name);
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(split_scatter_kernel, grid, dim3(kTile), 0, stream, n, flag, pos, s_out,
                       b_out, out);
    e = hipGetLastError();
  }
  const hipError_t f = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f;
#endif  // FORST_DIAG
}

}  // namespace

hipError_t launch_wal_verify(const WalArgs& a, hipStream_t stream, const char** name) {
  if (a.n_blocks == 0) return hipSuccess;
#ifdef FORST_DIAG
  if (wave_variant()) return launch_wal_verify_wave(a, stream, name);
#endif
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
  if ((e = scratch_alloc(&desc, sz_off + 3 * sz_len, stream)) != hipSuccess) {
    (void)scratch_free(scratch, stream);
    return e;
  }
  s.desc_off = static_cast<uint64_t*>(desc);
  s.desc_len = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(desc) + sz_off);
  s.computed = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(desc) + sz_off + sz_len);
  s.stored = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(desc) + sz_off + 2 * sz_len);
  hipLaunchKernelGGL(wal_fill_kernel, grid, dim3(kTile), 0, stream, a, s);
  *name = "wal_walk_kernel";
  // computed[] arrives pre-filled with the stored CRCs (wal_fill_kernel):
  // the CRC kernel writes only the records whose CRC differs
  if (total)
    e = crc_records(a.log, a.log_len, s.desc_off, s.desc_len, total, s.computed, stream, name,
                    FORST_WAL_EXPECT ? s.stored : nullptr);
  hipLaunchKernelGGL(wal_status_kernel, grid, dim3(kTile), 0, stream, a, s);
  if (e == hipSuccess) e = hipGetLastError();
  const hipError_t f1 = scratch_free(desc, stream), f2 = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f1 != hipSuccess ? f1 : f2;
}

hipError_t launch_wal_record_crc(const WalArgs& a, hipStream_t stream, const char** name) {
  if (a.n_records == 0) return hipSuccess;
#ifdef FORST_DIAG
  if (wave_variant()) return launch_wal_record_crc_wave(a, stream, name);
#endif
  const size_t n = a.n_records;
  // the lengths given (the writer's own, forst_wal_record_crc_lengths): the
  // rows kernel takes header offsets and payload lengths as its descriptors,
  // masks the CRCs and stores them in place itself -- no descriptor pass over
  // the headers, no finish pass (C5 writer: 0.35 + 0.50 ms of scattered
  // header reads and writes in separate kernels)
  if (a.payload_lengths && a.log_len >= 4096 && n < 0xffffffffull) {
    uint32_t* crc = a.crc_out;
    void* scratch = nullptr;
    if (!crc && a.write_in_place) {
      hipError_t e = scratch_alloc(&scratch, up256(4 * n), stream);
      if (e != hipSuccess) return e;
      crc = static_cast<uint32_t*>(scratch);
    }
    BlockArgs b{};
    b.base = a.log;
    b.base_len = a.log_len;
    b.offsets = a.header_offsets;
    b.sizes = a.payload_lengths;
    b.out32 = crc;
    b.n = n;
    b.kernel_hint = 1;  // the rows kernel (its WAL writer mode)
    b.wal_hs = a.recyclable ? kLogRHdr : kLogHdr;
    hipError_t e = launch_crc32c_blocks(kModeRaw, b, stream, name);
    if (e == hipSuccess && a.write_in_place) {
      hipLaunchKernelGGL(wal_rec_store_kernel, dim3(static_cast<uint32_t>((n + kTile - 1) / kTile)),
                         dim3(kTile), 0, stream, a, crc);
      e = hipGetLastError();
    }
    const hipError_t f = scratch ? scratch_free(scratch, stream) : hipSuccess;
    return e != hipSuccess ? e : f;
  }
  const size_t sz_off = up256(8 * n), sz_len = up256(4 * n);
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, sz_off + 2 * sz_len, stream);
  if (e != hipSuccess) return e;
  uint64_t* d_off = static_cast<uint64_t*>(scratch);
  uint32_t* d_len = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + sz_off);
  uint32_t* comp = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + sz_off + sz_len);
  const dim3 grid(static_cast<uint32_t>((n + kTile - 1) / kTile));
  hipLaunchKernelGGL(wal_rec_desc_kernel, grid, dim3(kTile), 0, stream, a, d_off, d_len);
  e = crc_records(a.log, a.log_len, d_off, d_len, n, comp, stream, name);
  hipLaunchKernelGGL(wal_rec_finish_kernel, grid, dim3(kTile), 0, stream, a, d_len, comp);
  if (e == hipSuccess) e = hipGetLastError();
  const hipError_t f = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f;
}

}  // namespace forst

namespace forst {

hipError_t launch_wal_record_xxh3(const WalArgs& a, uint64_t* out, uint64_t* out_first,
                                  uint64_t* n_logical_host, hipStream_t stream,
                                  const char** name) {
  *n_logical_host = 0;
  if (a.n_records == 0) return hipSuccess;
  const uint64_t n = a.n_records, nt = (n + kTile - 1) / kTile;
  const dim3 grid(static_cast<uint32_t>(nt));
  // scratch: start, lid, first_phys (u64 x n; the caller's out_first when
  // given), kind (u8 x n), packed header fields (u32 x n), tile sums
  const size_t s8 = up256(8 * n), s1 = up256(n), s4 = up256(4 * n), st = up256(8 * (nt + 2));
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, 3 * s8 + s1 + s4 + st, stream);
  if (e != hipSuccess) return e;
  uint8_t* p = static_cast<uint8_t*>(scratch);
  uint64_t* start = reinterpret_cast<uint64_t*>(p);
  uint64_t* lid = reinterpret_cast<uint64_t*>(p + s8);
  uint64_t* first = out_first ? out_first : reinterpret_cast<uint64_t*>(p + 2 * s8);
  uint8_t* kind = p + 3 * s8;
  uint32_t* pinfo = reinterpret_cast<uint32_t*>(p + 3 * s8 + s1);
  uint64_t* tiles = reinterpret_cast<uint64_t*>(p + 3 * s8 + s1 + s4);
  hipLaunchKernelGGL(rec_start_kernel, grid, dim3(kTile), 0, stream, a, start, pinfo);
  scan_u64(start, n, tiles, lid, stream);
  hipLaunchKernelGGL(rec_owner_kernel, grid, dim3(kTile), 0, stream, a, start, pinfo, lid, first,
                     kind);
  uint64_t n_logical = 0;
  if ((e = hipMemcpyAsync(&n_logical, tiles + (n + kScanTile - 1) / kScanTile, 8,
                          hipMemcpyDeviceToHost, stream)) != hipSuccess ||
      (e = hipStreamSynchronize(stream)) != hipSuccess) {
    (void)scratch_free(scratch, stream);
    return e;
  }
  if (n_logical) {
    const A14Frags f{a, first, kind, pinfo, n_logical};
    e = hash_logical_records(a.log, a.log_len, f, n_logical, out, stream, name);
  }
  *n_logical_host = n_logical;
  const hipError_t f1 = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f1;
}

}  // namespace forst
