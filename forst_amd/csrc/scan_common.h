// forst_amd/csrc/scan_common.h -- device-wide exclusive prefix sum of u64
// values, shared by the WAL pipelines and the a15 block walk: three passes
// (tile sums, one-workgroup scan of the tile sums, tile-local scans plus the
// tile prefix); a one-pass decoupled look-back form (round 6) is the A/B
// knob FORST_SCAN_LOOKBACK.
//
// A tile is 2048 values (256 threads x 8): the one-workgroup middle pass then
// sees n / 2048 tile sums (5.6 K for C5's 11.4 M records, one sequential run
// of 6 per thread and one block scan) instead of 44 K 256-value tiles in 44
// barrier-bound rounds (72 us -> a few us per scan); in-tile scans are wave
// shuffles plus one LDS exchange of the four wave totals.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace forst {
namespace {

constexpr uint32_t kScanWg = 256;
constexpr uint32_t kScanItems = 8;
constexpr uint32_t kScanTile = kScanWg * kScanItems;
constexpr uint32_t kScanTop = 1024;

__device__ __forceinline__ uint64_t scan_shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl(static_cast<uint32_t>(v), src);
  const uint32_t hi = __shfl(static_cast<uint32_t>(v >> 32), src);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// inclusive scan of v over the wave (64 lanes)
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
  const int lane = static_cast<int>(threadIdx.x & 63);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t u = scan_shfl64(v, lane >= d ? lane - d : lane);
    v += lane >= d ? u : 0ull;
  }
  return v;
}

// exclusive scan of one value per thread over the workgroup (nthreads a
// multiple of 64, <= 1024); *total = the workgroup's sum
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* wsum,
                                                      uint64_t* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t incl = wave_incl_scan64(v);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (uint32_t k = 0; k < nw; ++k) {
    const uint64_t s = wsum[k];
    before += k < w ? s : 0ull;
    all += s;
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

__global__ void __launch_bounds__(kScanWg) scan_tiles_kernel(const uint64_t* in, uint64_t n,
                                                              uint64_t* tile_sum) {
  __shared__ uint64_t wsum[kScanWg / 64];
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kScanTile;
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {  // coalesced: thread t reads t, t + 256, ...
    const uint64_t i = t0 + k * kScanWg + threadIdx.x;
    s += i < n ? in[i] : 0ull;
  }
  uint64_t tot;
  (void)block_excl_scan64(s, wsum, &tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

// one workgroup: tile_sum[0..n_tiles) -> exclusive prefix in place,
// tile_sum[n_tiles] = total; thread t owns a run of consecutive tiles
__global__ void __launch_bounds__(kScanTop) scan_top_kernel(uint64_t* tile_sum,
                                                            uint64_t n_tiles) {
  __shared__ uint64_t wsum[kScanTop / 64];
  const uint64_t per = (n_tiles + kScanTop - 1) / kScanTop;
  const uint64_t b = threadIdx.x * per;
  const uint64_t e = b + per < n_tiles ? b + per : n_tiles;
  uint64_t s = 0;
  for (uint64_t i = b; i < e; ++i) s += tile_sum[i];
  uint64_t tot;
  uint64_t run = block_excl_scan64(s, wsum, &tot);
  for (uint64_t i = b; i < e; ++i) {
    const uint64_t v = tile_sum[i];
    tile_sum[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) tile_sum[n_tiles] = tot;
}

__global__ void __launch_bounds__(kScanWg) scan_apply_kernel(const uint64_t* in, uint64_t n,
                                                              const uint64_t* tile_prefix,
                                                              uint64_t* out) {
  __shared__ uint64_t sh[kScanTile];
  __shared__ uint64_t wsum[kScanWg / 64];
  const uint32_t t = threadIdx.x;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kScanTile;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {  // coalesced load into tile order
    const uint64_t i = t0 + k * kScanWg + t;
    sh[k * kScanWg + t] = i < n ? in[i] : 0ull;
  }
  __syncthreads();
  uint64_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {  // thread t: tile items [8t, 8t + 8)
    v[k] = sh[kScanItems * t + k];
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = tile_prefix[blockIdx.x] + block_excl_scan64(s, wsum, &tot);
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    sh[kScanItems * t + k] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    const uint64_t i = t0 + k * kScanWg + t;
    if (i < n) out[i] = sh[k * kScanWg + t];
  }
}

// Single pass (round 6, FORST_SCAN_LOOKBACK): each workgroup claims the next tile id from a
// counter, scans its tile, publishes its aggregate and looks back over the
// earlier tiles' published words until one holds an inclusive prefix
// (decoupled look-back).  A tile's word is [flag:2 | value:62]: 0 = nothing
// yet, 1 = the tile's own sum, 2 = the sum of everything up to and including
// the tile (values are counts and byte lengths, far below 2^62).  Ids come
// from the counter, not blockIdx, so a waiting tile only waits for tiles
// that were claimed -- i.e. are running -- before it.  The counter is
// tiles[n_tiles], where the total goes: the tile that claims the last id
// writes the total there at its end, after every claim was made.  The input
// is read once (the three-pass form read it twice) in one launch (after a
// memset of the words) instead of three.
constexpr uint64_t kScanFlagAgg = 1ull << 62, kScanFlagInc = 2ull << 62;
constexpr uint64_t kScanMask = (1ull << 62) - 1;

__device__ __forceinline__ void scan_word_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t scan_word_load(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kScanWg) scan_lookback_kernel(const uint64_t* in, uint64_t n,
                                                                 uint64_t* tiles, uint64_t n_tiles,
                                                                 uint64_t* out) {
  __shared__ uint64_t sh[kScanTile];
  __shared__ uint64_t wsum[kScanWg / 64];
  __shared__ uint64_t s_tile, s_prefix;
  const uint32_t t = threadIdx.x;
  if (t == 0) s_tile = atomicAdd(reinterpret_cast<unsigned long long*>(tiles + n_tiles), 1ull);
  __syncthreads();
  const uint64_t tile = s_tile;
  const uint64_t t0 = tile * kScanTile;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {  // coalesced load into tile order
    const uint64_t i = t0 + k * kScanWg + t;
    sh[k * kScanWg + t] = i < n ? in[i] : 0ull;
  }
  __syncthreads();
  uint64_t v[kScanItems];
  uint64_t sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {  // thread t: tile items [8t, 8t + 8)
    v[k] = sh[kScanItems * t + k];
    sum += v[k];
  }
  uint64_t agg;
  const uint64_t excl = block_excl_scan64(sum, wsum, &agg);
  if (t == 0) scan_word_store(tiles + tile, (tile == 0 ? kScanFlagInc : kScanFlagAgg) | agg);
  if (t < 64) {
    // wave 0 looks back 64 tiles at a time: lane l reads tile base - l (a
    // word in front of tile 0 counts as an inclusive 0); the nearest
    // inclusive word ends the walk, else the window's 64 sums are added and
    // it moves back (bounded waits: a word that never appears ends the walk
    // with a wrong sum, which the callers' checks report, not a hung GPU)
    uint64_t prefix = 0;
    for (int64_t base = static_cast<int64_t>(tile) - 1; base >= 0; base -= 64) {
      const int64_t j = base - static_cast<int64_t>(t);
      uint64_t w = j >= 0 ? scan_word_load(tiles + j) : kScanFlagInc;
      for (uint32_t spin = 0; (w >> 62) == 0 && spin < (1u << 22); ++spin) {
        __builtin_amdgcn_s_sleep(1);
        w = scan_word_load(tiles + j);
      }
      const uint64_t inc = __ballot((w >> 62) == 2);
      const uint32_t stop = inc ? static_cast<uint32_t>(__ffsll(static_cast<long long>(inc)) - 1) : 64u;
      uint64_t x = t <= stop ? (w & kScanMask) : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = __shfl_xor(static_cast<uint32_t>(x), o);
        const uint32_t hi = __shfl_xor(static_cast<uint32_t>(x >> 32), o);
        x += (static_cast<uint64_t>(hi) << 32) | lo;
      }
      prefix += x;
      if (inc) break;
    }
    if (t == 0) {
      if (tile != 0) scan_word_store(tiles + tile, kScanFlagInc | (prefix + agg));
      if (tile == n_tiles - 1) scan_word_store(tiles + n_tiles, prefix + agg);  // the total
      s_prefix = prefix;
    }
  }
  __syncthreads();
  uint64_t run = s_prefix + excl;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    sh[kScanItems * t + k] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; ++k) {
    const uint64_t i = t0 + k * kScanWg + t;
    if (i < n) out[i] = sh[k * kScanWg + t];
  }
}

// Default: the three-pass form.  The single pass above is correct (the
// whole -m gpu suite and the full-size WAL / recovery tests pass through it)
// but measured slower: C5 recovery, ten scans of up to 11.4 M values, 17.72
// ms against 17.20-17.53 ms with the three passes, a14 alike
// (profiles/ab_r06/scan_lookback_r06.log, one box, three alternations).
#ifndef FORST_SCAN_LOOKBACK
#define FORST_SCAN_LOOKBACK 0  // (A/B knob)
#endif

// out[i] = sum(in[0..i)); tiles (n_tiles + 1 entries) ends with the total.
// Callers size `tiles` as n / kScanTile + 2.
inline void scan_u64(const uint64_t* in, uint64_t n, uint64_t* tiles, uint64_t* out,
                     hipStream_t st) {
  const uint64_t nt = (n + kScanTile - 1) / kScanTile;
  if (FORST_SCAN_LOOKBACK) {
    (void)hipMemsetAsync(tiles, 0, 8 * (nt + 1), st);
    if (nt)
      hipLaunchKernelGGL(scan_lookback_kernel, dim3(static_cast<uint32_t>(nt)), dim3(kScanWg), 0, st,
                         in, n, tiles, nt, out);
    return;
  }
  const dim3 grid(static_cast<uint32_t>(nt ? nt : 1));
  hipLaunchKernelGGL(scan_tiles_kernel, grid, dim3(kScanWg), 0, st, in, n, tiles);
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(kScanTop), 0, st, tiles, nt);
  hipLaunchKernelGGL(scan_apply_kernel, grid, dim3(kScanWg), 0, st, in, n, tiles, out);
}

}  // namespace
}  // namespace forst
