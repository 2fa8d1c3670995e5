// forst_amd/csrc/scan_common.h -- device-wide exclusive prefix sum of u64
// values in three passes (tile sums, one-workgroup scan of the tile sums,
// tile-local scans plus the tile prefix), shared by the WAL pipelines.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace forst {
namespace {

constexpr uint32_t kScanTile = 256;
constexpr uint32_t kScanTop = 1024;

// u64 exclusive scan in three passes: tile sums, one-workgroup scan of the
// tile sums, tile-local scans plus tile prefix
__global__ void __launch_bounds__(kScanTile) scan_tiles_kernel(const uint64_t* in, uint64_t n,
                                                           uint64_t* tile_sum) {
  __shared__ uint64_t sh[kScanTile];
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kScanTile + threadIdx.x;
  sh[threadIdx.x] = i < n ? in[i] : 0;
  __syncthreads();
  for (uint32_t d = kScanTile / 2; d >= 1; d >>= 1) {
    if (threadIdx.x < d) sh[threadIdx.x] += sh[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = sh[0];
}

__global__ void __launch_bounds__(kScanTop) scan_top_kernel(uint64_t* tile_sum,
                                                                uint64_t n_tiles) {
  __shared__ uint64_t sh[kScanTop];
  const uint32_t t = threadIdx.x;
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < n_tiles; c0 += kScanTop) {
    const uint64_t i = c0 + t;
    const uint64_t v = i < n_tiles ? tile_sum[i] : 0;
    sh[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kScanTop; d <<= 1) {
      const uint64_t add = t >= d ? sh[t - d] : 0;
      __syncthreads();
      sh[t] += add;
      __syncthreads();
    }
    if (i < n_tiles) tile_sum[i] = carry + sh[t] - v;  // in place: exclusive prefix
    carry += sh[kScanTop - 1];
    __syncthreads();
  }
  if (t == 0) tile_sum[n_tiles] = carry;
}

__global__ void __launch_bounds__(kScanTile) scan_apply_kernel(const uint64_t* in, uint64_t n,
                                                           const uint64_t* tile_prefix,
                                                           uint64_t* out) {
  __shared__ uint64_t sh[kScanTile];
  const uint32_t t = threadIdx.x;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kScanTile + t;
  const uint64_t v = i < n ? in[i] : 0;
  sh[t] = v;
  __syncthreads();
  for (uint32_t d = 1; d < kScanTile; d <<= 1) {
    const uint64_t add = t >= d ? sh[t - d] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  if (i < n) out[i] = tile_prefix[blockIdx.x] + sh[t] - v;
}


// out[i] = sum(in[0..i)); tiles (n_tiles + 1 entries) ends with the total
inline void scan_u64(const uint64_t* in, uint64_t n, uint64_t* tiles, uint64_t* out,
                     hipStream_t st) {
  const uint64_t nt = (n + kScanTile - 1) / kScanTile;
  const dim3 grid(static_cast<uint32_t>(nt ? nt : 1));
  hipLaunchKernelGGL(scan_tiles_kernel, grid, dim3(kScanTile), 0, st, in, n, tiles);
  hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(kScanTop), 0, st, tiles, nt);
  hipLaunchKernelGGL(scan_apply_kernel, grid, dim3(kScanTile), 0, st, in, n, tiles, out);
}

}  // namespace
}  // namespace forst
