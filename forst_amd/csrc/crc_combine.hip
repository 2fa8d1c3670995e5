// forst_amd/csrc/crc_combine.hip -- crc32c::Crc32cCombine (util/crc32c.cc:1279)
// and whole-buffer CRC32C on the device.
//
// CRC32C with its pre/post conditioning is affine, and the conditioning
// cancels in the combine identity
//     crc(A || B) = M(|B|) * crc(A) ^ crc(B),   M(n) = x^(8n) mod P
// (GF(2) product in the reflected domain; the reference computes the same
// thing with gf_multiply_sw over crc32c_powers, crc32c.cc:1143-1279).  Folding
// it over chunks gives the parallel form used here:
//     Extend(init, C_0 || ... || C_{k-1})
//         = M(total) * init  ^  XOR_i M(after_i) * Value(C_i)
// so a whole buffer is one raw batch over 64 KiB chunks (the block kernels,
// at streaming rate) plus one lane per chunk shifting its CRC to the end of
// the buffer and an XOR reduction -- used by FileChecksumGenCrc32c
// (util/file_checksum_helper.h:22) and the WritableFileWriter handoff CRC
// (file/writable_file_writer.cc:100-212) style chained CRCs.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/forst_checksum.h"
#include "crc32c_tables.h"
#include "device_common.h"
#include "engine.h"

namespace forst {
namespace {

constexpr uint32_t kPoly = 0x82f63b78u;  // util/crc32c.cc (reflected Castagnoli)
constexpr uint32_t kCombThreads = 256;
constexpr uint64_t kChunk = 65536;

// a * b mod P, reflected (bit 31 = x^0)
__host__ __device__ inline uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= (a & 0x80000000u) ? b : 0u;
    a <<= 1;
    b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
  }
  return p;
}

// M(n) = x^(8n) mod P from the powers x^(8 * 2^k) (kCrcX8Pow)
__device__ inline uint32_t x8n_dev(uint64_t n) {
  uint32_t r = 0x80000000u;  // x^0
  for (int k = 0; n; ++k, n >>= 1)
    if (n & 1) r = gf_mul(r, kCrcX8Pow[k]);
  return r;
}

inline uint32_t x8n_host(uint64_t n) {
  uint32_t r = 0x80000000u, sq = 0x00800000u;  // x^0, x^8
  for (; n; n >>= 1) {
    if (n & 1) r = gf_mul(r, sq);
    sq = gf_mul(sq, sq);
  }
  return r;
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
  for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m);
  return v;
}

__global__ void __launch_bounds__(kCombThreads)
    combine_batch_kernel(const uint32_t* crc1, const uint32_t* crc2, const uint64_t* len2,
                         uint32_t* out, uint64_t n) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kCombThreads + threadIdx.x;
  if (i < n) out[i] = gf_mul(x8n_dev(len2[i]), crc1[i]) ^ crc2[i];
}

__global__ void __launch_bounds__(kCombThreads)
    chunk_desc_kernel(uint64_t len, uint64_t n_chunks, uint64_t* offs, uint32_t* sizes) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kCombThreads + threadIdx.x;
  if (i >= n_chunks) return;
  offs[i] = i * kChunk;
  sizes[i] = static_cast<uint32_t>(i + 1 < n_chunks ? kChunk : len - i * kChunk);
}

// out ^= XOR_i M(after_i) * crc_i (+ M(total) * init from lane 0 of block 0);
// *out is zeroed on the stream before the launch
__global__ void __launch_bounds__(kCombThreads)
    chunk_fold_kernel(const uint32_t* crcs, uint64_t len, uint64_t n_chunks, uint32_t init,
                      uint32_t* out) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kCombThreads + threadIdx.x;
  uint32_t v = 0;
  if (i < n_chunks) {
    const uint64_t end = i + 1 < n_chunks ? (i + 1) * kChunk : len;
    v = gf_mul(x8n_dev(len - end), crcs[i]);
  }
  if (i == 0) v ^= gf_mul(x8n_dev(len), init);
  v = wave_xor(v);
  if ((threadIdx.x & 63) == 0 && v) atomicXor(out, v);
}

}  // namespace

hipError_t launch_crc32c_combine_batch(const uint32_t* crc1, const uint32_t* crc2,
                                       const uint64_t* len2, uint32_t* out, uint64_t n,
                                       hipStream_t stream, const char** name) {
  if (n == 0) return hipSuccess;
  *name = "combine_batch_kernel";
  hipLaunchKernelGGL(combine_batch_kernel, dim3(static_cast<uint32_t>((n + kCombThreads - 1) / kCombThreads)),
                     dim3(kCombThreads), 0, stream, crc1, crc2, len2, out, n);
  return hipGetLastError();
}

hipError_t launch_crc32c_buffer(const uint8_t* base, uint64_t len, uint32_t init, uint32_t* out,
                                hipStream_t stream, const char** name) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  const uint64_t nc = (len + kChunk - 1) / kChunk;
  const dim3 grid(static_cast<uint32_t>(nc ? (nc + kCombThreads - 1) / kCombThreads : 1));
  if (nc == 0) {  // Extend(init, "") = init
    hipLaunchKernelGGL(chunk_fold_kernel, grid, dim3(kCombThreads), 0, stream, nullptr,
                       uint64_t(0), uint64_t(0), init, out);
    *name = "chunk_fold_kernel";
    return hipGetLastError();
  }
  void* scratch = nullptr;
  const size_t so = (8 * nc + 255) & ~size_t(255), ss = (4 * nc + 255) & ~size_t(255);
  if ((e = scratch_alloc(&scratch, so + 2 * ss, stream)) != hipSuccess) return e;
  uint64_t* offs = static_cast<uint64_t*>(scratch);
  uint32_t* sizes = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + so);
  uint32_t* crcs = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + so + ss);
  hipLaunchKernelGGL(chunk_desc_kernel, grid, dim3(kCombThreads), 0, stream, len, nc, offs, sizes);
  BlockArgs b{};
  b.base = base;
  b.base_len = len;
  b.offsets = offs;
  b.sizes = sizes;
  b.out32 = crcs;
  b.n = nc;
  e = launch_crc32c_blocks(kModeRaw, b, stream, name);
  hipLaunchKernelGGL(chunk_fold_kernel, grid, dim3(kCombThreads), 0, stream, crcs, len, nc, init,
                     out);
  if (e == hipSuccess) e = hipGetLastError();
  const hipError_t f = scratch_free(scratch, stream);
  return e != hipSuccess ? e : f;
}

}  // namespace forst

// host: crc32c::Crc32cCombine (util/crc32c.h:32), no GPU involved
extern "C" __attribute__((visibility("default"))) uint32_t forst_crc32c_combine(uint32_t crc1,
                                                                                uint32_t crc2,
                                                                                uint64_t len2) {
  return forst::gf_mul(forst::x8n_host(len2), crc1) ^ crc2;
}
