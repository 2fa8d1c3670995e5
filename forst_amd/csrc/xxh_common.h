// forst_amd/csrc/xxh_common.h -- xxHash device helpers shared by the XXH3
// (xxh3.hip) and XXPH3 / Hash64 (kv_protect.hip) kernels: primes, the
// default 192-byte secret (util/xxhash.h:3644 == util/xxph3.h:920), 64x64
// multiply folds, unaligned 16-byte lane loads and the 16-lane stripe sum.
#pragma once
#include "device_common.h"

namespace forst {
namespace {

#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull

// util/xxhash.h:3644 XXH3_kSecret
__device__ __constant__ const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c,
    0xf7, 0x21, 0xad, 0x1c, 0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb,
    0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f, 0xcb, 0x79, 0xe6, 0x4e,
    0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6,
    0x81, 0x3a, 0x26, 0x4c, 0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb,
    0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3, 0x71, 0x64, 0x48, 0x97,
    0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7,
    0xc7, 0x0b, 0x4f, 0x1d, 0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31,
    0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, 0xea, 0xc5, 0xac, 0x83,
    0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26,
    0x29, 0xd4, 0x68, 0x9e, 0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc,
    0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce, 0x45, 0xcb, 0x3a, 0x8f,
    0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

__device__ __forceinline__ uint64_t sec64(uint32_t off) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 7; i >= 0; --i) v = (v << 8) | kSecret[off + i];
  return v;
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
__device__ __forceinline__ uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  const unsigned __int128 p = static_cast<unsigned __int128>(a) * b;
  return static_cast<uint64_t>(p) ^ static_cast<uint64_t>(p >> 64);
}
__device__ __forceinline__ uint64_t mul32to64(uint64_t v) {
  return static_cast<uint64_t>(static_cast<uint32_t>(v)) *
         static_cast<uint64_t>(static_cast<uint32_t>(v >> 32));
}

// 64-bit values as a register pair: built and split by bit casts, so a 64-bit
// add of two DPP moves is one v_lshl_add_u64 on the pair (the shift-or form
// made hipcc add the halves separately through zero-extended temporaries: six
// instructions per 64-bit DPP add instead of three)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) {
  u32x2 w;
  w.x = lo;
  w.y = hi;
  return __builtin_bit_cast(uint64_t, w);
}
// 16 bytes at an arbitrary address with dword-aligned loads + alignbyte.
// `m` = address & 3 (wave-uniform), q = address & ~3.
__device__ __forceinline__ void ld16u(const uint8_t* q, uint32_t m,
                                      uint64_t& d0, uint64_t& d1) {
  const u32x4a4 v = ld16_a4(q);
  uint32_t x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
  if (m) {
    const uint32_t x4 = ld4_a4(q + 16);
    x0 = __builtin_amdgcn_alignbyte(x1, x0, m);
    x1 = __builtin_amdgcn_alignbyte(x2, x1, m);
    x2 = __builtin_amdgcn_alignbyte(x3, x2, m);
    x3 = __builtin_amdgcn_alignbyte(x4, x3, m);
  }
  d0 = mk64(x0, x1);
  d1 = mk64(x2, x3);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int mask) {
  const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), mask);
  const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), mask);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  // every lane reads a live lane: no "old" operand to initialise
  const u32x2 w = __builtin_bit_cast(u32x2, v);
  return mk64(__builtin_amdgcn_mov_dpp(w.x, CTRL, 0xf, 0xf, true),
              __builtin_amdgcn_mov_dpp(w.y, CTRL, 0xf, 0xf, true));
}
// DPP row rotate (within 16-lane rows), one VALU op per half, no LDS traffic
template <int N>
__device__ __forceinline__ uint64_t row_ror64(uint64_t v) {
  return dpp64<0x120 + N>(v);
}
// the partner lane of a quad (lane ^ 1: quad_perm [1,0,3,2]; lane ^ 2:
// [2,3,0,1]) by DPP instead of ds_bpermute
template <int M>
__device__ __forceinline__ uint64_t quad_xor64(uint64_t v) {
  static_assert(M == 1 || M == 2, "quad partner");
  return dpp64<M == 1 ? 0xB1 : 0x4E>(v);
}

// sum over the 16 lanes that share L%4 (lane bits 2..5): two DPP row
// rotations, then the gfx950 cross-row swaps v_permlane16_swap /
// v_permlane32_swap (own + partner) -- all VALU, every lane gets the sum.
__device__ __forceinline__ uint64_t stripe_sum(uint64_t v) {
  v += row_ror64<4>(v);
  v += row_ror64<8>(v);
  {
    const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(v),
                                                     static_cast<uint32_t>(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(v >> 32),
                                                     static_cast<uint32_t>(v >> 32), false, false);
    v = mk64(lo[0], hi[0]) + mk64(lo[1], hi[1]);
  }
  {
    const auto lo = __builtin_amdgcn_permlane32_swap(static_cast<uint32_t>(v),
                                                     static_cast<uint32_t>(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(static_cast<uint32_t>(v >> 32),
                                                     static_cast<uint32_t>(v >> 32), false, false);
    v = mk64(lo[0], hi[0]) + mk64(lo[1], hi[1]);
  }
  return v;
}

}  // namespace
}  // namespace forst
