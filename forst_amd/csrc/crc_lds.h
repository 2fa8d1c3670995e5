// forst_amd/csrc/crc_lds.h -- the LDS table machinery of the CRC32C kernels
// (crc32c.hip) in the form the fused WAL-recovery kernel (xxh3.hip,
// xxh3_frag_kernel<.., true>) uses: slicing tables replicated 8x so the 32
// lanes of a ds_read_b32 bank group hit 32 distinct banks, each lookup
// address one v_perm_b32 of the data word and a per-lane constant.
//
// Layout [0, 64K): row e (byte value), dword d: d < 32 -> G_{d>>3}[e] copy
// d & 7 (G = advance 4 bytes, the slicing-by-4 step), d >= 32 -> J_{..}[e]
// (J = the chain's hop to its next chunk fused with the first dword step).
// Lane l (c = l & 7, g = (l >> 3) & 3) does lookup i on table i ^ g with byte
// i ^ g of the word: address 256 * byte + 4 (8 (i ^ g) + c) [+ 128 for J].
#pragma once
#include "device_common.h"

namespace forst {
namespace fcrc {

struct Lanes {
  uint32_t lpack;   // byte i: 4 (8 (i ^ g) + c)
  uint32_t sel[4];  // v_perm selector: {0, 0, x.byte(i ^ g), lpack.byte(i)}
};

__device__ __forceinline__ Lanes lanes(uint32_t lane) {
  Lanes k;
  const uint32_t c = lane & 7, g = (lane >> 3) & 3;
  k.lpack = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    const uint32_t tt = i ^ g;
    k.lpack |= (4 * (8 * tt + c)) << (8 * i);
    k.sel[i] = 0x0c0c0000u | ((4 + tt) << 8) | i;
  }
  return k;
}

__device__ __forceinline__ uint32_t lds32(const uint8_t* __restrict__ Lb, uint32_t addr) {
  return *reinterpret_cast<const uint32_t*>(Lb + addr);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// the four table reads of G(x) (J = false) or J(x) (J = true)
template <bool J>
__device__ __forceinline__ void look(const uint8_t* __restrict__ Lb, const Lanes& k, uint32_t x,
                                     uint32_t (&l)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    l[i] = lds32(Lb, __builtin_amdgcn_perm(x, k.lpack, k.sel[i]) + (J ? 128u : 0u));
}

// G(x) ^ e: the next chain input when e is the next data word
__device__ __forceinline__ uint32_t g_then(const uint8_t* __restrict__ Lb, const Lanes& k,
                                           uint32_t x, uint32_t e) {
  uint32_t l[4];
  look<false>(Lb, k, x, l);
  return xor3(l[0], l[1], xor3(l[2], l[3], e));
}

// one 16-byte chunk after a gap: state' = G(J'(s) ^ w0 ...) with the hop
// fused into the first step, i.e. J(s) ^ G(w0) then three dword steps
__device__ __forceinline__ uint32_t chunk_step(const uint8_t* __restrict__ Lb, const Lanes& k,
                                               uint32_t s, uint32_t w0, uint32_t w1, uint32_t w2,
                                               uint32_t w3) {
  uint32_t lj[4], lg[4];
  look<true>(Lb, k, s, lj);
  look<false>(Lb, k, w0, lg);
  uint32_t x = xor3(xor3(lj[0], lj[1], lj[2]), xor3(lj[3], lg[0], lg[1]), xor3(lg[2], lg[3], w1));
  x = g_then(Lb, k, x, w2);
  x = g_then(Lb, k, x, w3);
  return g_then(Lb, k, x, 0u);
}

// the mask of dword i of a 16-byte chunk whose first n bytes are kept (n >=
// 16: all): the high word of 0xffffffff << 8 clamp(n - 4 i, 0, 4)
__device__ __forceinline__ uint32_t keep_word(uint32_t n, uint32_t i) {
  const uint32_t b = n > 4 * i ? (n - 4 * i < 4u ? n - 4 * i : 4u) : 0u;
  return static_cast<uint32_t>((0xffffffffull << (8 * b)) >> 32);
}

// linear shift through an unreplicated 4 x 256 table at byte offset b
__device__ __forceinline__ uint32_t shift_at(const uint8_t* __restrict__ Lb, uint32_t b,
                                             uint32_t v) {
  return lds32(Lb, b + ((v & 0xffu) << 2)) ^ lds32(Lb, b + 1024 + (((v >> 8) & 0xffu) << 2)) ^
         lds32(Lb, b + 2048 + (((v >> 16) & 0xffu) << 2)) ^ lds32(Lb, b + 3072 + ((v >> 24) << 2));
}

// XOR of the 16 lanes of each row, valid in every lane of the row (DPP row_ror)
template <int N>
__device__ __forceinline__ uint32_t row_ror_xor(uint32_t v) {
  return v ^ static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x120 + N,
                                                               0xf, 0xf, false));
}

// bytes [a, b) of a 16-byte chunk kept (0 <= a <= b <= 16): the masks of its
// two little-endian 64-bit halves
__device__ __forceinline__ uint64_t keep64(uint32_t n) {  // low n bytes, n <= 8
  return n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1);
}
__device__ __forceinline__ void keep_mask(uint32_t a, uint32_t b, uint64_t& lo, uint64_t& hi) {
  const uint32_t a0 = a < 8 ? a : 8, b0 = b < 8 ? b : 8;
  const uint32_t a1 = a > 8 ? a - 8 : 0, b1 = b > 8 ? b - 8 : 0;
  lo = keep64(b0) & ~keep64(a0);
  hi = keep64(b1) & ~keep64(a1);
}

}  // namespace fcrc
}  // namespace forst
