// forst_amd/csrc/xxh3.hip -- XXH3_64bits (xxHash 0.8.1, seed 0) block kernels
// for gfx950, one 64-lane wavefront per block.
//
// Long inputs (> 240 B, util/xxhash.h:5123-5208): each XXH3 accumulate step
// adds a per-stripe contribution to 8 u64 accumulators, and within one
// 1 KiB XXH3-block those additions commute (sums mod 2^64, xxhash.h:
// 4924-4927).  So lane L takes 16 bytes (stripe L/4, accumulator pair L%4)
// of every XXH3-block -- one fully coalesced 1 KiB global_load_dwordx4 per
// XXH3-block -- and a 4-level xor butterfly sums the 16 stripes.  The
// non-linear scramble (xxhash.h:4962-4977) is applied in order, per
// accumulator, by the lanes that own it.  Short inputs (<= 240 B) run the
// reference's length-class formulas redundantly on all lanes.
#include <cstdlib>
#include <string>

#include "crc32c_tables.h"
#include "crc_lds.h"
#include "device_common.h"
#include "engine.h"
#include "stream_common.h"
#include "xxh_common.h"

namespace forst {
namespace {

constexpr uint32_t kWaves = 4;  // 256-thread workgroups, no LDS
constexpr uint32_t kThreads = kWaves * 64;
// the rows kernel: one 12-wave workgroup per CU (3 waves per SIMD), so the
// workgroup feed (stream_common.h) balances every wave of a CU
constexpr uint32_t kRowsWaves = 12;
constexpr uint32_t kRowsThreads = kRowsWaves * 64;
// workgroup-feed batch (stream_common.h): 4 descriptors, one per row (A/B
// against 8: C3 +0.4-0.6 %, NS16X +0.7 %; 16 was 1 % slower than 8)
#ifndef FORST_XX_WG_CHUNK
#define FORST_XX_WG_CHUNK 4
#endif
constexpr uint32_t kXxWgChunk = FORST_XX_WG_CHUNK;
// block modes: results staged in LDS and stored after the loop (1) or as
// rows finish (0); the workgroup's first kXxStageW results (96 KiB: the
// kernel runs one 12-wave workgroup per CU for its registers anyway)
#ifndef FORST_XX_STAGE
#define FORST_XX_STAGE 1
#endif
constexpr uint32_t kXxStageW = 16384;
// bytes a block weighs in the workgroup ranges on top of its own (its
// set-up and finish): see wg_range.  A/B on one box, 3 alternating runs
// (profiles/ab_r05/c3s_block_cost_staging.log): C3 sorted by size (C3S)
// verify 0.758 (0) -> 0.766 (512) / 0.760 (1536) / 0.748 (4096), shuffled
// C3 0.7665 unchanged -- a range of 4 KiB blocks is slower per byte than one
// of 64 KiB blocks.  Round 5, after the staged results and the LDS keys
// (profiles/ab_r05/c3s_block_cost.log, C3 and C3S on one box): C3S verify
// 0.775 (128) / 0.787 (256) / 0.784 (512) / 0.782 (1024) / 0.780 (2048),
// trailer 0.760 / 0.773 / 0.768 / 0.764 / 0.763; C3 0.789-0.790 at all three
#ifndef FORST_XX_BLOCK_COST
#define FORST_XX_BLOCK_COST 256
#endif
// fused WAL recovery: one CRC chain per lane through its four chunks of a
// window (1: a 240-byte hop between chunks, J244, so a fragment's finish
// needs no column merge), or one chain per chunk column (0: the round-3
// form, a 1008-byte hop, J1012, and three C256 shifts in every finish)
#ifndef FORST_FRAG_ONECHAIN
#define FORST_FRAG_ONECHAIN 1
#endif
constexpr uint32_t kNC = FORST_FRAG_ONECHAIN ? 1 : 4;
// the fragment kernel's lane constants recomputed where used (1) or left to
// the compiler, which hoists and, at 168 VGPRs, spills them (0)
#ifndef FORST_FRAG_FRESH
#define FORST_FRAG_FRESH 1
#endif
// the fused CRC's byte masks (bytes of a 16-byte chunk inside the fragment)
// read from a 17-entry LDS table (1), or computed in a branch per chunk (0)
#ifndef FORST_FRAG_MASK_LDS
#define FORST_FRAG_MASK_LDS 1
#endif
#if FORST_FRAG_FRESH
#define FR(x) fresh(x)
#else
#define FR(x) (x)
#endif
// the fragment kernel (WAL records): 4-wave workgroups and the global feed
// (the workgroup feed measured 5 % slower on C5's log-uniform records)
constexpr bool kFragWg = false;
constexpr uint32_t kFragWaves = kWaves;
constexpr uint32_t kFragThreads = kFragWaves * 64;
// ... with the fused physical-record CRC (WAL recovery): 124 KiB of CRC
// tables in LDS, so one 12-wave workgroup per CU
#ifndef FORST_FRAG_CRC_WAVES
#define FORST_FRAG_CRC_WAVES (FORST_FRAG_CRC_K == 8 ? 8 : 12)
#endif
constexpr uint32_t kFragCrcWaves = FORST_FRAG_CRC_WAVES;
constexpr uint32_t kFragCrcThreads = kFragCrcWaves * 64;
constexpr uint32_t kFcOffA16 = 65536;                  // A16[1..15], 4 KiB each
constexpr uint32_t kFcOffC256 = kFcOffA16 + 15 * 4096;  // C256[1..3], 4 KiB each
constexpr uint32_t kFcLds = kFcOffC256 + 3 * 4096;     // 136 KiB

__device__ __forceinline__ uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}
__device__ __forceinline__ uint64_t xxh3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= 0x165667919E3779F9ull;
  h ^= h >> 32;
  return h;
}
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= 0x9FB21C651E98DF25ull;
  h ^= (h >> 35) + len;
  h *= 0x9FB21C651E98DF25ull;
  return h ^ (h >> 28);
}
__device__ __forceinline__ uint64_t mix16B(const uint8_t* in, uint32_t s) {
  return mul128_fold64(ldu64(in) ^ sec64(s), ldu64(in + 8) ^ sec64(s + 8));
}

// util/xxhash.h:3918-4139, seed 0 (uniform scalar code on every lane)
__device__ uint64_t xxh3_short(const uint8_t* in, uint32_t len) {
  if (len <= 16) {
    if (len > 8) {
      const uint64_t lo = ldu64(in) ^ (sec64(24) ^ sec64(32));
      const uint64_t hi = ldu64(in + len - 8) ^ (sec64(40) ^ sec64(48));
      const uint64_t acc = len + __builtin_bswap64(lo) + hi + mul128_fold64(lo, hi);
      return xxh3_avalanche(acc);
    }
    if (len >= 4) {
      const uint32_t in1 = ldu32(in), in2 = ldu32(in + len - 4);
      const uint64_t in64 = in2 + (static_cast<uint64_t>(in1) << 32);
      return rrmxmx(in64 ^ (sec64(8) ^ sec64(16)), len);
    }
    if (len) {
      const uint32_t c1 = ldu8(in), c2 = ldu8(in + (len >> 1)), c3 = ldu8(in + len - 1);
      const uint32_t combined = (c1 << 16) | (c2 << 24) | c3 | (len << 8);
      const uint32_t bf = static_cast<uint32_t>(sec64(0)) ^
                          static_cast<uint32_t>(sec64(4));
      return xxh64_avalanche(static_cast<uint64_t>(combined ^ bf));
    }
    return xxh64_avalanche(sec64(56) ^ sec64(64));
  }
  if (len <= 128) {
    uint64_t acc = len * P64_1, acc_end;
    acc += mix16B(in, 0);
    acc_end = mix16B(in + len - 16, 16);
    if (len > 32) {
      acc += mix16B(in + 16, 32);
      acc_end += mix16B(in + len - 32, 48);
      if (len > 64) {
        acc += mix16B(in + 32, 64);
        acc_end += mix16B(in + len - 48, 80);
        if (len > 96) {
          acc += mix16B(in + 48, 96);
          acc_end += mix16B(in + len - 64, 112);
        }
      }
    }
    return xxh3_avalanche(acc + acc_end);
  }
  uint64_t acc = len * P64_1, acc_end;
  const uint32_t nbRounds = len / 16;
  for (uint32_t i = 0; i < 8; ++i) acc += mix16B(in + 16 * i, 16 * i);
  acc_end = mix16B(in + len - 16, 136 - 17);
  acc = xxh3_avalanche(acc);
  for (uint32_t i = 8; i < nbRounds; ++i)
    acc_end += mix16B(in + 16 * i, 16 * (i - 8) + 3);
  return xxh3_avalanche(acc + acc_end);
}

// ---- short inputs (<= 240 B) on a 16-lane row, from prefetched chunks -----
// Lane t of the row that owns the input loads ONE 16-byte chunk with the
// step's other prefetched loads, chosen so that the length class's formula
// (util/xxhash.h:3918-4139, xxh3_short above) becomes one mix16B per lane and
// two row sums -- no dependent loads in the finish:
//   129..240  t < len/16: [16t, +16) (t < 8: acc, else acc_end with secret
//             16(t-8)+3); t = 15: [len-16, +16) (acc_end, secret 119)
//   17..128   t < 4: front chunk r = t, [16r, +16), secret 32r; 4 <= t < 8:
//             back chunk r = t-4, [len-16-16r, +16), secret 32r+16 (r <=
//             (len-1)/32)
//   0..16     t = 0: the 16 bytes ending at the input end (from 0 when the
//             input ends in the buffer's first 16 bytes); the formula reads
//             its 1-3 bytes / two dwords / two qwords out of that window
// Unused lanes load the input's first byte's dword (never past its end).
__device__ __forceinline__ bool short_used(uint32_t L, uint32_t t) {
  if (L > 128) return t == 15 || t < L / 16;
  if (L > 16) {
    const uint32_t r = (L - 1) / 32;
    return t < 4 ? t <= r : (t < 8 && t - 4 <= r);
  }
  return t == 0;
}

// address of lane t's chunk of the input [P0, P0 + L)
__device__ __forceinline__ uint64_t short_phys(uint64_t P0, uint32_t L, uint32_t t) {
  if (L <= 16) return t == 0 && P0 + L >= 16 ? P0 + L - 16 : (t == 0 ? 0 : P0);
  if (!short_used(L, t)) return P0;
  if (L > 128) return P0 + (t == 15 ? L - 16 : 16 * t);
  return P0 + (t < 4 ? 16 * t : L - 16 - 16 * (t - 4));
}

// per-lane secret words of the two chunk classes (LDS, 4 x u64 per row lane):
// [0..1] 129..240, [2..3] 17..128
__device__ __forceinline__ void short_secrets_fill(uint64_t* sk, uint32_t tid) {
  if (tid < 16) {
    const uint32_t t = tid;
    const uint32_t sa = t < 8 ? 16 * t : (t == 15 ? 136 - 17 : 16 * (t - 8) + 3);
    const uint32_t sb = t < 4 ? 32 * t : (t < 8 ? 32 * (t - 4) + 16 : 0);
    sk[4 * t + 0] = sec64(sa);
    sk[4 * t + 1] = sec64(sa + 8);
    sk[4 * t + 2] = sec64(sb);
    sk[4 * t + 3] = sec64(sb + 8);
  }
}

// 8 / 4 / 1 bytes at byte position pos of the 16-byte window (d0 | d1 << 64)
__device__ __forceinline__ uint64_t win8(uint64_t d0, uint64_t d1, uint32_t pos) {
  if (pos == 0) return d0;
  if (pos >= 8) return d1 >> (8 * (pos - 8));
  return (d0 >> (8 * pos)) | (d1 << (64 - 8 * pos));
}
__device__ __forceinline__ uint32_t win1(uint64_t d0, uint64_t d1, uint32_t pos) {
  return static_cast<uint32_t>((pos < 8 ? d0 >> (8 * pos) : d1 >> (8 * (pos - 8))) & 0xffu);
}

// XXH3_64bits of the row's short input of L bytes; (d0, d1) = the lane's
// chunk, pb = the input's first byte in lane 0's window (L <= 16).  Every
// lane of the wave must call it (DPP row sums); the row's lanes agree on the
// result for L > 16, lane 0 holds it for L <= 16.
__device__ __forceinline__ uint64_t xxh3_short_row(uint64_t d0, uint64_t d1, uint32_t L,
                                                   uint32_t t, uint32_t pb,
                                                   const uint64_t* __restrict__ sk) {
  const bool big = L > 128;
  const bool used = L > 16 && short_used(L, t);
  const uint64_t k0 = big ? sk[4 * t + 0] : sk[4 * t + 2];
  const uint64_t k1 = big ? sk[4 * t + 1] : sk[4 * t + 3];
  const uint64_t mx = used ? mul128_fold64(d0 ^ k0, d1 ^ k1) : 0ull;
  uint64_t sa = t < 8 ? mx : 0ull, sb = t < 8 ? 0ull : mx;
  sa += row_ror64<1>(sa);
  sb += row_ror64<1>(sb);
  sa += row_ror64<2>(sa);
  sb += row_ror64<2>(sb);
  sa += row_ror64<4>(sa);
  sb += row_ror64<4>(sb);
  sa += row_ror64<8>(sa);
  sb += row_ror64<8>(sb);
  const uint64_t acc = static_cast<uint64_t>(L) * P64_1 + sa;
  if (L > 128) return xxh3_avalanche(xxh3_avalanche(acc) + sb);
  if (L > 16) return xxh3_avalanche(acc);
  if (L > 8) {
    const uint64_t lo = win8(d0, d1, pb) ^ (sec64(24) ^ sec64(32));
    const uint64_t hi = win8(d0, d1, pb + L - 8) ^ (sec64(40) ^ sec64(48));
    return xxh3_avalanche(L + __builtin_bswap64(lo) + hi + mul128_fold64(lo, hi));
  }
  if (L >= 4) {
    const uint64_t in1 = static_cast<uint32_t>(win8(d0, d1, pb));
    const uint64_t in2 = static_cast<uint32_t>(win8(d0, d1, pb + L - 4));
    return rrmxmx((in2 + (in1 << 32)) ^ (sec64(8) ^ sec64(16)), L);
  }
  if (L) {
    const uint32_t c1 = win1(d0, d1, pb), c2 = win1(d0, d1, pb + (L >> 1)),
                   c3 = win1(d0, d1, pb + L - 1);
    const uint32_t combined = (c1 << 16) | (c2 << 24) | c3 | (L << 8);
    const uint32_t bf = static_cast<uint32_t>(sec64(0)) ^ static_cast<uint32_t>(sec64(4));
    return xxh64_avalanche(static_cast<uint64_t>(combined ^ bf));
  }
  // (an opaque zero: the folded constant, kept live across the callers'
  // loops, was a spilled register pair)
  return xxh64_avalanche(sec64(56) ^ sec64(64) ^ fresh(0u));
}

// ---- short inputs (<= 240 B), one per 16-lane row ---------------------------
// Lane t of the row loads the 16-byte chunk of xxh3_short_row's layout
// (short_phys: one dword-aligned 16-byte load and the dword after it), so a
// row's loads are one contiguous stretch of the input, and the formula runs
// from registers with DPP row sums.  (One input per lane, with every 16-byte
// window of the input in that lane's registers, measured 0.23-0.56 ms for
// C5's 2.9 M short records against this: its scattered per-lane loads were
// address-bound.)  Bytes at or past base_len read as zero (byte loads, only
// at the buffer end).  WAL recovery's short candidates (wal_recover.hip).
__device__ __forceinline__ u32x4a4 ld16_lim(const uint8_t* base, uint64_t base_len, uint64_t a) {
  u32x4a4 v{0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j)
    if (a + j < base_len) v[j >> 2] |= ldu8(base + a + j) << (8 * (j & 3));
  return v;
}
__device__ __forceinline__ uint32_t ld4_lim(const uint8_t* base, uint64_t base_len, uint64_t a) {
  uint32_t v = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j)
    if (a + j < base_len) v |= ldu8(base + a + j) << (8 * j);
  return v;
}
constexpr uint32_t kShortRowsThreads = 256;
constexpr uint32_t kShortRowsU = 4;  // inputs per row in flight (loads issued together)
__global__ void __launch_bounds__(kShortRowsThreads) xxh3_short_rows_kernel(
    const uint8_t* base, uint64_t base_len, const uint64_t* off, const uint32_t* len, uint64_t n,
    const uint64_t* idx, uint64_t* out) {
  __shared__ uint64_t shsec[64];
  short_secrets_fill(shsec, threadIdx.x);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, t = lane & 15, row = lane >> 4;
  const uint64_t wave = uniform(threadIdx.x >> 6);
  constexpr uint64_t kPerWave = 4 * kShortRowsU;
  const uint64_t step = kPerWave * gridDim.x * (kShortRowsThreads / 64);
  for (uint64_t k0 = kPerWave * (static_cast<uint64_t>(blockIdx.x) * (kShortRowsThreads / 64) + wave);
       k0 < n; k0 += step) {  // (wave-uniform: the row sums need every lane)
    uint64_t P0[kShortRowsU];
    uint32_t L[kShortRowsU];
#pragma unroll
    for (uint32_t u = 0; u < kShortRowsU; ++u) {
      const uint64_t k = k0 + 4 * u + row;
      P0[u] = k < n ? off[k] : 0ull;
      L[u] = k < n ? len[k] : 0u;
    }
    u32x4a4 c[kShortRowsU];
    uint32_t nx[kShortRowsU];
    uint64_t ph[kShortRowsU];
    bool ok[kShortRowsU];
#pragma unroll
    for (uint32_t u = 0; u < kShortRowsU; ++u) {
      ok[u] = k0 + 4 * u + row < n && L[u] <= 240 && P0[u] <= base_len && L[u] <= base_len - P0[u];
      ph[u] = ok[u] ? short_phys(P0[u], L[u], t) : 0ull;
      const uint64_t q = ph[u] & ~3ull;
      // (an address past the buffer end: bytes loaded one by one, taken
      // after the other loads so the common path's loads stay together)
      const uint64_t qf = q + 20 <= base_len ? q : 0ull;
      c[u] = ld16_a4(base + qf);
      nx[u] = ld4_a4(base + qf + 16);
    }
#pragma unroll
    for (uint32_t u = 0; u < kShortRowsU; ++u) {
      const uint64_t q = ph[u] & ~3ull;
      if (q + 20 > base_len) {
        c[u] = ld16_lim(base, base_len, q);
        nx[u] = ld4_lim(base, base_len, q + 16);
      }
      const uint32_t m = static_cast<uint32_t>(ph[u] & 3);
      const uint64_t d0 = mk64(__builtin_amdgcn_alignbyte(c[u].y, c[u].x, m),
                               __builtin_amdgcn_alignbyte(c[u].z, c[u].y, m));
      const uint64_t d1 = mk64(__builtin_amdgcn_alignbyte(c[u].w, c[u].z, m),
                               __builtin_amdgcn_alignbyte(nx[u], c[u].w, m));
      const uint32_t pb = ok[u] ? static_cast<uint32_t>(P0[u] - short_phys(P0[u], L[u], 0)) : 0u;
      const uint64_t h = xxh3_short_row(d0, d1, L[u], t, pb, shsec);
      const uint64_t k = k0 + 4 * u + row;
      if (k < n && t == 0) out[idx ? idx[k] : k] = ok[u] ? h : 0ull;
    }
  }
}

struct LaneKeys {
  uint64_t k0, k1;    // accumulate keys for (stripe L/4, pair L%4)
  uint64_t kl0, kl1;  // last-stripe keys (XXH_SECRET_LASTACC_START = 7)
  uint64_t ks0, ks1;  // scramble keys for accumulators 2p, 2p+1
  uint64_t km0, km1;  // merge keys (XXH_SECRET_MERGEACCS_START = 11)
  uint64_t init0, init1;
};

__device__ __forceinline__ LaneKeys lane_keys(uint32_t lane) {
  const uint32_t s = lane >> 2, p = lane & 3;
  LaneKeys k;
  k.k0 = sec64(8 * s + 16 * p);
  k.k1 = sec64(8 * s + 16 * p + 8);
  k.kl0 = sec64(192 - 64 - 7 + 16 * p);
  k.kl1 = sec64(192 - 64 - 7 + 16 * p + 8);
  k.ks0 = sec64(192 - 64 + 16 * p);
  k.ks1 = sec64(192 - 64 + 16 * p + 8);
  k.km0 = sec64(11 + 16 * p);
  k.km1 = sec64(11 + 16 * p + 8);
  // XXH3_INIT_ACC (xxhash.h:5188)
  const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3,
                            P64_4, P32_2, P64_5, P32_1};
  k.init0 = p == 0 ? init[0] : p == 1 ? init[2] : p == 2 ? init[4] : init[6];
  k.init1 = p == 0 ? init[1] : p == 1 ? init[3] : p == 2 ? init[5] : init[7];
  return k;
}

__device__ __forceinline__ uint64_t scramble(uint64_t a, uint64_t key) {
  a ^= a >> 47;
  a ^= key;
  return a * P32_1;
}

// XXH3_64bits(p, len); all arguments wave-uniform, every lane returns it.
__device__ uint64_t wave_xxh3_64(const uint8_t* p, uint32_t len, uint32_t lane,
                                 const LaneKeys& K) {
  if (len <= 240) return xxh3_short(p, len);
  const uint32_t s = lane >> 2;
  const uint32_t nb = (len - 1) / 1024;
  const uint32_t nbStripes = ((len - 1) - 1024 * nb) / 64;
  const uint64_t A = reinterpret_cast<uint64_t>(p);
  const uint32_t m = static_cast<uint32_t>(A & 3);
  const uint8_t* q = p - m + 16 * lane;  // keeps the global address space
  uint64_t acc0 = K.init0, acc1 = K.init1;
  // full XXH3-blocks, 4 per round so 4 loads are in flight per lane
  uint32_t g = 0;
  for (; g + 4 <= nb; g += 4) {
    uint64_t c0[4], c1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t d0, d1;
      ld16u(q + 1024 * (g + j), m, d0, d1);
      const uint64_t dk0 = d0 ^ K.k0, dk1 = d1 ^ K.k1;
      c0[j] = mul32to64(dk0) + d1;  // acc[2p]   += lo*hi(dk0) ; acc[2p] += d1
      c1[j] = d0 + mul32to64(dk1);  // acc[2p+1] += d0 ; += lo*hi(dk1)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = scramble(acc0 + stripe_sum(c0[j]), K.ks0);
      acc1 = scramble(acc1 + stripe_sum(c1[j]), K.ks1);
    }
  }
  for (; g < nb; ++g) {
    uint64_t d0, d1;
    ld16u(q + 1024 * g, m, d0, d1);
    const uint64_t dk0 = d0 ^ K.k0, dk1 = d1 ^ K.k1;
    acc0 = scramble(acc0 + stripe_sum(mul32to64(dk0) + d1), K.ks0);
    acc1 = scramble(acc1 + stripe_sum(d0 + mul32to64(dk1)), K.ks1);
  }
  // last partial XXH3-block: stripes [0, nbStripes), no scramble
  {
    uint64_t c0 = 0, c1 = 0;
    if (s < nbStripes) {
      uint64_t d0, d1;
      ld16u(q + 1024 * nb, m, d0, d1);
      const uint64_t dk0 = d0 ^ K.k0, dk1 = d1 ^ K.k1;
      c0 = mul32to64(dk0) + d1;
      c1 = d0 + mul32to64(dk1);
    }
    acc0 += stripe_sum(c0);
    acc1 += stripe_sum(c1);
  }
  // last stripe at len-64 (xxhash.h:5146-5151), every lane does its pair
  {
    const uint8_t* lp = p + len - 64 + 16 * (lane & 3);
    const uint32_t ml = static_cast<uint32_t>((A + len) & 3);  // == lp & 3
    uint64_t d0, d1;
    ld16u(lp - ml, ml, d0, d1);
    const uint64_t dk0 = d0 ^ K.kl0, dk1 = d1 ^ K.kl1;
    acc0 += mul32to64(dk0) + d1;
    acc1 += d0 + mul32to64(dk1);
  }
  // XXH3_mergeAccs (xxhash.h:5164)
  uint64_t t = mul128_fold64(acc0 ^ K.km0, acc1 ^ K.km1);
  t += quad_xor64<1>(t);
  t += quad_xor64<2>(t);
  return xxh3_avalanche(static_cast<uint64_t>(len) * P64_1 + t);
}

// ---------------------------------------------------------------------------
// Streaming XXH3 block kernel (same shape as crc32c_stream_kernel): a wave
// walks its contiguous share of blocks as (block, round) steps, a round being
// 4 XXH3-blocks (4 KiB: per lane 4 x (dwordx4 + the dword after it, for
// unaligned starts)).  The loads of the next step -- plus the block's last
// stripe and trailer dwords -- are issued unconditionally (clamped to a safe
// address when not needed) before the current step's stripe sums and
// scrambles run, so the compiler's wait for the current step leaves the next
// one in flight.  Descriptors come in 64-block batches (stream_common.h);
// per-lane cold constants live in LDS so no VMEM load sits in the loop.
// ---------------------------------------------------------------------------
// Per-accumulator-pair constants used once per block (last-stripe keys,
// merge keys, XXH3_INIT_ACC), evaluated at compile time from the secret.
constexpr uint8_t kSecC[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad,
    0x1c, 0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3,
    0x67, 0x1f, 0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc,
    0xff, 0x72, 0x21, 0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6,
    0x81, 0x3a, 0x26, 0x4c, 0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65,
    0x8b, 0x1b, 0x53, 0x2e, 0xa3, 0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19,
    0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8, 0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9,
    0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d, 0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31,
    0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, 0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb,
    0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb, 0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0,
    0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e, 0x2b, 0x16, 0xbe, 0x58, 0x7d,
    0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce, 0x45, 0xcb, 0x3a, 0x8f,
    0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e};
constexpr uint64_t rd64c(uint32_t off) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | kSecC[off + i];
  return v;
}
enum { kColdL0 = 0, kColdL1, kColdM0, kColdM1, kColdI0, kColdI1, kColdN };
#define FORST_XX_COLD(p, i0, i1)                                                           \
  {rd64c(121 + 16 * (p)), rd64c(121 + 16 * (p) + 8), rd64c(11 + 16 * (p)),                 \
   rd64c(11 + 16 * (p) + 8), (i0), (i1)}
__device__ __constant__ const uint64_t kXxCold[4][kColdN] = {
    FORST_XX_COLD(0, P32_3, P64_1), FORST_XX_COLD(1, P64_2, P64_3),
    FORST_XX_COLD(2, P64_4, P32_2), FORST_XX_COLD(3, P64_5, P32_1)};
#undef FORST_XX_COLD

struct HotKeys {
  uint64_t k0, k1;    // accumulate keys for (stripe L/4, pair L%4)
  uint64_t ks0, ks1;  // scramble keys for accumulators 2p, 2p+1
};
__device__ __forceinline__ HotKeys hot_keys(uint32_t lane) {
  const uint32_t s = lane >> 2, p = lane & 3;
  return HotKeys{sec64(8 * s + 16 * p), sec64(8 * s + 16 * p + 8),
                 sec64(192 - 64 + 16 * p), sec64(192 - 64 + 16 * p + 8)};
}

constexpr int kXxRound = 4;  // XXH3-blocks per step

struct XBlk {
  uint64_t off;
  uint64_t q0;      // offset of lane 0's 16-byte slot of XXH3-block 0 (dword aligned)
  uint64_t lq;      // offset of pair 0's slot of the last stripe (dword aligned)
  uint64_t t0, t1;  // trailer dword offsets
  uint32_t size, mod, extra;
  uint32_t nb, nbS, R, m, ml, tb;  // tb: byte index of the type byte in t0
  bool valid, slow;
};

template <int MODE>
__device__ __forceinline__ XBlk xblk_setup(const BlockArgs& a, uint64_t k, uint64_t kend,
                                           uint64_t kb, const DescBatch& cb,
                                           const DescBatch& nb) {
  XBlk b;
  const Desc d = batch_desc(k, kb, cb, nb);
  b.off = d.off;
  b.size = d.size;
  b.mod = d.mod;
  b.extra = d.extra;
  b.valid = k < kend && desc_in_range<MODE>(a, d);
  b.slow = !b.valid || b.size <= 240;
  b.nb = (b.size - 1) / 1024;
  b.nbS = ((b.size - 1) - 1024 * b.nb) / 64;
  b.R = (b.nb + kXxRound) / kXxRound;  // XXH3-blocks 0..nb
  b.m = static_cast<uint32_t>(b.off & 3);
  const uint64_t E = b.off + b.size;
  b.ml = static_cast<uint32_t>(E & 3);
  b.q0 = b.off - b.m;
  b.lq = E - 64 - b.ml;
  // type byte at E, stored LE32 at E+1 (verify); type byte only (compute /
  // trailer without last_bytes[]); nothing otherwise (point at the block)
  const bool mem_last = MODE == kModeVerify || (MODE != kModeRaw && !a.last_bytes);
  b.tb = b.ml;
  b.t0 = mem_last ? (E & ~3ull) : b.q0;
  b.t1 = MODE == kModeVerify ? (E & ~3ull) + 4 : b.t0;
  if (b.slow) {  // dummy loads at the buffer start
    b.q0 = b.lq = b.t0 = b.t1 = 0;
    b.nb = b.nbS = 0;
  }
  return b;
}

struct XStep {
  uint32_t x[kXxRound][5];
  uint32_t l[5];
  uint32_t t0, t1;
};

__device__ __forceinline__ void xx_issue(const uint8_t* __restrict__ base, uint32_t lane,
                                         const XBlk& b, uint32_t r, XStep& d) {
  const uint32_t s = lane >> 2;
#pragma unroll
  for (int k = 0; k < kXxRound; ++k) {
    const uint32_t g = kXxRound * r + k;
    const bool need = g < b.nb || (g == b.nb && s < b.nbS);
    const uint64_t o = need ? b.q0 + 1024ull * g + 16 * lane : b.q0;
    const u32x4a4 v = ld16_a4(base + o);
    d.x[k][0] = v.x;
    d.x[k][1] = v.y;
    d.x[k][2] = v.z;
    d.x[k][3] = v.w;
    // the dword after the slot (unaligned starts); it always holds a message
    // byte when the slot is needed, so it never crosses into an unmapped page
    d.x[k][4] = ld4_a4(base + o + 16);
  }
  const uint8_t* lp = base + b.lq + 16 * (lane & 3);
  const u32x4a4 v = ld16_a4(lp);
  d.l[0] = v.x;
  d.l[1] = v.y;
  d.l[2] = v.z;
  d.l[3] = v.w;
  d.l[4] = ld4_a4(lp + 16);
  d.t0 = ld4v(base + b.t0);
  d.t1 = ld4v(base + b.t1);
}

__device__ __forceinline__ void xx_words(const uint32_t (&x)[5], uint32_t m, uint64_t& d0,
                                         uint64_t& d1) {
  // v_alignbyte_b32 by 0 returns the low word: no branch on m
  const uint32_t x0 = __builtin_amdgcn_alignbyte(x[1], x[0], m);
  const uint32_t x1 = __builtin_amdgcn_alignbyte(x[2], x[1], m);
  const uint32_t x2 = __builtin_amdgcn_alignbyte(x[3], x[2], m);
  const uint32_t x3 = __builtin_amdgcn_alignbyte(x[4], x[3], m);
  d0 = mk64(x0, x1);
  d1 = mk64(x2, x3);
}

// round r of block b (accumulate + scramble per XXH3-block, xxhash.h:5123-5140)
__device__ __forceinline__ void xx_step_round(const XBlk& b, uint32_t r, uint32_t lane,
                                              const HotKeys& K, const XStep& d, uint64_t& acc0,
                                              uint64_t& acc1) {
  const uint32_t s = lane >> 2;
#pragma unroll
  for (int k = 0; k < kXxRound; ++k) {
    const uint32_t g = kXxRound * r + k;
    if (g > b.nb) break;
    uint64_t d0, d1;
    xx_words(d.x[k], b.m, d0, d1);
    uint64_t c0 = mul32to64(d0 ^ K.k0) + d1;  // acc[2p]   (xxhash.h:4926-4927)
    uint64_t c1 = d0 + mul32to64(d1 ^ K.k1);  // acc[2p+1]
    if (g == b.nb && s >= b.nbS) c0 = c1 = 0;
    acc0 += stripe_sum(c0);
    acc1 += stripe_sum(c1);
    if (g < b.nb) {  // full XXH3-block: scramble (xxhash.h:5126-5128)
      acc0 = scramble(acc0, K.ks0);
      acc1 = scramble(acc1, K.ks1);
    }
  }
}

// PROBE = 1 (diagnostics build only, FORST_XXH3_VARIANT=probe_load): same
// loads and control flow, data only XOR-folded, every block reported ok.
template <int MODE, int PROBE>
__device__ __forceinline__ void xxh3_stream_body(const BlockArgs& a) {
  __shared__ uint64_t cold[4 * kColdN];
  if (threadIdx.x < 4 * kColdN) cold[threadIdx.x] = (&kXxCold[0][0])[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const HotKeys K = hot_keys(lane);
  const uint64_t* ck = cold + kColdN * (lane & 3);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * kWaves + wave;
  uint64_t kbeg, kend;
  wave_share(a.n, nw, gw, kbeg, kend);
  if (kbeg >= kend) return;

  DescBatch cb, nb;
  uint64_t kb = kbeg;
  load_batch<MODE>(a, kb, kend, lane, cb);
  load_batch<MODE>(a, kb + kBatch, kend, lane, nb);
  uint64_t k = kbeg;
  XBlk C = xblk_setup<MODE>(a, k, kend, kb, cb, nb);
  XBlk N = xblk_setup<MODE>(a, k + 1, kend, kb, cb, nb);
  uint32_t rOut = 0, rHi = 0, rSt = 0, rOk = 0;
  XStep X, Y;
  xx_issue(a.base, lane, C, 0, X);
  uint32_t r = 0;
  uint64_t acc0 = 0, acc1 = 0;

  auto flush = [&](uint32_t cnt) {
    const uint64_t i = kb + lane;
    const bool mine = lane < cnt;
    if (MODE == kModeRaw) {
      if (mine && a.out64) a.out64[i] = mk64(rOut, rHi);
    } else if (mine && a.out32) {
      a.out32[i] = rOut;
    }
    if (MODE == kModeVerify) {
      if (mine && a.stored_out) a.stored_out[i] = rSt;
      if (mine && a.ok_out) a.ok_out[i] = static_cast<uint8_t>(rOk);
      const uint64_t badm = __ballot(mine && rOk == 0);
      if (a.mismatches && badm && lane == 0)
        atomicAdd(a.mismatches, static_cast<unsigned long long>(__popcll(badm)));
    }
    if (MODE == kModeTrailer) {
      if (mine && rOk) {
        const uint64_t off = (static_cast<uint64_t>(cb.off_hi) << 32) | cb.off_lo;
        uint8_t* p = a.base_w + off + cb.size;
        if (a.last_bytes) p[0] = static_cast<uint8_t>(cb.extra);
        stu32_bytes(p + 1, rOut);
      }
    }
  };

  auto step = [&](XStep& cu, XStep& nx) -> bool {
    const bool last = C.slow || r + 1 >= C.R;
    if (last)
      xx_issue(a.base, lane, N, 0, nx);
    else
      xx_issue(a.base, lane, C, r + 1, nx);
    uint64_t h = 0;
    if (PROBE) {
      uint32_t f = 0;
#pragma unroll
      for (int q = 0; q < kXxRound; ++q) f ^= cu.x[q][0] ^ cu.x[q][1] ^ cu.x[q][2] ^ cu.x[q][3] ^ cu.x[q][4];
      acc0 ^= f ^ cu.l[0] ^ cu.l[4] ^ cu.t0;
      if (!last) {
        ++r;
        return true;
      }
      h = __ballot(static_cast<uint32_t>(acc0) == 0x9e3779b9u) ? 1 : 0;
      acc0 = 0;
    } else if (!C.slow) {
      if (r == 0) {  // XXH3_INIT_ACC (xxhash.h:5188)
        acc0 = ck[kColdI0];
        acc1 = ck[kColdI1];
      }
      xx_step_round(C, r, lane, K, cu, acc0, acc1);
      if (!last) {
        ++r;
        return true;
      }
      uint64_t d0, d1;  // last stripe at len-64 (xxhash.h:5146-5151)
      xx_words(cu.l, C.ml, d0, d1);
      acc0 += mul32to64(d0 ^ ck[kColdL0]) + d1;
      acc1 += d0 + mul32to64(d1 ^ ck[kColdL1]);
      uint64_t t = mul128_fold64(acc0 ^ ck[kColdM0], acc1 ^ ck[kColdM1]);  // mergeAccs
      t += quad_xor64<1>(t);
      t += quad_xor64<2>(t);
      h = xxh3_avalanche(static_cast<uint64_t>(C.size) * P64_1 + t);
    }
    uint32_t lastb = 0, stored = 0;
    if (!C.slow) {
      lastb = (cu.t0 >> (8 * C.tb)) & 0xffu;
      if (MODE == kModeVerify)
        stored = C.tb == 3 ? cu.t1 : __builtin_amdgcn_alignbyte(cu.t1, cu.t0, C.tb + 1);
    } else if (C.valid) {
      // short input: the length-class formulas, with their own loads; retire()
      // keeps those loads from merging into the hot path (see crc32c.hip)
      const uint8_t* p = a.base + C.off;
      const uint64_t hs = xxh3_short(p, C.size);
      h = mk64(retire(static_cast<uint32_t>(hs)), retire(static_cast<uint32_t>(hs >> 32)));
      if (MODE != kModeRaw) lastb = retire(ldu8(p + C.size));
      if (MODE == kModeVerify) stored = retire(ldu32(p + C.size + 1));
    }
    if ((MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes) lastb = C.extra;
    if (PROBE) {  // report ok: computed == stored
      lastb = 0;
      stored = static_cast<uint32_t>(h) + C.mod;
    }
    uint32_t out, hi = 0, st = 0, ok = C.valid ? 1u : 0u;
    if (MODE == kModeRaw) {
      out = static_cast<uint32_t>(h);
      hi = static_cast<uint32_t>(h >> 32);
    } else if (MODE == kModeVerify) {
      // ComputeBuiltinChecksum(kXXH3, data, size+1), format.cc:577-586
      const uint32_t computed = modify_for_last_byte(static_cast<uint32_t>(h), lastb);
      st = stored - C.mod;
      ok = (C.valid && st == computed) ? 1u : 0u;
      out = computed;
    } else {
      out = modify_for_last_byte(static_cast<uint32_t>(h), lastb) + C.mod;
    }
    if (!C.valid) out = hi = st = 0;
    const uint32_t kk = static_cast<uint32_t>(k - kb);
    rOut = lane == kk ? out : rOut;
    rHi = lane == kk ? hi : rHi;
    rSt = lane == kk ? st : rSt;
    rOk = lane == kk ? ok : rOk;
    ++k;
    if (k - kb == kBatch || k == kend) {
      flush(static_cast<uint32_t>(k - kb));
      if (k == kend) return false;
      kb = k;
      cb = nb;
      load_batch<MODE>(a, kb + kBatch, kend, lane, nb);
    }
    C = N;
    N = xblk_setup<MODE>(a, k + 1, kend, kb, cb, nb);
    r = 0;
    return true;
  };
  while (step(X, Y) && step(Y, X)) {
  }
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) xxh3_stream_kernel(BlockArgs a) {
  xxh3_stream_body<MODE, 0>(a);
}

#ifdef FORST_DIAG
__global__ void __launch_bounds__(kThreads) xxh3_stream_probe_kernel(BlockArgs a) {
  xxh3_stream_body<kModeVerify, 1>(a);
}
#endif

// ---------------------------------------------------------------------------
// XXH3 v2 ("rows"): four messages per wave, one per 16-lane row.
//
// In the one-message-per-wave layout every 16 bytes of input cost a 4-level
// cross-lane stripe sum (two DPP row rotations + permlane16/32 swaps) for each
// of two 64-bit accumulators -- about three times the hash arithmetic itself.
// Here row r (lanes 16r..16r+15) owns a message; lane t = 4 s4 + p of the row
// takes stripes s4, s4+4, s4+8, s4+12 (accumulator pair p) of each 1 KiB
// XXH3-block: four global_load_dwordx4 per lane, each instruction reading 256
// contiguous bytes per row.  The four stripes are summed in registers and the
// row reduction is two DPP row rotations.  One step = one XXH3-block per row
// (4 KiB per wave), with the next step's loads (data, last stripe, trailer
// dwords, modifier / type byte) in flight while the current one computes.
// Rows draw messages dynamically from the wave's contiguous share (a row that
// finishes takes the next unassigned message), so mixed 4/16/64 KiB batches
// stay balanced.  Descriptors come in 64-message batches held one per lane and
// are fetched by the rows with ds_bpermute.
// ---------------------------------------------------------------------------
constexpr uint32_t kNoMsg = 0xffffffffu;

// a row's position: message (relative to the wave share) and XXH3-block;
// row-uniform values, one copy per lane
struct RowPos {
  uint32_t off_lo, off_hi, size;
  uint32_t rel;  // message index - kbeg, kNoMsg when the share is exhausted
  uint32_t g;    // XXH3-block index
};

__device__ __forceinline__ uint64_t rp_off(const RowPos& p) {
  return (static_cast<uint64_t>(p.off_hi) << 32) | p.off_lo;
}

template <int MODE>
__device__ __forceinline__ bool rp_valid(const BlockArgs& a, const RowPos& p) {
  if (p.rel == kNoMsg) return false;
  const Desc d{rp_off(p), p.size, 0, 0};
  return desc_in_range<MODE>(a, d);
}

struct RStep {
  uint32_t x[4][5];  // 4 stripes x (16 bytes + the next dword)
  uint32_t l[5];     // last stripe piece
  uint32_t t0, t1;   // type byte / stored checksum dwords
  uint32_t mod, extra;
};

template <int MODE>
__device__ __forceinline__ void rows_issue(const BlockArgs& a, uint32_t lane, const RowPos& P,
                                           uint64_t kbeg, RStep& d) {
  const uint32_t t = lane & 15, s4 = t >> 2, p = t & 3;
  const uint64_t off = rp_off(P);
  const bool valid = rp_valid<MODE>(a, P);
  const bool lng = valid && P.size > 240;
  const uint32_t nb = (P.size - 1) >> 10, nbS = ((P.size - 1) & 1023) >> 6;
  const uint32_t m = static_cast<uint32_t>(off & 3);
  const uint64_t q0 = (off & ~3ull) + 1024ull * P.g + 64 * s4 + 16 * p;
  const bool shrt = valid && !lng;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    bool need = lng && (P.g < nb || s4 + 4 * k < nbS);
    uint64_t o = need ? q0 + 256 * k : 0;
    uint32_t mk = m;
    if (k == 0 && shrt) {  // a short message's chunk (xxh3_short_row)
      const uint64_t ph = short_phys(off, P.size, t);
      need = true;
      o = ph & ~3ull;
      mk = static_cast<uint32_t>(ph & 3);
    }
    const u32x4a4 v = ld16_a4(a.base + o);
    d.x[k][0] = v.x;
    d.x[k][1] = v.y;
    d.x[k][2] = v.z;
    d.x[k][3] = v.w;
    // the dword after the piece only matters for unaligned starts; then it
    // holds a message byte, so it never crosses into an unmapped page
    d.x[k][4] = ld4_a4(a.base + (need && mk ? o + 16 : o));
  }
  // the finishing step's words (last stripe, type byte / stored checksum,
  // modifier), loaded in every step (from offset 0 when not needed): a
  // step's load count must not depend on a branch, or the compiler's vmcnt
  // waits for the current step's data also wait for the step in flight
  const bool lastp = lng && P.g == nb;
  const uint64_t lq = off + P.size - 64 + 16 * p;
  const uint32_t ml = static_cast<uint32_t>(lq & 3);
  const uint64_t lo = lastp ? (lq & ~3ull) : 0;
  const u32x4a4 v = ld16_a4(a.base + lo);
  d.l[0] = v.x;
  d.l[1] = v.y;
  d.l[2] = v.z;
  d.l[3] = v.w;
  d.l[4] = ld4_a4(a.base + (lastp && ml ? lo + 16 : lo));
  // type byte at E = off + size, stored LE32 at E + 1 (verify); for compute /
  // trailer without last_bytes[] only the type byte
  const bool mem_last = MODE == kModeVerify || (MODE != kModeRaw && !a.last_bytes);
  const uint64_t E = off + P.size;
  const uint64_t t0 = ((lastp || shrt) && mem_last) ? (E & ~3ull) : 0;
  d.t0 = ld4v(a.base + t0);
  d.t1 = MODE == kModeVerify ? ld4v(a.base + ((lastp || shrt) ? t0 + 4 : 0)) : 0u;
  const uint64_t idx = kbeg + (P.rel == kNoMsg ? 0 : P.rel);
  d.mod = (MODE != kModeRaw && a.modifiers) ? a.modifiers[idx] : 0u;
  d.extra = ((MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes) ? a.last_bytes[idx]
                                                                              : 0u;
}

template <int MODE>
__global__ void __launch_bounds__(kRowsThreads) FORST_WAVES_PER_EU(3)
    xxh3_rows_kernel(BlockArgs a) {
  __shared__ uint64_t cold[4 * kColdN];
  __shared__ uint64_t shsec[64];
  feed_init();
  if (threadIdx.x < 4 * kColdN) cold[threadIdx.x] = (&kXxCold[0][0])[threadIdx.x];
  short_secrets_fill(shsec, threadIdx.x);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t t = lane & 15, s4 = t >> 2, p = t & 3;
  const uint64_t* ck = cold + kColdN * p;
  // accumulate keys of the lane's four stripes, scramble keys of its pair
  uint64_t K0[4], K1[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    K0[k] = sec64(8 * (s4 + 4 * k) + 16 * p);
    K1[k] = sec64(8 * (s4 + 4 * k) + 16 * p + 8);
  }
  const uint64_t ks0 = sec64(128 + 16 * p), ks1 = sec64(136 + 16 * p);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kRowsWaves;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * kRowsWaves + wave;
  // descriptor batches from the work feed (stream_common.h): lane j <->
  // message cg + j (cb), ng + j (nb); a row's rel is the message's global
  // index (n < 2^32 - 1), kbrel the stream position of cb's first entry
  BatchFeed feed;
  uint64_t cg = feed_first<MODE != kModeRaw, kXxWgChunk>(a, nw, gw, lane, feed);
  // block modes: results staged in LDS and stored after the loop by the
  // whole workgroup (as crc32c_rows_kernel: stores share vmcnt with the
  // stream's loads), so every wave reaches the end: no early return
  constexpr bool kStage = FORST_XX_STAGE && MODE != kModeRaw;
  __shared__ uint32_t st_out[kStage ? kXxStageW : 1];
  __shared__ uint8_t st_ok[kStage ? kXxStageW : 4];  // verify: ok; else: valid
  __shared__ uint8_t st_lb[MODE == kModeTrailer && kStage ? kXxStageW : 4];
  if (!kStage && cg >= a.n) return;
  uint32_t clen = feed.len;  // entries of cb / nb (a batch holds up to 64)
  uint64_t ng = feed_next<MODE != kModeRaw, kXxWgChunk>(a, nw, lane, feed);
  uint32_t nlen = feed.len;
  const uint64_t kbeg = 0;
  DescBatch cb, nb;
  uint64_t kbrel = 0;
  load_batch<MODE>(a, cg, a.n, lane, cb);
  load_batch<MODE>(a, ng, a.n, lane, nb);
  auto fetch = [&](uint64_t rel, RowPos& P) {
    const BatchSlot q = batch_slot(rel, kbrel, cg, clen, ng, nlen, a.n);
    const uint32_t lo_c = __shfl(cb.off_lo, q.src), hi_c = __shfl(cb.off_hi, q.src);
    const uint32_t sz_c = __shfl(cb.size, q.src);
    const uint32_t lo_n = __shfl(nb.off_lo, q.src), hi_n = __shfl(nb.off_hi, q.src);
    const uint32_t sz_n = __shfl(nb.size, q.src);
    P.off_lo = q.in_n ? lo_n : lo_c;
    P.off_hi = q.in_n ? hi_n : hi_c;
    P.size = q.in_n ? sz_n : sz_c;
    P.rel = q.valid ? static_cast<uint32_t>(q.gi) : kNoMsg;
    P.g = 0;
  };
  // rows start on messages 0..3 of the stream
  const uint32_t row = lane >> 4;
  uint64_t next = 4;
  RowPos C;
  fetch(row, C);

  // I = the position after P: next XXH3-block, or a newly assigned message
  auto advance = [&](const RowPos& P, RowPos& I) {
    const bool lng = rp_valid<MODE>(a, P) && P.size > 240;
    const uint32_t nbP = (P.size - 1) >> 10;
    const bool more = lng && P.g < nbP;
    const bool need = P.rel != kNoMsg && !more;
    const uint64_t rows = __ballot(need && t == 0);  // one bit per row leader
    I = P;
    if (more) I.g = P.g + 1;
    if (rows) {  // descriptor work only in steps where some row takes a message
      const uint32_t rank = static_cast<uint32_t>(__popcll(rows & ((1ull << (lane & ~15u)) - 1)));
      RowPos F;
      fetch(next + rank, F);
      next += static_cast<uint64_t>(__popcll(rows));
      if (need) I = F;
      if (next >= kbrel + clen) {  // every message of cb is assigned: slide the batches
        kbrel += clen;
        clen = nlen;
        cb = nb;
        cg = ng;
        ng = feed_next<MODE != kModeRaw, kXxWgChunk>(a, nw, lane, feed);
        nlen = feed.len;
        load_batch<MODE>(a, ng, a.n, lane, nb);
      }
    }
  };

  RowPos I;
  advance(C, I);
  RStep X, Y;
  rows_issue<MODE>(a, lane, C, kbeg, X);
  uint64_t acc0 = 0, acc1 = 0;
  const bool has_extra = (MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes;

  auto step = [&](RStep& cu, RStep& nx) -> bool {
    // (early exit kept here: the frag kernel's no-exit loop shape measured
    // slower on uniform messages, NS16X 0.724 vs 0.702 on one box)
    if (__ballot(C.rel != kNoMsg) == 0) return false;
    rows_issue<MODE>(a, lane, I, kbeg, nx);
    const uint64_t off = rp_off(C);
    const bool valid = rp_valid<MODE>(a, C);
    const bool lng = valid && C.size > 240;
    const uint32_t nbC = (C.size - 1) >> 10, nbSC = ((C.size - 1) & 1023) >> 6;
    const uint32_t m = static_cast<uint32_t>(off & 3);
    // ---- one XXH3-block of every row (xxhash.h:5123-5140) ----
    if (C.g == 0) {  // XXH3_INIT_ACC (xxhash.h:5188)
      acc0 = ck[kColdI0];
      acc1 = ck[kColdI1];
    }
    uint64_t sum0 = 0, sum1 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      uint64_t d0, d1;
      xx_words(cu.x[k], m, d0, d1);
      const uint64_t c0 = mul32to64(d0 ^ K0[k]) + d1;  // acc[2p]   (xxhash.h:4926-4927)
      const uint64_t c1 = d0 + mul32to64(d1 ^ K1[k]);  // acc[2p+1]
      const bool use = C.g < nbC || s4 + 4 * k < nbSC;
      sum0 += use ? c0 : 0ull;
      sum1 += use ? c1 : 0ull;
    }
    sum0 += row_ror64<4>(sum0);  // the row's four stripe groups
    sum1 += row_ror64<4>(sum1);
    sum0 += row_ror64<8>(sum0);
    sum1 += row_ror64<8>(sum1);
    acc0 += sum0;
    acc1 += sum1;
    const bool full = C.g < nbC;
    if (full) {  // xxhash.h:5126-5128
      acc0 = scramble(acc0, ks0);
      acc1 = scramble(acc1, ks1);
    }
    // ---- rows that finish a message in this step ----
    const bool fin = C.rel != kNoMsg && !(lng && full);
    if (__ballot(fin)) {
      uint64_t h = 0;
      {  // last stripe at len - 64, merge (xxhash.h:5146-5208)
        uint64_t d0, d1;
        const uint32_t ml = static_cast<uint32_t>((off + C.size) & 3);
        xx_words(cu.l, ml, d0, d1);
        const uint64_t a0 = acc0 + mul32to64(d0 ^ ck[kColdL0]) + d1;
        const uint64_t a1 = acc1 + d0 + mul32to64(d1 ^ ck[kColdL1]);
        uint64_t tm = mul128_fold64(a0 ^ ck[kColdM0], a1 ^ ck[kColdM1]);
        tm += quad_xor64<1>(tm);
        tm += quad_xor64<2>(tm);
        h = xxh3_avalanche(static_cast<uint64_t>(C.size) * P64_1 + tm);
      }
      const uint64_t E = off + C.size;
      const uint32_t tb = static_cast<uint32_t>(E & 3);
      uint32_t lastb = (cu.t0 >> (8 * tb)) & 0xffu;
      uint32_t stored = MODE == kModeVerify
                            ? (tb == 3 ? cu.t1 : __builtin_amdgcn_alignbyte(cu.t1, cu.t0, tb + 1))
                            : 0u;
      if (__ballot(fin && valid && !lng)) {  // short inputs: the row's chunks
        const uint64_t ph = short_phys(off, C.size, t);
        uint64_t d0, d1;
        xx_words(cu.x[0], static_cast<uint32_t>(ph & 3), d0, d1);
        const uint32_t pb = static_cast<uint32_t>(off - short_phys(off, C.size, 0));
        const uint64_t hs = xxh3_short_row(d0, d1, C.size, t, pb, shsec);
        if (fin && valid && !lng) h = hs;
      }
      if (has_extra) lastb = cu.extra;
      const uint64_t i = kbeg + (C.rel == kNoMsg ? 0 : C.rel);
      const bool mine = fin && t == 0;
      bool ok = valid;
      if (MODE == kModeRaw) {
        if (mine && a.out64) a.out64[i] = valid ? h : 0ull;
      } else if (MODE == kModeVerify) {
        // ComputeBuiltinChecksum(kXXH3, data, size+1), format.cc:577-586
        const uint32_t computed = modify_for_last_byte(static_cast<uint32_t>(h), lastb);
        const uint32_t st = stored - cu.mod;
        ok = valid && st == computed;
        const uint64_t sj = i - feed.wlo;
        const bool staged = kStage && sj < kXxStageW;
        if (mine && staged) {
          st_out[sj] = valid ? computed : 0u;
          st_ok[sj] = ok ? 1 : 0;
        }
        if (mine && !staged && a.out32) a.out32[i] = valid ? computed : 0u;
        if (mine && a.stored_out) a.stored_out[i] = valid ? st : 0u;
        if (mine && !staged && a.ok_out) a.ok_out[i] = ok ? 1 : 0;
        if (staged) ok = true;  // (counted after the loop)
      } else {
        const uint32_t out = modify_for_last_byte(static_cast<uint32_t>(h), lastb) + cu.mod;
        const uint64_t sj = i - feed.wlo;
        const bool staged = kStage && sj < kXxStageW;
        if (mine && staged) {
          st_out[sj] = valid ? out : 0u;
          st_ok[sj] = valid ? 1 : 0;
          if (MODE == kModeTrailer) st_lb[sj] = static_cast<uint8_t>(lastb);
        }
        if (mine && !staged && a.out32) a.out32[i] = valid ? out : 0u;
        if (MODE == kModeTrailer && mine && valid && !staged) {
          uint8_t* w = a.base_w + off + C.size;
          w[0] = static_cast<uint8_t>(lastb);
          stu32_bytes(w + 1, out);
        }
      }
      if (MODE == kModeVerify) {
        const uint64_t badm = __ballot(mine && !ok);
        if (a.mismatches && badm && lane == 0)
          atomicAdd(a.mismatches, static_cast<unsigned long long>(__popcll(badm)));
      }
    }
    C = I;
    advance(C, I);
    return true;
  };
  while (step(X, Y) && step(Y, X)) {
  }
  if constexpr (kStage) {  // the staged results, coalesced
    __syncthreads();
    const uint64_t lo = feed.wlo, hi = feed.whi;
    const uint64_t m = hi > lo ? (hi - lo < kXxStageW ? hi - lo : kXxStageW) : 0;
    uint32_t bad = 0;
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
      const uint64_t g = lo + j;
      if (a.out32) a.out32[g] = st_out[j];
      if (MODE == kModeVerify) {
        if (a.ok_out) a.ok_out[g] = st_ok[j];
        bad += st_ok[j] ? 0u : 1u;
      }
      if (MODE == kModeTrailer && st_ok[j]) {  // [last byte][LE32] at offset + size
        uint8_t* w = a.base_w + a.offsets[g] + a.sizes[g];
        w[0] = st_lb[j];
        stu32_bytes(w + 1, st_out[j]);
      }
    }
    if (MODE == kModeVerify && a.mismatches) {
      uint32_t wb = bad;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) wb += __shfl_xor(wb, o);
      if (lane == 0 && wb) atomicAdd(a.mismatches, static_cast<unsigned long long>(wb));
    }
  }
}

// ---------------------------------------------------------------------------
// Fragment-aware XXH3 of WAL logical records (log::Reader::ReadRecord's record
// checksum, db/log_reader.cc:95-165), read in place from the log.
//
// log::Writer::AddRecord (db/log_writer.cc:65-160) fills every log block: a
// First or Middle fragment runs to the block end, the next fragment's payload
// starts hs = 7 (11 recyclable) header bytes into the next block.  So a
// logical record of L bytes whose first payload byte is at P0 is the log
// bytes from P0 on with an hs-byte hole at every block start it crosses:
// logical offset p lives at P0 + p + hs * j(p), j(p) = fragment boundaries
// <= p, the first at l0 = 32768 - P0 % 32768, then every D = 32768 - hs bytes.
// The rows kernel layout (one message per 16-lane row, one 1 KiB XXH3-block
// per step) is kept; each row carries (j at the window start, the next
// boundary), at most one boundary falls in a 1 KiB window (D > 1024), and the
// one 16-byte lane slot that straddles it gets a second load hs bytes further
// on, merged bytewise.  Per-message descriptors: offsets = P0, sizes = L,
// init_crcs (reused) = frag_info = hs | j_last << 8 (hs = 0: one fragment;
// j_last = the fragment index of the last stripe).  Records this does not
// describe (short multi-fragment records, a last fragment under 64 bytes,
// middles that do not fill their block) are hashed from a gathered copy by
// the caller.
// ---------------------------------------------------------------------------
constexpr uint32_t kWalBlock = 32768;  // db/log_format.h:45
constexpr uint32_t kNoBound = 0xffffffffu;

struct FRow {
  uint32_t off_lo, off_hi, size, rel, g;
  uint32_t item;  // (fused CRC) the physical record of the first non-empty fragment
  uint32_t info;  // hs | j_last << 8
  uint32_t jc;    // fragment of the window start
  uint32_t bn;    // next boundary (logical offset), kNoBound
  __device__ __forceinline__ uint64_t off() const {
    return (static_cast<uint64_t>(off_hi) << 32) | off_lo;
  }
  __device__ __forceinline__ uint32_t hs() const { return info & 0xffu; }
};

// the window geometry of K chunks per lane (engine.h)
template <uint32_t K>
struct FragGeo {
  static constexpr uint32_t kWin = 256 * K, kShift = K == 8 ? 11 : 10;
  static constexpr uint32_t kXB = kWin / 1024;  // XXH3-blocks (1 KiB) per window
  // FStep::fm bits after m0..m(K-1)
  static constexpr uint32_t kStr = 2 * K, kKs = kStr + 1, kCut = kKs + 3, kOwn = kCut + 5,
                            kQuad = kOwn + 2;
  static_assert(kQuad < 32, "fm bits");
};
template <bool CRC>
constexpr uint32_t frag_k() { return CRC ? kFragKFused : kFragKA14; }
// the fused kernel's candidates are all over 240 bytes with the short path
// (FORST_REC_SHORT, rw_cand_kernel): its rows need no length test
template <bool CRC>
constexpr bool kFusedLong() { return CRC && FORST_REC_SHORT; }

template <uint32_t K>
struct FStep {
  // chunk k's 16 bytes in x[k][0..3]; x[k][4] (the dword after them, for the
  // realignment) is loaded for the last chunk only and made in the step for
  // the others: lane t's next dword is lane t+1's first (lane 15: lane 0's
  // next chunk)
  uint32_t x[K][5];
  uint32_t aux[5];  // the row's last stripe (one quad), or the straddling chunk's own frame
  uint32_t ez[4];  // (fused CRC) E, Z of the window's fragment and of the next one
  // m0..m(K-1) (2 bits each) | straddle:1 | ks:3 | cut:5 (1..16) | m_own:2 |
  // last-stripe quad:1 (0: lanes 0-3, 1: lanes 4-7), at FragGeo's bits
  uint32_t fm;
};

__device__ __forceinline__ void frow_start(FRow& P) {
  P.g = 0;
  P.jc = 0;
  const uint32_t hs = P.hs();
  const uint32_t l0 = kWalBlock - static_cast<uint32_t>(P.off() & (kWalBlock - 1));
  P.bn = (hs && l0 < P.size) ? l0 : kNoBound;
}

template <uint32_t K>
__device__ __forceinline__ void frow_next(FRow& P) {  // window g -> g + 1
  ++P.g;
  if (P.bn != kNoBound && FragGeo<K>::kWin * P.g >= P.bn) {
    ++P.jc;
    const uint32_t nb = P.bn + (kWalBlock - P.hs());
    P.bn = nb < P.size ? nb : kNoBound;
  }
}

template <bool CRC>
__device__ __forceinline__ void frag_issue(const BlockArgs& a, uint32_t lane, const FRow& P,
                                           FStep<frag_k<CRC>()>& d) {
  constexpr uint32_t kFragK = frag_k<CRC>();
  using G = FragGeo<kFragK>;
  const uint32_t t = lane & 15, s4 = t >> 2;
  const uint64_t P0 = P.off();
  const bool valid = P.rel != kNoMsg && P0 <= a.base_len;
  const bool lng = valid && (kFusedLong<CRC>() || P.size > 240);
  const uint32_t nb = (P.size - 1) >> G::kShift;
  const uint32_t hs = P.hs();
  // one fragment (wal_hash.h gathers the others); the fused kernel's
  // candidates are all longer (FORST_REC_SHORT: rw_cand_kernel)
  const bool shrt = (!CRC || !FORST_REC_SHORT) && valid && !lng;
  // Chunk k of lane t sits at window offset 16 t + 256 k, logical offset
  // wpos + 16 t + 256 k.  All chunks of a lane share two physical frames: B
  // (before the window's fragment boundary) and B + hs (past it); their
  // dword-aligned starts differ by dA.  bn >= wpos always (frow_next), so dl
  // (the boundary's offset from the lane's chunk 0) fits in 32 bits.
  const uint32_t lof = 16 * t;
  const uint32_t wpos = G::kWin * P.g;
  const uint32_t dw = P.bn - wpos;
  const int32_t dl = static_cast<int32_t>(dw < 4096u ? dw : 4096u) - static_cast<int32_t>(lof);
  const uint64_t B = P0 + wpos + lof + static_cast<uint64_t>(hs) * P.jc;
  const uint32_t m0 = static_cast<uint32_t>(B) & 3u;
  const uint32_t m1 = (static_cast<uint32_t>(B) + hs) & 3u;
  const uint32_t dA = ((static_cast<uint32_t>(B) + hs) & ~3u) - (static_cast<uint32_t>(B) & ~3u);
  // Every chunk of a long record's window is loaded, needed or not: the
  // callers (wh_prep_kernel, rw_cand_kernel) keep records that end within
  // kFragTail bytes of the log end out of this kernel, so a window's 1 KiB
  // (plus the header hole and the realignment dwords) past the record end is
  // in the buffer.  Rows without a record load [0, 1 KiB) of the buffer
  // (launches need 4 KiB).  A chunk's address is the lane's frame, plus the
  // hole when the boundary lies at or before the chunk's END (so a chunk
  // that straddles the boundary, or ends exactly at it, is loaded from the
  // shifted frame and its own-frame bytes come from the aux load below), with
  // the chunk's 256 k as the load's immediate offset.  The short-record,
  // boundary and last-stripe addresses are worked out only in steps where
  // some row needs them; the loads themselves are unconditional, so every
  // step issues the same loads (the compiler's vmcnt waits stay precise).
  const uint8_t* R = a.base + (valid ? (B & ~3ull) : 0ull);
  // XXH3 only: a chunk that starts past the record end (its first dword may
  // still hold the realignment bytes of the lane in front) is read from the
  // buffer start instead -- the last window's tail is the next record's,
  // which its own row reads (C5 a14 -1.7 %).  The fused kernel loads them
  // (A/B: the redirect's registers cost it 3.6 %)
  const uint32_t rem4 = (valid ? P.size - wpos : 0u) + 4u;
  uint32_t fm = 0;
#pragma unroll
  for (uint32_t k = 0; k < kFragK; ++k) {
    const bool past = lng && dl <= static_cast<int32_t>(256 * k + 16);
    const bool need = CRC || (valid && 16 * t + 256 * k < rem4);
    const uint8_t* pq = (need ? R : a.base) + (past ? dA : 0u) + 256 * k;
    uint32_t mm = past ? m1 : m0;
    if (k >= 2 && k < 4 && __ballot(shrt)) {
      // a short record: its window layout in x[0], x[1] (the fused CRC reads
      // it), its XXH3 chunk (xxh3_short_row) in x[2] and the 16 bytes after
      // that in x[3], whose first dword realigns it (the record ends >=
      // kFragTail bytes before the log end)
      const uint64_t sp = short_phys(P0, P.size, FR(lane) & 15u);
      if (shrt) {
        pq = a.base + (sp & ~3ull) + 16 * (k - 2);
        mm = static_cast<uint32_t>(sp) & 3u;
      }
    }
    const u32x4a4 v = ld16_a4(pq);
    d.x[k][0] = v.x;
    d.x[k][1] = v.y;
    d.x[k][2] = v.z;
    d.x[k][3] = v.w;
    if (k == kFragK - 1) d.x[k][4] = ld4_a4(pq + 16);
    fm |= mm << (2 * k);
  }
  // The chunk that straddles the boundary or ends at it (0 < dl - 256 ks <=
  // 16): its bytes before the boundary come from its own frame, loaded into
  // aux with their realignment dword.  (Geometric, not "needed": the lane in
  // front of it takes its realignment dword from this aux, see the step.)
  bool straddle = false;
  uint32_t ks = 0;
  if (__ballot(lng && dw <= G::kWin)) {  // a boundary in, or at the end of, some row's window
    ks = static_cast<uint32_t>(dl - 1) >> 8;
    const int32_t cut = dl - static_cast<int32_t>(256 * ks);
    straddle = lng && dl > 0 && dl <= static_cast<int32_t>(256 * (kFragK - 1) + 16) && cut <= 16;
    if (straddle)
      fm |= (1u << G::kStr) | (ks << G::kKs) | (static_cast<uint32_t>(cut) << G::kCut) |
            (m0 << G::kOwn);
  }
  // The last stripe at L - 64, inside the last fragment (fragment j_last):
  // every quad of the row would compute the same merge, so one quad loads
  // it -- quad 0, or quad 1 when quad 0 holds the row's straddling chunk --
  // into the same aux slot (one aux load per step instead of two)
  const bool lastp = lng && P.g == nb;
  const uint8_t* q0 = a.base;
  const uint8_t* q4 = a.base;
  if (__ballot(lastp || straddle)) {
    const uint32_t rowm = static_cast<uint32_t>(__ballot(straddle) >> (lane & 48u)) & 0xffffu;
    const uint32_t ql = (rowm & 0xfu) ? 1u : 0u;
    if (lastp && ql) fm |= 1u << G::kQuad;
    if (straddle) {
      q0 = R + 256 * ks;
      q4 = q0 + 16;
    } else if (lastp && s4 == ql) {
      const uint64_t lq = P0 + (P.size - 64u + 16u * (FR(lane) & 3u)) +
                            static_cast<uint64_t>(hs) * (P.info >> 8);
      q0 = a.base + (lq & ~3ull);
      q4 = (lq & 3) ? q0 + 16 : q0;  // (the stripe ends at the record end)
    }
  }
  const u32x4a4 av = ld16_a4(q0);
  d.aux[0] = av.x;
  d.aux[1] = av.y;
  d.aux[2] = av.z;
  d.aux[3] = av.w;
  d.aux[4] = ld4_a4(q4);
  d.fm = fm;
  if (CRC) {  // E, Z of the window's fragment jc and of jc + 1 (one 16-byte
              // load: crc_ez holds one entry more than there are items)
    const uint64_t i0 = valid && P.size > 0 ? static_cast<uint64_t>(P.item) + P.jc : 0;
    const u32x4a4 ez = ld16_a4(reinterpret_cast<const uint8_t*>(a.crc_ez + i0));
    d.ez[0] = ez.x;
    d.ez[1] = ez.y;
    d.ez[2] = ez.z;
    d.ez[3] = ez.w;
  }
}

// WPE: waves per SIMD the register allocation targets (3, the default: round
// 5 builds, the a14 kernel 167 VGPRs and the fused one 164, no VGPR spills;
// C5 a14 21.5 vs 24.8 ms at 2 in round 2)
// the fused CRC's tables: [0, 64K) G and J244 (one chain per lane; J1012 for
// the column chains) replicated (crc_lds.h), [64K, 124K) A16[1..15], [124K,
// 136K) C256[1..3]; constant trip counts (see fill_tables3)
template <uint32_t NT>
__device__ __forceinline__ void fill_frag_crc_tables(uint32_t* L) {
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t kN1 = (16384 + NT - 1) / NT, kN2 = (18 * 1024 + NT - 1) / NT;
  uint32_t v1[kN1], v2[kN2];
#pragma unroll
  for (uint32_t k = 0; k < kN1; ++k) {
    const uint32_t i = tid + k * NT;
    const uint32_t e = (i >> 6) & 255, d = i & 63, t = (d >> 3) & 3;
    v1[k] = i < 16384 ? (d < 32 ? kCrcG[t * 256 + e]
                                : (kNC == 1 ? kCrcJ244[t * 256 + e] : kCrcJ1012[t * 256 + e]))
                      : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kN2; ++k) {
    const uint32_t i = tid + k * NT;
    v2[k] = i < 15 * 1024 ? kCrcA16[i] : (i < 18 * 1024 ? kCrcC256[i - 15 * 1024] : 0u);
  }
#pragma unroll
  for (uint32_t k = 0; k < kN1; ++k)
    if (tid + k * NT < 16384) L[tid + k * NT] = v1[k];
#pragma unroll
  for (uint32_t k = 0; k < kN2; ++k)
    if (tid + k * NT < 18 * 1024) L[kFcOffA16 / 4 + tid + k * NT] = v2[k];
}

// ---- WAL recovery's short candidates: CRC32C and XXH3 on one 16-lane row --
// One record per row (wal_recover.hip's short list: CRC'd bytes under 253,
// payload <= 240).  CRC: the message right-aligned in a 256-byte window
// behind the 4 bytes P with raw_0(P) = ~0 (so the window's raw CRC from 0 is
// crc32c's value with its init) and zeros; lane t holds window bytes
// [16 t, 16 t + 16): its raw chunk CRC (16 G lookups) moved to the window
// end (A16[14 - t], the fused kernel's tables), then a DPP XOR over the row.
// XXH3: the chunk of xxh3_short_row's layout, as xxh3_short_rows_kernel.
// A record within 32 bytes of the log start (whose window would begin before
// the buffer) or near its end is CRC'd byte by byte by lane 0 of its row.
constexpr uint32_t kShortCrcThreads = 1024;  // one workgroup per CU: 136 KiB of tables
constexpr uint32_t kShortCrcU = 2;           // records per row in flight
constexpr uint32_t kCrcInitPrefix = 0x641f6454u;  // P, little-endian: raw CRC from 0 = 0xffffffff
__device__ __forceinline__ uint32_t fcrc_chunk_raw(const uint8_t* __restrict__ Lb,
                                                   const fcrc::Lanes& K, uint32_t w0, uint32_t w1,
                                                   uint32_t w2, uint32_t w3) {
  uint32_t l[4];
  fcrc::look<false>(Lb, K, w0, l);
  uint32_t x = fcrc::xor3(l[0], l[1], fcrc::xor3(l[2], l[3], w1));
  x = fcrc::g_then(Lb, K, x, w2);
  x = fcrc::g_then(Lb, K, x, w3);
  return fcrc::g_then(Lb, K, x, 0u);
}
__global__ void __launch_bounds__(kShortCrcThreads) wal_short_rows_kernel(
    const uint8_t* base, uint64_t base_len, const uint64_t* coff, const uint32_t* clen,
    const uint64_t* p0, const uint32_t* plen, const uint64_t* item, uint64_t n,
    const uint32_t* stored, uint8_t* crc_ok, uint64_t* hash_out) {
  __shared__ uint32_t crcL[kFcLds / 4];
  __shared__ __attribute__((aligned(16))) uint32_t kmask[17 * 4];
  __shared__ uint64_t shsec[64];
  fill_frag_crc_tables<kShortCrcThreads>(crcL);
  if (threadIdx.x < 17 * 4) kmask[threadIdx.x] = fcrc::keep_word(threadIdx.x >> 2, threadIdx.x & 3);
  short_secrets_fill(shsec, threadIdx.x);
  __syncthreads();
  const uint8_t* Lb = reinterpret_cast<const uint8_t*>(crcL);
  const uint32_t lane = threadIdx.x & 63, t = lane & 15, row = lane >> 4;
  const uint64_t wave = uniform(threadIdx.x >> 6);
  const fcrc::Lanes FK = fcrc::lanes(lane);
  constexpr uint64_t kPerWave = 4 * kShortCrcU;
  const uint64_t step = kPerWave * gridDim.x * (kShortCrcThreads / 64);
  // the list entries of the next round are loaded while this round's data
  // loads are in flight (one memory round trip per round, not two)
  uint64_t co[kShortCrcU], pp[kShortCrcU], it[kShortCrcU];
  uint32_t cl[kShortCrcU], pl[kShortCrcU];
  auto load_list = [&](uint64_t kb) {
#pragma unroll
    for (uint32_t u = 0; u < kShortCrcU; ++u) {
      const uint64_t k = kb + 4 * u + row;
      const bool v = k < n;
      co[u] = v ? coff[k] : 0ull;
      cl[u] = v ? clen[k] : 0u;
      pp[u] = v ? p0[k] : 0ull;
      pl[u] = v ? plen[k] : 0u;
      it[u] = v ? item[k] : 0ull;
    }
  };
  uint64_t k0 = kPerWave * (static_cast<uint64_t>(blockIdx.x) * (kShortCrcThreads / 64) + wave);
  load_list(k0);
  for (; k0 < n; k0 += step) {  // (wave-uniform: the row sums need every lane)
    u32x4a4 cc[kShortCrcU], xc[kShortCrcU];
    uint32_t cn[kShortCrcU], xn[kShortCrcU], stv[kShortCrcU];
    uint64_t ca[kShortCrcU], xp[kShortCrcU];
    bool fast[kShortCrcU], ok[kShortCrcU];
#pragma unroll
    for (uint32_t u = 0; u < kShortCrcU; ++u) {
      const uint64_t k = k0 + 4 * u + row;
      ok[u] = k < n && pl[u] <= 240 && pp[u] <= base_len && pl[u] <= base_len - pp[u];
      // CRC: window byte 16 t is message byte 16 t - s, s = 256 - clen
      fast[u] = k < n && cl[u] <= 252 && co[u] >= 32 && co[u] <= base_len &&
                base_len - co[u] >= uint64_t(cl[u]) + 4;
      ca[u] = fast[u] ? co[u] + 16 * t - (256 - cl[u]) : 0ull;  // (>= co - 260 + 16 t)
      const uint64_t cq = (fast[u] && 16 * t + 16 > 256 - cl[u] - 4) ? (ca[u] & ~3ull) : 0ull;
      cc[u] = ld16_a4(base + cq);
      cn[u] = ld4_a4(base + cq + 16);
      // XXH3: the chunk of xxh3_short_row's layout
      xp[u] = ok[u] ? short_phys(pp[u], pl[u], t) : 0ull;
      const uint64_t xq = (xp[u] & ~3ull) + 20 <= base_len ? (xp[u] & ~3ull) : 0ull;
      xc[u] = ld16_a4(base + xq);
      xn[u] = ld4_a4(base + xq + 16);
      stv[u] = k < n ? stored[it[u]] : 0u;
    }
    // this round's list values, then the next round's list loads
    uint64_t co_[kShortCrcU], pp_[kShortCrcU], it_[kShortCrcU];
    uint32_t cl_[kShortCrcU], pl_[kShortCrcU];
#pragma unroll
    for (uint32_t u = 0; u < kShortCrcU; ++u) {
      co_[u] = co[u];
      pp_[u] = pp[u];
      it_[u] = it[u];
      cl_[u] = cl[u];
      pl_[u] = pl[u];
    }
    load_list(k0 + step);
#pragma unroll
    for (uint32_t u = 0; u < kShortCrcU; ++u) {
      const uint64_t k = k0 + 4 * u + row;
      // ---- CRC
      const uint32_t sw = 256 - cl_[u];  // the message's window start
      const bool live = fast[u] && 16 * t + 16 > sw - 4;
      const uint32_t m = static_cast<uint32_t>(ca[u] & 3);
      uint32_t w[4] = {__builtin_amdgcn_alignbyte(cc[u].y, cc[u].x, m),
                       __builtin_amdgcn_alignbyte(cc[u].z, cc[u].y, m),
                       __builtin_amdgcn_alignbyte(cc[u].w, cc[u].z, m),
                       __builtin_amdgcn_alignbyte(cn[u], cc[u].w, m)};
      const int32_t b0 = static_cast<int32_t>(sw) - static_cast<int32_t>(16 * t);
      const uint32_t bk = live ? (b0 <= 0 ? 0u : (b0 >= 16 ? 16u : static_cast<uint32_t>(b0))) : 16u;
      const u32x4 km = *reinterpret_cast<const u32x4*>(kmask + 4 * bk);
      const int32_t o = b0 - 4;  // P's first byte in the lane's chunk
      uint32_t pd[4];
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) {
        const int32_t x = o - static_cast<int32_t>(4 * i) + 4;
        pd[i] = live && x >= 0 && x < 8
                    ? static_cast<uint32_t>((static_cast<uint64_t>(kCrcInitPrefix) << (8 * x)) >> 32)
                    : 0u;
      }
      w[0] = (w[0] & ~km.x) | pd[0];
      w[1] = (w[1] & ~km.y) | pd[1];
      w[2] = (w[2] & ~km.z) | pd[2];
      w[3] = (w[3] & ~km.w) | pd[3];
      uint32_t v = fcrc_chunk_raw(Lb, FK, w[0], w[1], w[2], w[3]);
      v = t == 15 ? v : fcrc::shift_at(Lb, kFcOffA16 + 4096 * (14 - t), v);
      v = fcrc::row_ror_xor<1>(v);
      v = fcrc::row_ror_xor<2>(v);
      v = fcrc::row_ror_xor<4>(v);
      v = fcrc::row_ror_xor<8>(v);
      uint32_t crc = ~v;
      if (k < n && !fast[u] && t == 0) {  // byte by byte (G3: table 3, copy 0)
        uint32_t r = 0xffffffffu;
        const uint64_t e = co_[u] + cl_[u];
        for (uint64_t q = co_[u]; q < e && q < base_len; ++q)
          r = (r >> 8) ^ fcrc::lds32(Lb, 256 * ((r ^ ldu8(base + q)) & 0xffu) + 96);
        crc = co_[u] <= base_len && base_len - co_[u] >= cl_[u] ? ~r : ~stv[u];
      }
      // ---- XXH3
      if ((xp[u] & ~3ull) + 20 > base_len) {
        xc[u] = ld16_lim(base, base_len, xp[u] & ~3ull);
        xn[u] = ld4_lim(base, base_len, (xp[u] & ~3ull) + 16);
      }
      const uint32_t xm = static_cast<uint32_t>(xp[u] & 3);
      const uint64_t d0 = mk64(__builtin_amdgcn_alignbyte(xc[u].y, xc[u].x, xm),
                               __builtin_amdgcn_alignbyte(xc[u].z, xc[u].y, xm));
      const uint64_t d1 = mk64(__builtin_amdgcn_alignbyte(xc[u].w, xc[u].z, xm),
                               __builtin_amdgcn_alignbyte(xn[u], xc[u].w, xm));
      const uint32_t pb = ok[u] ? static_cast<uint32_t>(pp_[u] - short_phys(pp_[u], pl_[u], 0)) : 0u;
      const uint64_t h = xxh3_short_row(d0, d1, pl_[u], t, pb, shsec);
      if (k < n && t == 0) {
        crc_ok[it_[u]] = crc == stv[u] ? 1 : 0;
        hash_out[it_[u]] = ok[u] ? h : 0ull;
      }
    }
  }
}

// CRC = true (fused WAL recovery, wal_recover.hip): besides the XXH3 of every
// logical record, the CRC32C of each of its physical records (fragments) is
// checked from the same loads.  CRC32C is linear: a fragment's CRC over
// header[6..hs) || payload is H * x^(8|p|) + raw(payload) (H = the state after
// the header bytes from ~0), and raw(payload) is the XOR of every payload
// chunk's contribution moved to a common end.  Lane t of a row holds the 16 B
// chunks at window offsets 16t + 256k and runs one chain per column k over
// the windows (J1012: the 1008-byte hop to the column's next chunk fused with
// the first dword step; four independent chains, so the LDS lookups of one
// step form four short dependency chains, not one 16 deep); after the window
// column k sits 16 (15 - t) + 256 (3 - k) bytes before the window end.  A
// fragment that ends in the window is finished by moving the columns onto
// column 3 (C256), every lane to the window end (A16[15 - t]), XOR-reducing
// the row, and comparing with Z = ~stored * x^(8m) (m = bytes
// from the fragment end to the window end).  Bytes outside the fragment are
// masked to zero.  H enters as E = H * x^(8 (window end - fragment start)),
// added at the end of the fragment's first window (into lane 15's column-3
// chain, which ends at the window end).  E and Z per physical record come from the caller
// (rw_cand_kernel); the verdict goes to crc_ok[physical record].  A window
// holding a fragment boundary runs a second pass for the next fragment.
// DEPTH: steps of loads in flight per wave (DEPTH + 1 step buffers rotate):
// the kernel's memory rate is its bytes in flight (waves x DEPTH x 4 KiB per
// CU) over the load latency, so fewer waves can carry more steps each
template <int WPE, bool CRC, int DEPTH = 1>
__global__ void __launch_bounds__(CRC ? kFragCrcThreads : kFragThreads) FORST_WAVES_PER_EU(WPE)
xxh3_frag_kernel(BlockArgs a) {
  static_assert(DEPTH >= 1 && DEPTH <= 3, "1..3 steps in flight");
  constexpr uint32_t kFragK = frag_k<CRC>();
  using G = FragGeo<kFragK>;
  using FStep = forst::FStep<kFragK>;
  // cold per-pair constants and the accumulate keys live in LDS (registers
  // go to the fragment bookkeeping): key of stripe s, pair p = secret64[s + 2p]
  __shared__ uint64_t cold[4 * kColdN];
  __shared__ uint64_t keys[24];
  __shared__ uint64_t shsec[64];
  __shared__ uint32_t crcL[CRC ? kFcLds / 4 : 1];
  // kmask[4 n + i]: the mask of dword i of a chunk whose first n bytes are
  // kept (n = 0..16)
  __shared__ __attribute__((aligned(16))) uint32_t kmask[CRC ? 17 * 4 : 4];
  constexpr uint32_t FW = CRC ? kFragCrcWaves : kFragWaves;
  if (kFragWg) feed_init();
  if (threadIdx.x < 4 * kColdN) cold[threadIdx.x] = (&kXxCold[0][0])[threadIdx.x];
  if (threadIdx.x < 24) keys[threadIdx.x] = sec64(8 * threadIdx.x);
  short_secrets_fill(shsec, threadIdx.x);
  if constexpr (CRC) {
    fill_frag_crc_tables<kFragCrcThreads>(crcL);
    if (threadIdx.x < 17 * 4) kmask[threadIdx.x] = fcrc::keep_word(threadIdx.x >> 2, threadIdx.x & 3);
  }
  __syncthreads();
  const uint8_t* Lb = reinterpret_cast<const uint8_t*>(crcL);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t t = lane & 15, s4 = t >> 2, p = t & 3;
  // K0[k] = keys[s4 + 2p + 4k], K1[k] = keys[s4 + 2p + 4k + 1]
  // (the scramble keys sec64(128 + 16p), sec64(136 + 16p) are keys[16 + 2p],
  // keys[17 + 2p], read where used: one spilled register pair fewer)
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * FW;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * FW + wave;
  BatchFeed feed;
  uint64_t cg = feed_first<kFragWg, 64>(a, nw, gw, lane, feed);
  if (cg >= a.n) return;
  uint32_t clen = feed.len;  // entries of cb / nb (a batch holds up to 64)
  uint64_t ng = feed_next<kFragWg, 64>(a, nw, lane, feed);
  uint32_t nlen = feed.len;
  DescBatch cb, nb;
  uint64_t kbrel = 0;
  load_batch<kModeRaw>(a, cg, a.n, lane, cb);  // extra = frag_info (init_crcs)
  load_batch<kModeRaw>(a, ng, a.n, lane, nb);  // mod = first physical record (fused CRC)
  auto fetch = [&](uint64_t rel, FRow& P) {
    const BatchSlot q = batch_slot(rel, kbrel, cg, clen, ng, nlen, a.n);
    const uint32_t lo_c = __shfl(cb.off_lo, q.src), hi_c = __shfl(cb.off_hi, q.src);
    const uint32_t sz_c = __shfl(cb.size, q.src), in_c = __shfl(cb.extra, q.src);
    const uint32_t lo_n = __shfl(nb.off_lo, q.src), hi_n = __shfl(nb.off_hi, q.src);
    const uint32_t sz_n = __shfl(nb.size, q.src), in_nn = __shfl(nb.extra, q.src);
    P.off_lo = q.in_n ? lo_n : lo_c;
    P.off_hi = q.in_n ? hi_n : hi_c;
    P.size = q.in_n ? sz_n : sz_c;
    P.info = q.in_n ? in_nn : in_c;
    if (CRC) {
      const uint32_t it_c = __shfl(cb.mod, q.src), it_n = __shfl(nb.mod, q.src);
      P.item = q.in_n ? it_n : it_c;
    } else {
      P.item = 0;
    }
    P.rel = q.valid ? static_cast<uint32_t>(q.gi) : kNoMsg;
    frow_start(P);
  };
  const uint32_t row = lane >> 4;
  uint64_t next = 4;
  FRow C;
  fetch(row, C);
  auto advance = [&](const FRow& P, FRow& I) {
    const bool lng = P.rel != kNoMsg && (kFusedLong<CRC>() || P.size > 240);
    const uint32_t nbP = (P.size - 1) >> G::kShift;
    const bool more = lng && P.g < nbP;
    const bool need = P.rel != kNoMsg && !more;
    const uint64_t rows = __ballot(need && t == 0);
    I = P;
    if (more) frow_next<kFragK>(I);
    if (rows) {  // descriptor work only in steps where some row takes a record
      const uint32_t rank = static_cast<uint32_t>(__popcll(rows & ((1ull << (lane & ~15u)) - 1)));
      FRow F;
      fetch(next + rank, F);
      next += static_cast<uint64_t>(__popcll(rows));
      if (need) I = F;
      if (next >= kbrel + clen) {
        kbrel += clen;
        clen = nlen;
        cb = nb;
        cg = ng;
        ng = feed_next<kFragWg, 64>(a, nw, lane, feed);
        nlen = feed.len;
        load_batch<kModeRaw>(a, ng, a.n, lane, nb);
#ifndef FORST_HOST_EMULATION
        // retire the descriptor loads on this (rare) path: left pending, they
        // make the compiler's waits at the next step's start count them on
        // every path, i.e. wait out the data loads in flight
        asm volatile("" ::"v"(nb.off_lo), "v"(nb.off_hi), "v"(nb.size), "v"(nb.extra));
#endif
      }
    }
  };
  // Q[d]: the row position d + 1 steps ahead of C; the step issues the loads
  // of Q[DEPTH - 1]
  FRow Q[DEPTH];
  advance(C, Q[0]);
#pragma unroll
  for (int d = 1; d < DEPTH; ++d) advance(Q[d - 1], Q[d]);
  FStep B[DEPTH + 1];
  frag_issue<CRC>(a, lane, C, B[0]);
#pragma unroll
  for (int d = 1; d < DEPTH; ++d) frag_issue<CRC>(a, lane, Q[d - 1], B[d]);
  uint64_t acc0 = 0, acc1 = 0;
  uint32_t crc_s[kNC];  // (fused CRC) the lane's chain(s)
#pragma unroll
  for (uint32_t k = 0; k < kNC; ++k) crc_s[k] = 0u;
  const fcrc::Lanes FK = fcrc::lanes(lane);
  auto step = [&](FStep& cu, FStep& nx) -> bool {
    // no early return: both step copies issue on every path round the loop,
    // so the compiler's waits at the loop head see the other copy's loads as
    // the younger ones (an exit path between the copies made them wait out
    // the step in flight before issuing the next)
    const bool live = __ballot(C.rel != kNoMsg) != 0;
    frag_issue<CRC>(a, lane, Q[DEPTH - 1], nx);
#ifndef FORST_HOST_EMULATION
    // keep the next step's loads here, ahead of this step's compute (without
    // the fence they are sunk below the step's conditional code, and the
    // step waits out its own data before the next one is even issued)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
    const bool valid = C.rel != kNoMsg && C.off() <= a.base_len;
    const bool lng = valid && (kFusedLong<CRC>() || C.size > 240);
    // XXH3-blocks: nbC full ones (scrambled), then nbSC stripes of the last
    const uint32_t nbC = (C.size - 1) >> 10, nbSC = ((C.size - 1) & 1023) >> 6;
    if (C.g == 0) {  // XXH3_INIT_ACC (xxhash.h:5188)
      const uint64_t* ci = cold + kColdN * (FR(lane) & 3u);
      acc0 = ci[kColdI0];
      acc1 = ci[kColdI1];
    }
    uint64_t sum0 = 0, sum1 = 0;
    uint32_t fm = cu.fm;
    // realignment dwords of chunks 0..2: lane t's next dword is lane t+1's
    // first, lane 15's is lane 0's in the next chunk (DPP row_ror 15 reads
    // lane t+1 of the row); a short row's chunk 0 is followed by its x[1]
#pragma unroll
    for (uint32_t k = 0; k + 1 < kFragK; ++k) {
      const uint32_t nx = __builtin_amdgcn_mov_dpp(cu.x[k][0], 0x12F, 0xf, 0xf, true);
      const uint32_t nn = __builtin_amdgcn_mov_dpp(cu.x[k + 1][0], 0x12F, 0xf, 0xf, true);
      cu.x[k][4] = t == 15 ? nn : nx;
    }
    if ((!CRC || !FORST_REC_SHORT) && valid && !lng) cu.x[2][4] = cu.x[3][0];
    // the chunk across the boundary (one lane per row, in ~1 step in 32):
    // its bytes before the boundary come from its own frame (aux), the rest
    // from the shifted frame (x), merged once, out of line, into that chunk's
    // words (realigned, m := 0), so the chunk loop below carries no
    // per-chunk test.  The lane in front of it realigns with the aux frame.
    if (__ballot((fm >> G::kStr) & 1u)) {
      uint32_t f2 = fm;
#ifndef FORST_HOST_EMULATION
      asm volatile("" : "+v"(f2));  // nothing of the merge is hoisted out of the branch
#endif
      const uint32_t sk = ((f2 >> G::kStr) & 1u) ? (f2 >> G::kKs) & 7u : 31u;
      const uint32_t nsk = __builtin_amdgcn_mov_dpp(sk, 0x12F, 0xf, 0xf, true);
      const uint32_t na0 = __builtin_amdgcn_mov_dpp(cu.aux[0], 0x12F, 0xf, 0xf, true);
#pragma unroll
      for (uint32_t k = 0; k + 1 < kFragK; ++k)
        if (nsk == (t == 15 ? k + 1 : k)) cu.x[k][4] = na0;
      if ((f2 >> G::kStr) & 1u) {
        uint64_t a0, a1;
        xx_words(cu.aux, (f2 >> G::kOwn) & 3u, a0, a1);
        const uint32_t cut = (f2 >> G::kCut) & 31u;  // bytes before the boundary, 1..16
        const uint64_t mlo = cut >= 8 ? ~0ull : ((1ull << (8 * cut)) - 1);
        const uint64_t mhi = cut >= 16 ? ~0ull : (cut > 8 ? ((1ull << (8 * (cut - 8))) - 1) : 0ull);
        const uint32_t ks = (f2 >> G::kKs) & 7u;
#pragma unroll
        for (uint32_t k = 0; k < kFragK; ++k) {
          if (ks == k) {
            uint64_t d0, d1;
            xx_words(cu.x[k], (f2 >> (2 * k)) & 3u, d0, d1);
            d0 = (a0 & mlo) | (d0 & ~mlo);
            d1 = (a1 & mhi) | (d1 & ~mhi);
            cu.x[k][0] = static_cast<uint32_t>(d0);
            cu.x[k][1] = static_cast<uint32_t>(d0 >> 32);
            cu.x[k][2] = static_cast<uint32_t>(d1);
            cu.x[k][3] = static_cast<uint32_t>(d1 >> 32);
          }
        }
        fm = f2 & ~(3u << (2 * ks));
      }
    }
    // re-read the keys from LDS every step (an opaque index keeps the
    // compiler from hoisting them back into registers)
    uint32_t kix = s4 + 2 * p;
#ifndef FORST_HOST_EMULATION
    asm volatile("" : "+v"(kix));
#endif
    const uint64_t* kq = keys + kix;
    // (fused CRC) this window's bytes of fragment jc: [0, hiA)
    // (short records: their one fragment from the window layout in x[0], x[1];
    // an empty one is CRC'd by the rows kernel, rw_cand_kernel)
    const bool crow = CRC && valid && C.size > 0;
    uint32_t hiA = G::kWin;
    if (CRC) {
      const uint32_t fe = C.bn < C.size ? C.bn : C.size;
      const uint32_t W0 = G::kWin * C.g;
      hiA = fe - W0 < G::kWin ? fe - W0 : G::kWin;
    }
    uint32_t cs[kNC];
#pragma unroll
    for (uint32_t k = 0; k < kNC; ++k) cs[k] = crc_s[k];
    uint64_t sumB0 = 0, sumB1 = 0;  // (kFragK = 8) the window's second XXH3-block
#pragma unroll
    for (uint32_t k = 0; k < kFragK; ++k) {
      uint64_t d0, d1;
      xx_words(cu.x[k], (fm >> (2 * k)) & 3u, d0, d1);
      const uint32_t kk = k & 3u;  // stripe s4 + 4 kk of XXH3-block kFragXB g + k / 4
      const uint64_t c0 = mul32to64(d0 ^ kq[4 * kk]) + d1;  // acc[2p] (xxhash.h:4926-4927)
      const uint64_t c1 = d0 + mul32to64(d1 ^ kq[4 * kk + 1]);  // acc[2p+1]
      const uint32_t xb = G::kXB * C.g + (k >> 2);
      const bool use = xb < nbC || (xb == nbC && s4 + 4 * kk < nbSC);
      if (k < 4) {
        sum0 += use ? c0 : 0ull;
        sum1 += use ? c1 : 0ull;
      } else {
        sumB0 += use ? c0 : 0ull;
        sumB1 += use ? c1 : 0ull;
      }
      if (CRC) {
        const uint32_t kc = kNC == 1 ? 0u : k;  // the chain: the lane's one, or column k's
        const uint32_t q = 16 * t + 256 * k;
#if FORST_FRAG_MASK_LDS
        const uint32_t n = hiA > q ? (hiA - q < 16u ? hiA - q : 16u) : 0u;
        const u32x4 m = *reinterpret_cast<const u32x4*>(kmask + 4 * n);
        cs[kc] = fcrc::chunk_step(Lb, FK, cs[kc], static_cast<uint32_t>(d0) & m.x,
                                 static_cast<uint32_t>(d0 >> 32) & m.y,
                                 static_cast<uint32_t>(d1) & m.z,
                                 static_cast<uint32_t>(d1 >> 32) & m.w);
#else
        uint64_t m0 = ~0ull, m1 = ~0ull;
        if (hiA < q + 16) fcrc::keep_mask(0, hiA > q ? hiA - q : 0u, m0, m1);
        const uint64_t e0 = d0 & m0, e1 = d1 & m1;
        cs[kc] = fcrc::chunk_step(Lb, FK, cs[kc], static_cast<uint32_t>(e0),
                                  static_cast<uint32_t>(e0 >> 32), static_cast<uint32_t>(e1),
                                  static_cast<uint32_t>(e1 >> 32));
#endif
      }
    }
    if (CRC) {
      // the fragment's end in this window: finish it (and a fragment that
      // starts here: second pass); else carry the chain, E added at the end
      // of the fragment's first window
      const uint32_t W0 = G::kWin * C.g, L = C.size;
      const uint32_t fe = C.bn < L ? C.bn : L;
      const bool ends = crow && fe - W0 <= G::kWin;
      const uint32_t l0 = kWalBlock - static_cast<uint32_t>(C.off() & (kWalBlock - 1));
      const uint32_t fs = C.jc == 0 ? 0u : l0 + (C.jc - 1) * (kWalBlock - C.hs());
      const bool started = (fs >> G::kShift) == C.g;
      const bool carry = crow && !ends;
      uint32_t ns[kNC];
#pragma unroll
      for (uint32_t k = 0; k < kNC; ++k) ns[k] = carry ? cs[k] : 0u;
      if (carry && started && t == 15) ns[kNC - 1] ^= cu.ez[0];
      auto row_value = [&](const uint32_t (&c)[kNC]) {  // chains -> the row's value at the window end
        uint32_t v = c[kNC - 1];
        if (kNC == 4)  // columns 0..2 onto column 3 (256 (3 - k) bytes on)
          v ^= fcrc::shift_at(Lb, kFcOffC256, c[kNC == 4 ? 2 : 0]) ^
               fcrc::shift_at(Lb, kFcOffC256 + 4096, c[kNC == 4 ? 1 : 0]) ^
               fcrc::shift_at(Lb, kFcOffC256 + 8192, c[0]);
        v = t == 15 ? v : fcrc::shift_at(Lb, kFcOffA16 + 4096 * (14 - t), v);
        v = fcrc::row_ror_xor<1>(v);
        v = fcrc::row_ror_xor<2>(v);
        v = fcrc::row_ror_xor<4>(v);
        return fcrc::row_ror_xor<8>(v);
      };
      if (__ballot(ends)) {
        const uint32_t V = row_value(cs) ^ (started ? cu.ez[0] : 0u);
        // every verdict is stored (the caller pre-fills crc_ok with 0: a
        // fragment whose row never reaches its end reads as a mismatch)
        if (ends && t == 0) a.crc_ok[static_cast<uint64_t>(C.item) + C.jc] = V == cu.ez[1] ? 1 : 0;

        const bool pb = ends && C.bn < L && C.bn - W0 < G::kWin;
        if (__ballot(pb)) {  // fragment jc + 1 starts in this window: [B, hiB)
          const uint32_t B = C.bn - W0;
          const uint32_t hiB = L - W0 < G::kWin ? L - W0 : G::kWin;
          uint32_t sb[kNC];
#pragma unroll
          for (uint32_t k = 0; k < kNC; ++k) sb[k] = 0u;
#pragma unroll
          for (uint32_t k = 0; k < kFragK; ++k) {
            uint64_t d0, d1;
            xx_words(cu.x[k], (fm >> (2 * k)) & 3u, d0, d1);
            const uint32_t q = 16 * t + 256 * k;
            const uint32_t ka = B > q ? (B - q < 16u ? B - q : 16u) : 0u;
            const uint32_t kb = hiB > q ? (hiB - q < 16u ? hiB - q : 16u) : 0u;
#if FORST_FRAG_MASK_LDS
            // bytes [ka, kb): mask(kb) & ~mask(ka)
            const u32x4 mb = *reinterpret_cast<const u32x4*>(kmask + 4 * (kb > ka ? kb : ka));
            const u32x4 ma = *reinterpret_cast<const u32x4*>(kmask + 4 * ka);
            const uint32_t kc = kNC == 1 ? 0u : k;
            sb[kc] = fcrc::chunk_step(
                Lb, FK, sb[kc], __builtin_amdgcn_bitop3_b32(static_cast<uint32_t>(d0), mb.x, ma.x, 0x40),
                __builtin_amdgcn_bitop3_b32(static_cast<uint32_t>(d0 >> 32), mb.y, ma.y, 0x40),
                __builtin_amdgcn_bitop3_b32(static_cast<uint32_t>(d1), mb.z, ma.z, 0x40),
                __builtin_amdgcn_bitop3_b32(static_cast<uint32_t>(d1 >> 32), mb.w, ma.w, 0x40));
#else
            const uint32_t kc = kNC == 1 ? 0u : k;
            uint64_t m0, m1;
            fcrc::keep_mask(ka, kb > ka ? kb : ka, m0, m1);
            const uint64_t e0 = d0 & m0, e1 = d1 & m1;
            sb[kc] = fcrc::chunk_step(Lb, FK, sb[kc], static_cast<uint32_t>(e0),
                                     static_cast<uint32_t>(e0 >> 32), static_cast<uint32_t>(e1),
                                     static_cast<uint32_t>(e1 >> 32));
#endif
          }
          const bool endsB = pb && L - W0 <= G::kWin;
          const uint32_t VB = row_value(sb) ^ cu.ez[2];
          if (endsB && t == 0)
            a.crc_ok[static_cast<uint64_t>(C.item) + C.jc + 1] = VB == cu.ez[3] ? 1 : 0;
          if (pb && !endsB) {
#pragma unroll
            for (uint32_t k = 0; k < kNC; ++k) ns[k] = sb[k];
            if (t == 15) ns[kNC - 1] ^= cu.ez[2];
          }
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < kNC; ++k) crc_s[k] = ns[k];
    }
    sum0 += row_ror64<4>(sum0);
    sum1 += row_ror64<4>(sum1);
    sum0 += row_ror64<8>(sum0);
    sum1 += row_ror64<8>(sum1);
    acc0 += sum0;
    acc1 += sum1;
    if (G::kXB * C.g < nbC) {  // a full XXH3-block: scrambled (xxhash.h:5129-5133)
      acc0 = scramble(acc0, kq[16 - s4]);  // keys[16 + 2p] (kq = keys + s4 + 2p)
      acc1 = scramble(acc1, kq[17 - s4]);
    }
    if (G::kXB == 2) {  // the window's second XXH3-block
      sumB0 += row_ror64<4>(sumB0);
      sumB1 += row_ror64<4>(sumB1);
      sumB0 += row_ror64<8>(sumB0);
      sumB1 += row_ror64<8>(sumB1);
      acc0 += sumB0;
      acc1 += sumB1;
      if (G::kXB * C.g + 1 < nbC) {
        acc0 = scramble(acc0, kq[16 - s4]);
        acc1 = scramble(acc1, kq[17 - s4]);
      }
    }
    // the record's last XXH3-block (nbC) is in this window: finish it
    const bool full = (nbC >> (G::kShift - 10)) > C.g;
    const bool fin = C.rel != kNoMsg && !(lng && full);
    if (__ballot(fin)) {
      uint64_t h;
      {
        uint64_t d0, d1;
        const uint64_t le = C.off() + C.size + static_cast<uint64_t>(C.hs()) * (C.info >> 8);
        xx_words(cu.aux, static_cast<uint32_t>(le & 3), d0, d1);
        const uint64_t* cf = cold + kColdN * (FR(lane) & 3u);
        const uint64_t a0 = acc0 + mul32to64(d0 ^ cf[kColdL0]) + d1;
        const uint64_t a1 = acc1 + d0 + mul32to64(d1 ^ cf[kColdL1]);
        uint64_t tm = mul128_fold64(a0 ^ cf[kColdM0], a1 ^ cf[kColdM1]);
        tm += quad_xor64<1>(tm);
        tm += quad_xor64<2>(tm);
        h = xxh3_avalanche(static_cast<uint64_t>(C.size) * P64_1 + tm);
      }
      if ((!CRC || !FORST_REC_SHORT) && __ballot(fin && valid && !lng)) {  // short records: the row's chunks
        uint64_t d0, d1;
        xx_words(cu.x[2], (fm >> 4) & 3u, d0, d1);
        const uint64_t P0 = C.off();
        const uint32_t pb = static_cast<uint32_t>(P0 - short_phys(P0, C.size, 0));
        const uint64_t hs2 = xxh3_short_row(d0, d1, C.size, FR(lane) & 15u, pb, shsec);
        if (fin && valid && !lng) h = hs2;
      }
      // (the quad that loaded the last stripe: fm bit 18)
      if (fin && (FR(lane) & 15u) == 4 * ((fm >> G::kQuad) & 1u) && a.out64)
        a.out64[C.rel] = valid ? h : 0ull;

    }
#ifndef FORST_HOST_EMULATION
    // the last-stripe and boundary words are read only on some paths; a use
    // on every path retires their loads here (a precise wait: the next step's
    // loads are younger), so the registers can be reused in the next step
    // without a full vmcnt(0) wait on the step in flight
    asm volatile("" ::"v"(cu.aux[0]), "v"(cu.aux[1]), "v"(cu.aux[2]), "v"(cu.aux[3]),
                 "v"(cu.aux[4]));
    if (CRC) asm volatile("" ::"v"(cu.ez[0]), "v"(cu.ez[1]), "v"(cu.ez[2]), "v"(cu.ez[3]));
#endif
    C = Q[0];
#pragma unroll
    for (int d = 1; d < DEPTH; ++d) Q[d - 1] = Q[d];
    advance(DEPTH > 1 ? Q[DEPTH > 1 ? DEPTH - 2 : 0] : C, Q[DEPTH - 1]);
    return live;
  };
  // step k computes on B[k mod (DEPTH + 1)] and loads into B[(k + DEPTH) mod
  // (DEPTH + 1)]; one bottom exit (see the loop-shape note)
  if constexpr (DEPTH == 1) {
    for (bool more = true; more;) {
      step(B[0], B[1]);
      more = step(B[1], B[0]);
    }
  } else if constexpr (DEPTH == 2) {
    for (bool more = true; more;) {
      step(B[0], B[2]);
      step(B[1], B[0]);
      more = step(B[2], B[1]);
    }
  } else {
    for (bool more = true; more;) {
      step(B[0], B[3]);
      step(B[1], B[0]);
      step(B[2], B[1]);
      more = step(B[3], B[2]);
    }
  }
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) xxh3_block_kernel_simple(BlockArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const LaneKeys K = lane_keys(lane);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kWaves + wave; i < a.n;
       i += nw) {
    const uint64_t off = a.offsets[i];
    const uint32_t size = a.sizes[i];
    const uint8_t* p = a.base + off;
    uint64_t need = size;
    if (MODE == kModeVerify || MODE == kModeTrailer) need += 5;
    if (MODE == kModeCompute && a.last_bytes == nullptr) need += 1;
    const bool inb = off <= a.base_len && need <= a.base_len - off;
    if (!inb) {
      if (lane == 0) {
        if (a.out32) a.out32[i] = 0;
        if (MODE == kModeRaw && a.out64) a.out64[i] = 0;
        if (MODE == kModeVerify) {
          if (a.ok_out) a.ok_out[i] = 0;
          if (a.stored_out) a.stored_out[i] = 0;
          if (a.mismatches) atomicAdd(a.mismatches, 1ull);
        }
      }
      continue;
    }
    const uint64_t h = wave_xxh3_64(p, size, lane, K);
    if (MODE == kModeRaw) {
      if (lane == 0) a.out64[i] = h;
    } else if (MODE == kModeVerify) {
      // ComputeBuiltinChecksum(kXXH3, data, size+1), format.cc:577-586
      const uint32_t computed = modify_for_last_byte(static_cast<uint32_t>(h), ldu8(p + size));
      const uint32_t mod = a.modifiers ? a.modifiers[i] : 0u;
      const uint32_t stored = ldu32(p + size + 1) - mod;
      const bool ok = stored == computed;
      if (lane == 0) {
        if (a.out32) a.out32[i] = computed;
        if (a.stored_out) a.stored_out[i] = stored;
        if (a.ok_out) a.ok_out[i] = ok ? 1 : 0;
        if (!ok && a.mismatches) atomicAdd(a.mismatches, 1ull);
      }
    } else {
      const uint32_t last = a.last_bytes ? a.last_bytes[i] : ldu8(p + size);
      const uint32_t mod = a.modifiers ? a.modifiers[i] : 0u;
      const uint32_t c = modify_for_last_byte(static_cast<uint32_t>(h), last) + mod;
      if (lane == 0) {
        if (a.out32) a.out32[i] = c;
        if (MODE == kModeTrailer) {
          uint8_t* w = a.base_w + off + size;
          w[0] = static_cast<uint8_t>(last);
          stu32_bytes(w + 1, c);
        }
      }
    }
  }
}

// kNoChecksum: computed value is always 0 (format.cc:588-590); the stored
// trailer then only carries the context modifier.
template <int MODE>
__global__ void __launch_bounds__(kThreads) noop_block_kernel(BlockArgs a) {
  const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  for (uint64_t i = i0; i < a.n; i += static_cast<uint64_t>(gridDim.x) * kThreads) {
    const uint64_t off = a.offsets[i];
    const uint32_t size = a.sizes[i];
    uint64_t need = size;
    if (MODE == kModeVerify || MODE == kModeTrailer) need += 5;
    if (MODE == kModeCompute && a.last_bytes == nullptr) need += 1;
    const bool inb = off <= a.base_len && need <= a.base_len - off;
    const uint32_t mod = a.modifiers ? a.modifiers[i] : 0u;
    if (MODE == kModeVerify) {
      const uint32_t stored = inb ? ldu32(a.base + off + size + 1) - mod : 1u;
      const bool ok = inb && stored == 0;
      if (a.out32) a.out32[i] = 0;
      if (a.stored_out) a.stored_out[i] = inb ? stored : 0;
      if (a.ok_out) a.ok_out[i] = ok;
      if (!ok && a.mismatches) atomicAdd(a.mismatches, 1ull);
    } else {
      if (a.out32) a.out32[i] = inb ? mod : 0;
      if (MODE == kModeTrailer && inb) {
        uint8_t* w = a.base_w + off + size;
        w[0] = a.last_bytes ? a.last_bytes[i] : w[0];
        stu32_bytes(w + 1, mod);
      }
    }
  }
}

// resident workgroups per CU of the stream kernel: its grid is exactly what
// fits at once, so every wave's contiguous share runs concurrently (no tail
// of late workgroups)
template <int MODE>
uint32_t stream_occupancy() {
  static const uint32_t occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, xxh3_stream_kernel<MODE>, kThreads,
                                                     0) != hipSuccess ||
        o < 1)
      o = 1;
    return static_cast<uint32_t>(o);
  }();
  return occ;
}

template <int MODE>
uint32_t rows_occupancy() {
  static const uint32_t occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, xxh3_rows_kernel<MODE>, kRowsThreads, 0) !=
            hipSuccess ||
        o < 1)
      o = 1;
    return static_cast<uint32_t>(o);
  }();
  return occ;
}

}  // namespace

namespace {

enum class XxKernel {
  kSimple,  // one wave per block: buffers shorter than 4 KiB
  kRows,    // one message per 16-lane row (xxh3_rows_kernel)
  kV1,      // one message per wave (xxh3_stream_kernel)
#ifdef FORST_DIAG
  kProbeLoad,
#endif
};

hipError_t launch_kernel(void (*k)(BlockArgs), uint32_t grid, BlockArgs a, hipStream_t s,
                         uint32_t threads = kThreads) {
  hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 0, s, a);
  return hipGetLastError();
}

template <int M>
hipError_t launch_xxh3_mode(XxKernel k, const BlockArgs& a, hipStream_t s, const char** name) {
  static const char* const kNames[][4] = {
      {"xxh3_block_kernel_simple<compute>", "xxh3_block_kernel_simple<trailer>",
       "xxh3_block_kernel_simple<verify>", "xxh3_block_kernel_simple<raw>"},
      {"xxh3_rows_kernel<compute>", "xxh3_rows_kernel<trailer>", "xxh3_rows_kernel<verify>",
       "xxh3_rows_kernel<raw>"},
      {"xxh3_stream_kernel<compute>", "xxh3_stream_kernel<trailer>", "xxh3_stream_kernel<verify>",
       "xxh3_stream_kernel<raw>"},
  };
  const DeviceInfo& di = device_info();
  const uint64_t want = (a.n + kWaves - 1) / kWaves;
  switch (k) {
    case XxKernel::kSimple: {
      *name = kNames[0][M];
      const uint32_t grid = static_cast<uint32_t>(
          std::max<uint64_t>(1, std::min<uint64_t>(want, uint64_t(di.num_cus) * 8)));
      return launch_kernel(xxh3_block_kernel_simple<M>, grid, a, s);
    }
    case XxKernel::kRows: {
      *name = kNames[1][M];
      const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
          1, std::min<uint64_t>((a.n + 4 * kRowsWaves - 1) / (4 * kRowsWaves),
                                uint64_t(di.num_cus) * rows_occupancy<M>())));
      // block modes: the workgroup feed (stream_common.h), no ticket counter
      if (M != kModeRaw) {
        BlockArgs b = a;
        b.wg_cost = FORST_XX_BLOCK_COST;
        return launch_kernel(xxh3_rows_kernel<M>, grid, b, s, kRowsThreads);
      }
      BlockArgs b = a;
      hipError_t e = feed_setup(b, uint64_t(grid) * kRowsWaves, s);
      if (e != hipSuccess) return e;
      e = launch_kernel(xxh3_rows_kernel<M>, grid, b, s, kRowsThreads);
      const hipError_t f = scratch_free(b.ticket, s);
      return e != hipSuccess ? e : f;
    }
    case XxKernel::kV1: {
      *name = kNames[2][M];
      const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
          1, std::min<uint64_t>(want, uint64_t(di.num_cus) * stream_occupancy<M>())));
      return launch_kernel(xxh3_stream_kernel<M>, grid, a, s);
    }
#ifdef FORST_DIAG
    case XxKernel::kProbeLoad: {
      *name = "xxh3_stream_probe_kernel";
      const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
          1, std::min<uint64_t>(want, uint64_t(di.num_cus) * stream_occupancy<M>())));
      return launch_kernel(xxh3_stream_probe_kernel, grid, a, s);
    }
#endif
  }
  return hipErrorInvalidValue;
}

}  // namespace

template <int WPE, bool CRC, int DEPTH = 1>
uint32_t frag_occupancy() {
  static const uint32_t occ = [] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, xxh3_frag_kernel<WPE, CRC, DEPTH>,
                                                     CRC ? kFragCrcThreads : kFragThreads,
                                                     0) != hipSuccess ||
        o < 1)
      o = 1;
    return static_cast<uint32_t>(o);
  }();
  return occ;
}

template <int WPE, bool CRC, int DEPTH = 1>
hipError_t launch_frag(const BlockArgs& a, hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  constexpr uint32_t FW = CRC ? kFragCrcWaves : kFragWaves;
  const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
      1, std::min<uint64_t>((a.n + 4 * FW - 1) / (4 * FW),
                            uint64_t(di.num_cus) * frag_occupancy<WPE, CRC, DEPTH>())));
  BlockArgs b = a;
  hipError_t e = feed_setup(b, uint64_t(grid) * FW, stream);
  if (e != hipSuccess) return e;
  *name = CRC ? (WPE == 3 ? "xxh3_frag_kernel<3, crc>" : "xxh3_frag_kernel<2, crc>") : WPE == 4 ? "xxh3_frag_kernel<4>" : WPE == 3 ? "xxh3_frag_kernel<3>" : "xxh3_frag_kernel<2>";
  hipLaunchKernelGGL((xxh3_frag_kernel<WPE, CRC, DEPTH>), dim3(grid),
                     dim3(CRC ? kFragCrcThreads : kFragThreads), 0, stream, b);
  e = hipGetLastError();
  const hipError_t f = scratch_free(b.ticket, stream);
  return e != hipSuccess ? e : f;
}

hipError_t launch_xxh3_frag(const BlockArgs& a, hipStream_t stream, const char** name) {
  if (a.n == 0) return hipSuccess;
  if (a.n >= 0xffffffffull || a.base_len < 4096 || !a.init_crcs) return hipErrorInvalidValue;
#ifdef FORST_DIAG
  if (std::string(diag_env("FORST_FRAG_WPE")) == "2") return launch_frag<2, false>(a, stream, name);
#endif
#ifndef FORST_FRAG_WPE_DEF
#define FORST_FRAG_WPE_DEF 3
#endif
  return launch_frag<FORST_FRAG_WPE_DEF, false>(a, stream, name);
}

hipError_t launch_xxh3_frag_crc(const BlockArgs& a, hipStream_t stream, const char** name) {
  if (a.n == 0) return hipSuccess;
  if (a.n >= 0xffffffffull || a.base_len < 4096 || !a.init_crcs || !a.modifiers || !a.crc_ez ||
      !a.crc_ok)
    return hipErrorInvalidValue;
// 3 waves per SIMD (one 12-wave workgroup per CU, its 136 KiB of tables):
// 164 VGPRs, no spills (round 4); A/B against 2 waves (8-wave workgroups):
// 2 waves ran the kernel 5 % slower
#ifndef FORST_FRAG_CRC_WPE
#define FORST_FRAG_CRC_WPE (FORST_FRAG_CRC_K == 8 ? 2 : 3)
#endif
#ifndef FORST_FRAG_CRC_DEPTH
#define FORST_FRAG_CRC_DEPTH 1
#endif
  return launch_frag<FORST_FRAG_CRC_WPE, true, FORST_FRAG_CRC_DEPTH>(a, stream, name);
}

hipError_t launch_xxh3_short_rows(const uint8_t* base, uint64_t base_len, const uint64_t* off,
                                  const uint32_t* len, uint64_t n, const uint64_t* idx,
                                  uint64_t* out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (!base || !off || !len || !out) return hipErrorInvalidValue;
  const uint64_t per_wg = 4 * kShortRowsU * (kShortRowsThreads / 64);
  const uint32_t grid = static_cast<uint32_t>(
      std::min<uint64_t>((n + per_wg - 1) / per_wg, uint64_t(device_info().num_cus) * 32));
  hipLaunchKernelGGL(xxh3_short_rows_kernel, dim3(grid), dim3(kShortRowsThreads), 0, stream, base,
                     base_len, off, len, n, idx, out);
  return hipGetLastError();
}

hipError_t launch_wal_short_rows(const uint8_t* base, uint64_t base_len, const uint64_t* coff,
                                 const uint32_t* clen, const uint64_t* p0, const uint32_t* plen,
                                 const uint64_t* item, uint64_t n, const uint32_t* stored,
                                 uint8_t* crc_ok, uint64_t* hash_out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (!base || !coff || !clen || !p0 || !plen || !item || !stored || !crc_ok || !hash_out)
    return hipErrorInvalidValue;
  const uint64_t per_wg = 4 * kShortCrcU * (kShortCrcThreads / 64);
  const uint32_t grid = static_cast<uint32_t>(
      std::min<uint64_t>((n + per_wg - 1) / per_wg, uint64_t(device_info().num_cus)));
  hipLaunchKernelGGL(wal_short_rows_kernel, dim3(grid), dim3(kShortCrcThreads), 0, stream, base,
                     base_len, coff, clen, p0, plen, item, n, stored, crc_ok, hash_out);
  return hipGetLastError();
}

hipError_t launch_xxh3_blocks(int mode, const BlockArgs& a, hipStream_t stream,
                              const char** name) {
  if (a.n == 0) return hipSuccess;
  // the rows kernel for every block size (it indexes descriptors with 32
  // bits).  Round 1 sent uniform >= 48 KiB blocks to v1 (X64 rows 0.49 vs v1
  // 0.62); with the workgroup feed rows win there too (X64 0.759 vs 0.644,
  // profiles/ab_r02_late/xxh3_rows_vs_v1_wgfeed.log).  Buffers shorter than
  // 4 KiB take the simple kernel (the streaming kernels' dummy loads read
  // [0, 4 KiB)).
  XxKernel k = a.base_len < 4096           ? XxKernel::kSimple
               : a.n >= 0xffffffffull ? XxKernel::kV1
                                           : XxKernel::kRows;
  // kernel_hint 3: one message per wave (a short list of long messages, e.g.
  // wal_hash.h's gathered records: rows would leave most rows idle while a
  // few walk 32 KiB records 1 KiB per step)
  if (a.kernel_hint == 3 && a.base_len >= 4096) k = XxKernel::kV1;
#ifdef FORST_DIAG
  if (a.base_len >= 4096) {
    const std::string v = diag_env("FORST_XXH3_VARIANT");
    if (v == "simple") k = XxKernel::kSimple;
    if (v == "v1") k = XxKernel::kV1;
    if (v == "rows" && a.n < 0xffffffffull) k = XxKernel::kRows;
    if (v == "probe_load" && mode == kModeVerify) k = XxKernel::kProbeLoad;
  }
#endif
  switch (mode) {
    case kModeCompute:
      return launch_xxh3_mode<kModeCompute>(k, a, stream, name);
    case kModeTrailer:
      return launch_xxh3_mode<kModeTrailer>(k, a, stream, name);
    case kModeVerify:
      return launch_xxh3_mode<kModeVerify>(k, a, stream, name);
    default:
      return launch_xxh3_mode<kModeRaw>(k, a, stream, name);
  }
}

hipError_t launch_noop_blocks(int mode, const BlockArgs& a, hipStream_t stream,
                              const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  const uint64_t want = (a.n + kThreads - 1) / kThreads;
  const uint32_t grid = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>(want, uint64_t(di.num_cus) * 8)));
  switch (mode) {
    case kModeCompute:
      *name = "noop_block_kernel<compute>";
      hipLaunchKernelGGL(noop_block_kernel<kModeCompute>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    case kModeTrailer:
      *name = "noop_block_kernel<trailer>";
      hipLaunchKernelGGL(noop_block_kernel<kModeTrailer>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    default:
      *name = "noop_block_kernel<verify>";
      hipLaunchKernelGGL(noop_block_kernel<kModeVerify>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// synthetic stream fill (bench/test utility)
// ---------------------------------------------------------------------------
namespace {
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void __launch_bounds__(256) fill_stream_kernel(uint8_t* dst, uint64_t start,
                                                          uint64_t n, uint64_t seed) {
  // each thread produces one aligned 8-byte word of the stream
  const uint64_t w0 = start >> 3;
  const uint64_t w1 = (start + n + 7) >> 3;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t w = w0 + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
       w < w1; w += stride) {
    const uint64_t v = splitmix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
    const uint64_t b0 = w << 3;
    if (b0 >= start && b0 + 8 <= start + n && ((b0 - start) & 7) == 0) {
      *reinterpret_cast<uint64_t*>(dst + (b0 - start)) = v;
    } else {
      for (int k = 0; k < 8; ++k) {
        const uint64_t b = b0 + k;
        if (b >= start && b < start + n) dst[b - start] = static_cast<uint8_t>(v >> (8 * k));
      }
    }
  }
}
}  // namespace

hipError_t launch_fill_stream(uint8_t* dev, uint64_t start, uint64_t n, uint64_t seed,
                              hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const DeviceInfo& di = device_info();
  const uint64_t words = (n + 15) / 8;
  const uint32_t grid = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>((words + 255) / 256, uint64_t(di.num_cus) * 16)));
  hipLaunchKernelGGL(fill_stream_kernel, dim3(grid), dim3(256), 0, stream, dev, start, n, seed);
  return hipGetLastError();
}

}  // namespace forst
