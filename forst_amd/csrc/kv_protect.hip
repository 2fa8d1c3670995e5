// forst_amd/csrc/kv_protect.hip -- per-KV protection info (db/kv_checksum.h)
// and Hash64 / NPHash64 (util/hash.cc:81-88 -> XXPH3_64bits_withSeed,
// util/xxph3.h:1733) as batched gfx950 kernels.
//
// XXPH3 is the xxHash 0.7.2 PREVIEW that RocksDB standardised on for Hash64;
// it is not the kXXH3 block checksum (0.8.1): different short-input formulas
// (xxph3.h:1082-1140, including RocksDB's non-zero empty hash), no lane swap in
// the accumulate (acc_64bits, xxph3.h:1333-1338), nb_blocks = len / 1024, the
// last stripe only when len % 64 != 0 (xxph3.h:1527-1543), avalanche with
// PRIME64_3 (xxph3.h:1069) and, for a seed, a custom secret (kSecret +/- seed
// on alternating 8-byte words, xxph3.h:1609-1620).
//
// ProtectionInfo<T> (kv_checksum.h:296-460) XORs NPHash64 of every field with
// its own seed (:84-88); op type (1 byte), sequence number (8) and column
// family id (4) are hashed as their native little-endian bytes (:27-29).
//
// Layout (round 6): ONE 16-LANE ROW PER ENTRY.  A wave takes a tile of 64
// entries: lane i loads entry i's descriptors (coalesced) and hashes its
// op/seq/cf fields; then 16 rounds, in round r row R hashes the key and value
// of entry 16R + r.  Every byte an entry's hashes read is loaded by the lanes
// of that row at once -- adjacent 16-byte pieces of one key / value, so a
// row's loads hit the same few cache lines -- and every formula is split over
// the row's lanes:
//   * 17..240 bytes: the XXPH3 sum of mix16B terms (xxph3.h:1651-1707) is a
//     sum of independent terms: lane t computes term t, two segmented row sums
//     (lanes 0-7, 8-15) give both accumulation phases;
//   * > 240 bytes: lane t takes the 16-byte chunks 16t + 256k of each 1 KiB
//     block (stripe t/4 + 4k, accumulator pair t%4), the first block and the
//     last stripe loaded together with the short terms;
//   * <= 16 bytes: one lane (7: key, 6: value).
// Row r's hash lands in an LDS slot of its owner lane; the owner XORs it with
// the op/seq/cf hashes and writes / verifies.  (Round 5 hashed short fields
// one LANE per entry with scattered 8-byte loads -- 64 entries, 64 cache
// lines per load -- and long values in a second pass that fetched the same
// lines again: 0.18 of peak, 1.4x traffic.)
#include <cstdlib>
#include <type_traits>

#include "device_common.h"
#include "engine.h"
#include "stream_common.h"
#include "xxh_common.h"

namespace forst {
namespace {

constexpr uint32_t kWaves = 4;
constexpr uint32_t kThreads = kWaves * 64;
constexpr uint32_t kSecWords = 26;  // kSecret as 24 LE u64 words + 2 zero words

// db/kv_checksum.h:84-88
constexpr uint64_t kSeedK = 0;
constexpr uint64_t kSeedV = 0xD28AAD72F49BD50Bull;
constexpr uint64_t kSeedO = 0xA5155AE5E937AA16ull;
constexpr uint64_t kSeedS = 0x77A00858DDD37F21ull;
constexpr uint64_t kSeedC = 0x4A2AB5CBD26F542Cull;

// xxph3.h:1069
__device__ __forceinline__ uint64_t xxph3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}

// 8 bytes at byte offset `off` of the secret for `seed` (xxph3.h:1609-1620:
// word 2i gets +seed, word 2i+1 gets -seed; seed 0 = the default secret),
// from the LDS copy of kSecret's words
__device__ __forceinline__ uint64_t psec(const uint64_t* S, uint32_t off, uint64_t seed) {
  const uint32_t w = off >> 3, sh = off & 7;
  const uint64_t x = S[w] + ((w & 1) ? (0 - seed) : seed);
  if (sh == 0) return x;
  const uint64_t y = S[w + 1] + ((w & 1) ? seed : (0 - seed));
  return (x >> (8 * sh)) | (y << (64 - 8 * sh));
}

// xxph3.h:1098 XXPH3_len_4to8_64b on the input already folded to 64 bits
__device__ __forceinline__ uint64_t xxph3_4to8(uint64_t in64, uint32_t len, uint64_t seed) {
  const uint64_t keyed = in64 ^ (sec64(0) + seed);
  const uint64_t mix64 = len + ((keyed ^ (keyed >> 51)) * P32_1);
  return xxph3_avalanche((mix64 ^ (mix64 >> 47)) * P64_2);
}
// xxph3.h:1082 XXPH3_len_1to3_64b
__device__ __forceinline__ uint64_t xxph3_1to3(uint32_t c1, uint32_t c2, uint32_t c3, uint32_t len,
                                               uint64_t seed) {
  const uint32_t combined = c1 | (c2 << 8) | (c3 << 16) | (len << 24);
  const uint64_t keyed = static_cast<uint64_t>(combined) ^
                         (static_cast<uint64_t>(static_cast<uint32_t>(sec64(0))) + seed);
  return xxph3_avalanche(keyed * P64_1);
}

// Where a round's field bytes come from: global memory (GSrc) or the wave's
// LDS stage (LSrc, the sub-tile's byte span loaded coalesced); offsets are
// bytes from the field start.
struct GSrc {
  const uint8_t* p;
  __device__ __forceinline__ void ld16(uint32_t o, uint64_t& d0, uint64_t& d1) const {
    const uint8_t* e = p + o;
    const uint32_t m = static_cast<uint32_t>(reinterpret_cast<uint64_t>(e) & 3);
    ld16u(e - m, m, d0, d1);
  }
  __device__ __forceinline__ uint64_t u64(uint32_t o) const { return ldu64(p + o); }
  __device__ __forceinline__ uint32_t u32(uint32_t o) const { return ldu32(p + o); }
  __device__ __forceinline__ uint32_t u8(uint32_t o) const { return ldu8(p + o); }
};
struct LSrc {
  const uint32_t* L;  // the wave's stage (dwords)
  uint32_t x;         // the field's byte offset in it
  __device__ __forceinline__ uint32_t u32(uint32_t o) const {
    const uint32_t b = x + o;
    return __builtin_amdgcn_alignbyte(L[(b >> 2) + 1], L[b >> 2], b & 3);
  }
  __device__ __forceinline__ void ld16(uint32_t o, uint64_t& d0, uint64_t& d1) const {
    const uint32_t b = x + o, w = b >> 2, sh = b & 3;
    const uint32_t v0 = L[w], v1 = L[w + 1], v2 = L[w + 2], v3 = L[w + 3], v4 = L[w + 4];
    d0 = mk64(__builtin_amdgcn_alignbyte(v1, v0, sh), __builtin_amdgcn_alignbyte(v2, v1, sh));
    d1 = mk64(__builtin_amdgcn_alignbyte(v3, v2, sh), __builtin_amdgcn_alignbyte(v4, v3, sh));
  }
  __device__ __forceinline__ uint64_t u64(uint32_t o) const { return mk64(u32(o), u32(o + 4)); }
  __device__ __forceinline__ uint32_t u8(uint32_t o) const {
    const uint32_t b = x + o;
    return (L[b >> 2] >> (8 * (b & 3))) & 0xffu;
  }
};

// The bytes a 0..16-byte field's formula reads (xxph3.h:1082-1140), loaded
// exactly: 9..16 -> d0 = first 8, d1 = last 8; 4..8 -> d0 = first 4 | last 4
// << 32; 1..3 -> d0 = in[0] | in[len/2] << 8 | in[len-1] << 16.
template <class Src>
__device__ __forceinline__ void tiny_load(const Src& in, uint32_t len, uint64_t& d0, uint64_t& d1) {
  if (len > 8) {
    d0 = in.u64(0);
    d1 = in.u64(len - 8);
  } else if (len >= 4) {
    d0 = in.u32(0) | (static_cast<uint64_t>(in.u32(len - 4)) << 32);
  } else if (len) {
    d0 = in.u8(0) | (in.u8(len >> 1) << 8) | (in.u8(len - 1) << 16);
  }
}
__device__ __forceinline__ uint64_t tiny_hash(uint64_t d0, uint64_t d1, uint32_t len, uint64_t seed) {
  if (len > 8) {
    const uint64_t lo = d0 ^ (sec64(0) + seed);
    const uint64_t hi = d1 ^ (sec64(8) - seed);
    return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
  }
  if (len >= 4) return xxph3_4to8(d0, len, seed);
  if (len) {
    const uint32_t w = static_cast<uint32_t>(d0);
    return xxph3_1to3(w & 0xff, (w >> 8) & 0xff, (w >> 16) & 0xff, len, seed);
  }
  return mul128_fold64(seed + sec64(0), P64_2);  // xxph3.h:1133-1138 (RocksDB)
}

// Which 16 bytes of a 17..240-byte field lane t mixes (xxph3.h:1651-1707):
//   17..128:  term t < nt (nt = 2/4/6/8 for len > 0/32/64/96): even t at
//             in + 8t, odd t at in + len - 8(t+1); secret 16t
//   129..240: t < 8 at in + 16t, secret 16t; 8 <= t < len/16 (t < 15) at
//             in + 16t, secret 16(t-8) + 3; t = 15 at in + len - 16, secret 119
// Returns false for a lane without a term.
__device__ __forceinline__ bool term_at(uint32_t t, uint32_t len, uint32_t& d) {
  if (len <= 128) {
    const uint32_t nt = len > 96 ? 8 : len > 64 ? 6 : len > 32 ? 4 : 2;
    d = (t & 1) ? len - 8 * (t + 1) : 8 * t;
    return t < nt;
  }
  d = t == 15 ? len - 16 : 16 * t;
  return t < 8 || t == 15 || t < (len >> 4);
}
__device__ __forceinline__ uint32_t term_secret(uint32_t t) {
  return t < 8 ? 16 * t : t < 15 ? 16 * (t - 8) + 3 : 119;
}

// DPP row_shr:n with bound_ctrl (lanes without a source get 0)
template <int N>
__device__ __forceinline__ uint64_t row_shr64(uint64_t v) {
  return dpp64<0x110 + N>(v);
}

// lane 7 of each row: the XXPH3 hash of a 17..240-byte field from the row's
// mix16B terms (0 in lanes without one): the segmented sums over lanes 0-7
// and 8-15 are the two accumulation phases
__device__ __forceinline__ uint64_t short_finish(uint64_t term, uint32_t len) {
  term += row_shr64<1>(term);
  term += row_shr64<2>(term);
  term += row_shr64<4>(term);  // lane 7: sum of 0..7, lane 15: sum of 8..15
  const uint64_t s2 = row_ror64<8>(term);
  uint64_t x = static_cast<uint64_t>(len) * P64_1 + term;
  if (len > 128) x = xxph3_avalanche(x) + s2;
  return xxph3_avalanche(x);
}

__device__ __forceinline__ uint64_t scramble_acc(uint64_t a, uint64_t key) {
  a ^= a >> 47;
  a ^= key;
  return a * P32_1;
}

// The chunks lane t mixes in 1 KiB block g of a > 240-byte field: bytes
// 1024g + 16t + 256k (stripe t/4 + 4k, accumulator pair t%4), k = 0..3;
// bit k of the mask = the chunk exists (whole blocks, then the nbS stripes of
// the last partial block).
struct Block {
  uint64_t d0[4], d1[4];
  uint32_t mask;
};
template <class Src>
__device__ __forceinline__ void long_block_load(const Src& p, uint32_t len, uint32_t g,
                                                uint32_t t, bool act, Block& b) {
  const uint32_t nb = len >> 10, nbS = (len & 1023) >> 6;
  b.mask = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t st = (t >> 2) + 4 * k;
    b.d0[k] = b.d1[k] = 0;
    if (act && (g < nb || (g == nb && st < nbS))) {
      p.ld16(1024 * g + 16 * t + 256 * k, b.d0[k], b.d1[k]);
      b.mask |= 1u << k;
    }
  }
}
// the last stripe (len - 64 + 16 (t%4), xxph3.h:1539-1542), when len % 64
template <class Src>
__device__ __forceinline__ void long_last_load(const Src& p, uint32_t len, uint32_t t, bool act,
                                               uint64_t& l0, uint64_t& l1) {
  l0 = l1 = 0;
  if (act && (len & 63)) p.ld16(len - 64 + 16 * (t & 3), l0, l1);
}

// Row-wide XXPH3 of a > 240-byte field (xxph3.h:1514-1583, 1630-1637) whose
// first block `b` and last stripe (l0, l1) are already loaded; every lane of
// a row with act gets the hash.  Rows may differ in length: the block loop
// runs to the wave's largest, uniform around the DPP row sums.
// The 14 secret words lane t of a row uses for a > 240-byte field: the chunk
// pairs of stripes t/4 + 4k (j = 2k, 2k + 1), the scramble pair (8, 9), the
// last-stripe pair (10, 11) and the merge pair (12, 13).
constexpr uint32_t kLongSec = 14;
__device__ __forceinline__ uint32_t long_sec_off(uint32_t t, uint32_t j) {
  const uint32_t pp = t & 3;
  if (j < 8) return 8 * ((t >> 2) + 4 * (j >> 1)) + 16 * pp + 8 * (j & 1);
  constexpr uint32_t kBase[6] = {128, 136, 121, 129, 11, 19};
  return kBase[j - 8] + 16 * pp;
}

// TAB: T = lane t's kLongSec words for `seed`, precomputed in LDS (the value
// seed: every round's long value), else derived from S here (keys)
template <bool TAB, class Src>
__device__ uint64_t row_long(const uint64_t* S, const uint64_t* T, const Src& p, uint32_t len,
                             uint64_t seed, bool act, uint32_t t, Block& b, uint64_t l0,
                             uint64_t l1) {
  const uint32_t pp = t & 3;
  uint64_t acc0 = pp == 0 ? P32_3 : pp == 1 ? P64_2 : pp == 2 ? P64_4 : P64_5;  // INIT_ACC
  uint64_t acc1 = pp == 0 ? P64_1 : pp == 1 ? P64_3 : pp == 2 ? P32_2 : P32_1;
  const uint32_t nb = act ? len >> 10 : 0;
  auto sec = [&](uint32_t j) { return TAB ? T[j] : psec(S, long_sec_off(t, j), seed); };
  // the chunk secrets: stripe st's at 8 st + 16 pp (aligned words)
  uint64_t k0[4], k1[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    k0[k] = sec(2 * k);
    k1[k] = sec(2 * k + 1);
  }
  const uint64_t ks0 = sec(8), ks1 = sec(9);
  for (uint32_t g = 0;; ++g) {
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
      if (b.mask & (1u << k)) {  // acc_64bits: acc[i] += data + lo*hi(data ^ key)
        c0 += b.d0[k] + mul32to64(b.d0[k] ^ k0[k]);
        c1 += b.d1[k] + mul32to64(b.d1[k] ^ k1[k]);
      }
    c0 += row_ror64<4>(c0);
    c1 += row_ror64<4>(c1);
    c0 += row_ror64<8>(c0);
    c1 += row_ror64<8>(c1);
    acc0 += c0;
    acc1 += c1;
    if (g < nb) {
      acc0 = scramble_acc(acc0, ks0);
      acc1 = scramble_acc(acc1, ks1);
    }
    if (!__ballot(g < nb)) break;
    long_block_load(p, len, g + 1, t, act && g < nb, b);
  }
  if (len & 63) {
    acc0 += l0 + mul32to64(l0 ^ sec(10));
    acc1 += l1 + mul32to64(l1 ^ sec(11));
  }
  // XXPH3_mergeAccs from secret + 11 (xxph3.h:1554-1582)
  uint64_t h = mul128_fold64(acc0 ^ sec(12), acc1 ^ sec(13));
  h += quad_xor64<1>(h);
  h += quad_xor64<2>(h);
  return xxph3_avalanche(static_cast<uint64_t>(len) * P64_1 + h);
}

__device__ __forceinline__ bool in_range(uint64_t off, uint64_t len, uint64_t base_len) {
  return off <= base_len && len <= base_len - off;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  return mk64(__shfl(static_cast<uint32_t>(v), src), __shfl(static_cast<uint32_t>(v >> 32), src));
}

// 16 bytes at byte position pos as 4 LE dwords; bytes at or past base_len
// read as 0 and *avail = how many of the 16 lie inside the buffer
struct W16 {
  uint32_t w[4];
};
__device__ __forceinline__ W16 load16_bounded(const uint8_t* base, uint64_t base_len, uint64_t pos,
                                              uint32_t& avail) {
  W16 r;
  avail = pos >= base_len ? 0u : base_len - pos >= 16 ? 16u : static_cast<uint32_t>(base_len - pos);
  const uint64_t q = pos & ~3ull;
  if (q + 20 <= base_len) {
    const uint32_t m = static_cast<uint32_t>(pos & 3);
    const u32x4a4 v = ld16_a4(base + q + vzero());
    const uint32_t x4 = m ? ld4_a4(base + q + 16 + vzero()) : 0u;
    r.w[0] = __builtin_amdgcn_alignbyte(v.y, v.x, m);
    r.w[1] = __builtin_amdgcn_alignbyte(v.z, v.y, m);
    r.w[2] = __builtin_amdgcn_alignbyte(v.w, v.z, m);
    r.w[3] = __builtin_amdgcn_alignbyte(x4, v.w, m);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) r.w[k] = 0;
    for (uint32_t k = 0; k < avail; ++k) r.w[k >> 2] |= ldu8(base + pos + k) << (8 * (k & 3));
  }
  return r;
}
__device__ __forceinline__ uint32_t byte_of(const W16& v, uint32_t k) {
  return (v.w[k >> 2] >> (8 * (k & 3))) & 0xffu;
}
// GetVarint32Ptr(p, p + 5, &val) (util/coding.h:109, coding.cc
// GetVarint32PtrFallback) on window byte k0: the bytes consumed, 0 when five
// bytes all carry the continuation bit, kVarOut when the varint runs past the
// buffer (the reference reads on; the engine reports it)
constexpr uint32_t kVarOut = 0xff;
__device__ __forceinline__ uint32_t varint32_at(const W16& v, uint32_t k0, uint32_t avail,
                                                uint32_t& val) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t j = 0; j < 5; ++j) {
    if (k0 + j >= avail) return kVarOut;
    const uint32_t b = byte_of(v, k0 + j);
    r |= (b & 127u) << (7 * j);  // (shift 28: the bits past 32 drop, as in the reference)
    if (!(b & 128u)) {
      val = r;
      return j + 1;
    }
  }
  return 0;
}

// MemTable entry (memtable.cc:696-732 layout, :273-307 decode):
//   varint32 internal_key_len | user_key | tag = seq << 8 | type (LE64) |
//   varint32 value_len | value | protection_bytes checksum
// -> key / value / checksum positions, type and seq; returns a KvMemStatus.
__device__ __forceinline__ uint32_t decode_mem_entry(const KvArgs& a, uint64_t pos, uint64_t& ko,
                                                     uint32_t& kl, uint64_t& vo, uint32_t& vl,
                                                     uint64_t& co, uint64_t& tag) {
  uint32_t av;
  const W16 e = load16_bounded(a.base, a.base_len, pos, av);
  uint32_t ikl = 0;
  const uint32_t n1 = varint32_at(e, 0, av, ikl);
  if (n1 == kVarOut) return kMemOutOfRange;
  if (n1 == 0) return kMemBadKeyLength;
  if (ikl < 8) return kMemKeyTooShort;
  ko = pos + n1;
  kl = ikl - 8;
  const uint64_t tp = ko + kl;
  uint32_t av2;
  const W16 t = load16_bounded(a.base, a.base_len, tp, av2);
  if (av2 < 8) return kMemOutOfRange;
  tag = mk64(t.w[0], t.w[1]);
  const uint32_t n2 = varint32_at(t, 8, av2, vl);
  if (n2 == kVarOut) return kMemOutOfRange;
  if (n2 == 0) return kMemBadValue;
  vo = tp + 8 + n2;
  co = vo + vl;
  return in_range(co, a.prot_bytes, a.base_len) ? kMemOk : kMemOutOfRange;
}

// sub-tiles (kv_kernel): kSub entries, their bytes staged in LDS when they
// span at most kStage bytes (4 workgroups of 4 waves per CU fit the LDS)
#ifndef FORST_KV_STAGE
#define FORST_KV_STAGE 1
#endif
#ifndef FORST_KV_WAVES_PER_EU
#define FORST_KV_WAVES_PER_EU 4
#endif
constexpr uint32_t kSub = 8;
constexpr uint64_t kSubMask = (1ull << kSub) - 1;
#ifndef FORST_KV_STAGE_BYTES
#define FORST_KV_STAGE_BYTES 8704
#endif
constexpr uint32_t kStage = FORST_KV_STAGE_BYTES;
constexpr uint32_t kStageChunks = (kStage + 1023) / 1024;

// field classes
constexpr uint32_t kTiny = 0, kShort = 1, kLong = 2, kNone = 3;
__device__ __forceinline__ uint32_t field_class(bool valid, uint32_t len) {
  return !valid ? kNone : len <= 16 ? kTiny : len <= 240 ? kShort : kLong;
}

// MODE: kKvHash (Hash64 per buffer), kKvProtect, kKvVerify
template <int MODE>
__global__ void __launch_bounds__(kThreads) FORST_WAVES_PER_EU(FORST_KV_WAVES_PER_EU) kv_kernel(KvArgs a) {
  __shared__ uint64_t s_sec[kSecWords];
  __shared__ uint64_t s_slot[kWaves][64];
  __shared__ uint64_t s_vsec[16 * kLongSec];  // the value seed's long-field secrets per t
  __shared__ u32x4 s_stage[kWaves][(kStage + 32) / 16];  // per wave: a sub-tile's bytes
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t t = lane & 15;
  if (threadIdx.x < kSecWords) s_sec[threadIdx.x] = threadIdx.x < 24 ? sec64(8 * threadIdx.x) : 0;
  __syncthreads();
  const uint64_t* S = s_sec;
  static_assert(16 * kLongSec <= kThreads, "one table word per thread");
  if (threadIdx.x < 16 * kLongSec)
    s_vsec[threadIdx.x] = psec(S, long_sec_off(threadIdx.x / kLongSec, threadIdx.x % kLongSec), kSeedV);
  __syncthreads();
  const uint64_t* VT = s_vsec + t * kLongSec;
  // this lane's mix16B secret pair (seed applied per field)
  const uint64_t SA = psec(S, term_secret(t), 0), SB = psec(S, term_secret(t) + 8, 0);
  uint64_t* slot = s_slot[wave];
  const uint32_t* stage = reinterpret_cast<const uint32_t*>(s_stage[wave]);
  uint8_t* stage_w = reinterpret_cast<uint8_t*>(s_stage[wave]);
  // staging needs 16-byte alignment of the buffer and one buffer for keys and values
  const bool stage_ok = FORST_KV_STAGE && a.key_base == nullptr &&
                        (reinterpret_cast<uint64_t>(a.base) & 15) == 0;

  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWaves * 64;
  for (uint64_t b0 = (static_cast<uint64_t>(blockIdx.x) * kWaves + wave) * 64; b0 < a.n;
       b0 += stride) {
    // ---- lane = entry: descriptors and the op / seq / cf hashes
    const uint64_t i = b0 + lane;
    const bool act = i < a.n;
    uint64_t ko = 0, vo = 0, co = 0, kseed = kSeedK, hs = 0;
    uint32_t kl = 0, vl = 0, mst = kMemOk;
    bool valid = false;
    if (MODE == kKvMemVerify || MODE == kKvMemProtect) {
      if (act) {
        uint64_t tag = 0;
        mst = decode_mem_entry(a, a.key_off[i], ko, kl, vo, vl, co, tag);
        valid = mst == kMemOk;
        // ProtectKVO(user_key, value, type).ProtectS(seq) (memtable.cc:298-302)
        const uint32_t op = static_cast<uint32_t>(tag & 0xff);
        hs = xxph3_1to3(op, op, op, 1, kSeedO) ^ xxph3_4to8(tag >> 8, 8, kSeedS);
      }
    } else if (act) {
      ko = a.key_off[i];
      kl = a.key_len[i];
      valid = in_range(ko, kl, a.key_base ? a.key_base_len : a.base_len);
      if (MODE == kKvHash) {
        kseed = a.seeds ? a.seeds[i] : a.seed;
      } else {
        vo = a.val_off[i];
        vl = a.val_len[i];
        valid = valid && in_range(vo, vl, a.base_len);
        if (a.ops) {  // NPHash64(&op_type, 1, kSeedO)
          const uint32_t op = a.ops[i];
          hs ^= xxph3_1to3(op, op, op, 1, kSeedO);
        }
        if (a.seqs) hs ^= xxph3_4to8(a.seqs[i], 8, kSeedS);  // native LE bytes
        if (a.cfs) {
          const uint64_t cf = a.cfs[i];
          hs ^= xxph3_4to8(cf | (cf << 32), 4, kSeedC);
        }
      }
      if (MODE == kKvVerify) {
        co = a.chk_off[i];
        valid = valid && in_range(co, a.prot_bytes, a.base_len);
      }
    }
    const uint64_t vmask = __ballot(valid);
    // the bytes this lane's fields cover (the sub-tile spans below)
    uint64_t flo = ~0ull, fhi = 0;
    if (valid) {
      flo = ko;
      fhi = ko + kl;
      if (MODE != kKvHash) {
        flo = vo < flo ? vo : flo;
        fhi = vo + vl > fhi ? vo + vl : fhi;
      }
    }

    // ---- one round: row R hashes the key and value of entry src (ST: the
    // bytes from the wave's stage, which holds [sb, ...) of the buffer)
    auto round = [&](uint32_t src, auto stc, uint64_t sb) {
      constexpr bool ST = decltype(stc)::value;
      using Src = std::conditional_t<ST, LSrc, GSrc>;
      const bool rv = (vmask >> src) & 1;
      const uint64_t rko = shfl64(ko, src);
      const uint32_t rkl = __shfl(kl, src);
      const uint64_t rks = MODE == kKvHash ? shfl64(kseed, src) : kSeedK;
      uint64_t rvo = 0;
      uint32_t rvl = 0;
      if (MODE != kKvHash) {
        rvo = shfl64(vo, src);
        rvl = __shfl(vl, src);
      }
      const uint32_t kc = field_class(rv, rkl);
      const uint32_t vc = MODE == kKvHash ? kNone : field_class(rv, rvl);
      Src kp, vp;
      if constexpr (ST) {  // (rows without a valid entry, and hash64's absent values, read at 0)
        kp = LSrc{stage, rv ? static_cast<uint32_t>(rko - sb) : 0u};
        vp = LSrc{stage, rv && MODE != kKvHash ? static_cast<uint32_t>(rvo - sb) : 0u};
      } else {  // (rows without a valid entry load nothing: no pointer from their offsets)
        kp = GSrc{(a.key_base ? a.key_base : a.base) + (rv ? rko : 0)};
        vp = GSrc{a.base + (rv ? rvo : 0)};
      }

      // -- every load of the round, issued before any of it is used
      uint64_t kd0 = 0, kd1 = 0, vd0 = 0, vd1 = 0;
      uint32_t dk = 0, dv = 0;
      const bool kterm = kc == kShort && term_at(t, rkl, dk);
      const bool vterm = vc == kShort && term_at(t, rvl, dv);
      if (kterm) {
        kp.ld16(dk, kd0, kd1);
      } else if (kc == kTiny && t == 7) {
        tiny_load(kp, rkl, kd0, kd1);
      }
      if (vterm) {
        vp.ld16(dv, vd0, vd1);
      } else if (vc == kTiny && t == 6) {
        tiny_load(vp, rvl, vd0, vd1);
      }
      Block vb;
      uint64_t vl0, vl1;
      long_block_load(vp, rvl, 0, t, vc == kLong, vb);
      long_last_load(vp, rvl, t, vc == kLong, vl0, vl1);

      // -- 17..240-byte fields: the row's terms (each class's code only when
      // one of the wave's four rows needs it)
      uint64_t h = 0;
      if (__ballot(kc == kShort)) {
        const uint64_t tk = kterm ? mul128_fold64(kd0 ^ (SA + rks), kd1 ^ (SB - rks)) : 0;
        const uint64_t fk = short_finish(tk, rkl);
        if (kc == kShort) h ^= fk;
      }
      if (MODE != kKvHash && __ballot(vc == kShort)) {
        const uint64_t tv = vterm ? mul128_fold64(vd0 ^ (SA + kSeedV), vd1 ^ (SB - kSeedV)) : 0;
        const uint64_t fv = short_finish(tv, rvl);
        if (vc == kShort) h ^= fv;
      }
      // -- 0..16-byte fields: lane 7 the key's, lane 6 the value's
      if (__ballot(kc == kTiny || vc == kTiny)) {
        const bool k7 = t == 7 && kc == kTiny, v6 = t == 6 && vc == kTiny;
        const uint64_t x = tiny_hash(k7 ? kd0 : vd0, k7 ? kd1 : vd1, k7 ? rkl : rvl,
                                     k7 ? rks : kSeedV);
        const uint64_t y = (k7 || v6) ? x : 0;
        h ^= y ^ dpp64<0x121>(y);  // row_ror:1 -> lane 7 also gets lane 6's
      }
      // -- > 240-byte fields
      if (__ballot(vc == kLong)) {
        const uint64_t hl = row_long<true>(S, VT, vp, rvl, kSeedV, vc == kLong, t, vb, vl0, vl1);
        if (vc == kLong) h ^= hl;
      }
      if (__ballot(kc == kLong)) {  // (keys over 240 bytes: rare, loaded here)
        Block kb;
        uint64_t kl0, kl1;
        long_block_load(kp, rkl, 0, t, kc == kLong, kb);
        long_last_load(kp, rkl, t, kc == kLong, kl0, kl1);
        const uint64_t hl = row_long<false>(S, nullptr, kp, rkl, rks, kc == kLong, t, kb, kl0, kl1);
        if (kc == kLong) h ^= hl;
      }
      if (t == 7) slot[src] = h;
    };

    // ---- sub-tiles of kSub entries.  A sub-tile whose keys and values lie
    // in one span of at most kStage bytes (packed entries: kv_checksum's
    // key | value | protection layout, memtable entries) is loaded into the
    // wave's stage with coalesced 16-byte loads, 1 KiB per instruction, and
    // its rounds read the stage; any other sub-tile's rounds load from global
    // memory.  Round r of sub-tile j: row R hashes entry kSub j + 4 r + R.
#pragma unroll 1
    for (uint32_t j = 0; j < 64 / kSub; ++j) {
      if (!((vmask >> (kSub * j)) & kSubMask)) continue;  // (wave-uniform)
      uint64_t lo = flo, hi = fhi;
#pragma unroll
      for (uint32_t o = 1; o < kSub; o <<= 1) {
        const uint64_t l2 = shfl_xor64(lo, o), h2 = shfl_xor64(hi, o);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
      }
      lo = uniform64(shfl64(lo, kSub * j));
      hi = uniform64(shfl64(hi, kSub * j));
      const uint64_t sb = lo & ~15ull, se = (hi + 15) & ~15ull;
      if (stage_ok && se > sb && se - sb <= kStage && se <= a.base_len) {
        const uint32_t nbytes = static_cast<uint32_t>(se - sb);
        // (chunks past the span re-read its first 16 bytes: the loads are
        // not predicated, so the compiler keeps them all in flight, and no
        // load leaves [sb, se))
        u32x4a4 v[kStageChunks];
#pragma unroll
        for (uint32_t c = 0; c < kStageChunks; ++c) {
          const uint32_t o = 1024 * c + 16 * lane;
          v[c] = ld16_a4(a.base + sb + (o < nbytes ? o : 0u) + vzero());
        }
#pragma unroll
        for (uint32_t c = 0; c < kStageChunks; ++c) {
          const uint32_t o = 1024 * c + 16 * lane;
          if (o < nbytes) *reinterpret_cast<u32x4*>(stage_w + o) = u32x4{v[c].x, v[c].y, v[c].z, v[c].w};
        }
        wave_lds_sync();
#pragma unroll 1
        for (uint32_t r = 0; r < kSub / 4; ++r)
          round(kSub * j + 4 * r + (lane >> 4), std::true_type{}, sb);
        wave_lds_sync();  // (the next sub-tile rewrites the stage)
      } else {
#pragma unroll 1
        for (uint32_t r = 0; r < kSub / 4; ++r)
          round(kSub * j + 4 * r + (lane >> 4), std::false_type{}, 0);
      }
    }
    wave_lds_sync();
    uint64_t h = valid ? hs ^ slot[lane] : 0;
    wave_lds_sync();  // (the next tile's rounds overwrite the slots)

    if (MODE == kKvMemProtect) {
      // MemTable::UpdateEntryChecksum (memtable.cc:676-693): Encode(prot_bytes)
      if (valid && a.write_in_place) {
        uint8_t* c = const_cast<uint8_t*>(a.base) + co;
        for (uint32_t b = 0; b < a.prot_bytes; ++b) c[b] = static_cast<uint8_t>(h >> (8 * b));
      }
      if (act && a.out) a.out[i] = h;
      if (act && a.status) a.status[i] = static_cast<uint8_t>(mst);
    } else if (MODE == kKvVerify || MODE == kKvMemVerify) {
      // ProtectionInfo<T>::Verify (kv_checksum.h:117-133): low prot_bytes bytes, LE
      uint64_t stored = 0;
      if (valid) {
        const uint8_t* c = a.base + co;
        if (a.prot_bytes == 8) {
          stored = ldu64(c);
        } else if (a.prot_bytes == 4) {
          stored = ldu32(c);
        } else {
          for (uint32_t b = 0; b < a.prot_bytes; ++b)
            stored |= static_cast<uint64_t>(ldu8(c + b)) << (8 * b);
        }
      }
      const uint64_t mask = a.prot_bytes >= 8 ? ~0ull : ((1ull << (8 * a.prot_bytes)) - 1);
      const bool ok = valid && ((stored ^ h) & mask) == 0;
      if (act && a.out) a.out[i] = h;
      if (act && a.ok) a.ok[i] = ok ? 1 : 0;
      if (MODE == kKvMemVerify && act && a.status)
        a.status[i] = static_cast<uint8_t>(mst != kMemOk ? mst : ok ? kMemOk : kMemMismatch);
      const uint64_t badm = __ballot(act && !ok);
      if (a.mismatches && badm && lane == 0)
        atomicAdd(a.mismatches, static_cast<unsigned long long>(__popcll(badm)));
    } else if (act) {
      if (a.out) a.out[i] = h;
      if (a.enc_out)  // Encode(prot_bytes) (kv_checksum.h:97-115)
        for (uint32_t b = 0; b < a.prot_bytes; ++b)
          a.enc_out[i * a.prot_bytes + b] = static_cast<uint8_t>(h >> (8 * b));
    }
  }
}

}  // namespace

hipError_t launch_kv(int mode, const KvArgs& a, hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  const uint64_t per_wg = uint64_t(kWaves) * 64;
#ifndef FORST_KV_WG_PER_CU
#define FORST_KV_WG_PER_CU 16  // (grid: 4 resident per CU by LDS, the rest queue behind them: the grid-stride
                               // tiles end more evenly; A/B 4 / 8 / 16 in profiles/ab_r06/kv_grid_r06m.log)
#endif
  const uint32_t wg_per_cu = FORST_KV_WG_PER_CU;
  const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
      1, std::min<uint64_t>((a.n + per_wg - 1) / per_wg, uint64_t(di.num_cus) * wg_per_cu)));
  switch (mode) {
    case kKvHash:
      *name = "kv_kernel<hash64>";
      hipLaunchKernelGGL(kv_kernel<kKvHash>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    case kKvProtect:
      *name = "kv_kernel<protect>";
      hipLaunchKernelGGL(kv_kernel<kKvProtect>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    case kKvMemVerify:
      *name = "kv_kernel<mem_verify>";
      hipLaunchKernelGGL(kv_kernel<kKvMemVerify>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    case kKvMemProtect:
      *name = "kv_kernel<mem_protect>";
      hipLaunchKernelGGL(kv_kernel<kKvMemProtect>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    default:
      *name = "kv_kernel<verify>";
      hipLaunchKernelGGL(kv_kernel<kKvVerify>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
  }
  return hipGetLastError();
}

}  // namespace forst
