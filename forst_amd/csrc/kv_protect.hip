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
// Layout: one wave per 64 entries, one LANE per entry for fields <= 240 bytes
// (keys, small values, op/seq/cf: the length-class formulas need no cross-lane
// work); every field > 240 bytes is hashed by the WHOLE wave in turn (ballot
// of the long fields, the XXH3-style lane split: lane L takes 16 bytes --
// stripe L/4, accumulator pair L%4 -- of each 1 KiB block, 16-lane stripe sum,
// serial scramble), and the owner lane XORs the result in.
#include <cstdlib>

#include "device_common.h"
#include "engine.h"
#include "stream_common.h"
#include "xxh_common.h"

namespace forst {
namespace {

constexpr uint32_t kWaves = 4;
constexpr uint32_t kThreads = kWaves * 64;

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

// 8 bytes at byte offset `off` of the seeded custom secret (xxph3.h:1609-1620:
// word 2i gets +seed, word 2i+1 gets -seed)
__device__ __forceinline__ uint64_t psec64(uint32_t off, uint64_t seed) {
  const uint32_t w = off >> 3, sh = off & 7;
  const uint64_t a = sec64(8 * w) + ((w & 1) ? (0 - seed) : seed);
  if (sh == 0) return a;
  const uint64_t b = sec64(8 * w + 8) + ((w & 1) ? seed : (0 - seed));
  return (a >> (8 * sh)) | (b << (64 - 8 * sh));
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
// xxph3.h:1640 XXPH3_mix16B (default secret, explicit seed)
__device__ __forceinline__ uint64_t xxph3_mix16B(const uint8_t* in, uint32_t s, uint64_t seed) {
  return mul128_fold64(ldu64(in) ^ (sec64(s) + seed), ldu64(in + 8) ^ (sec64(s + 8) - seed));
}

// XXPH3_64bits_withSeed for len <= 240 (per lane, xxph3.h:1126-1140,
// 1651-1707)
__device__ uint64_t xxph3_short(const uint8_t* in, uint32_t len, uint64_t seed) {
  if (len <= 16) {
    if (len > 8) {
      const uint64_t lo = ldu64(in) ^ (sec64(0) + seed);
      const uint64_t hi = ldu64(in + len - 8) ^ (sec64(8) - seed);
      return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
    }
    if (len >= 4) {
      const uint64_t in64 = ldu32(in) | (static_cast<uint64_t>(ldu32(in + len - 4)) << 32);
      return xxph3_4to8(in64, len, seed);
    }
    if (len) return xxph3_1to3(ldu8(in), ldu8(in + (len >> 1)), ldu8(in + len - 1), len, seed);
    return mul128_fold64(seed + sec64(0), P64_2);  // xxph3.h:1133-1138 (RocksDB)
  }
  if (len <= 128) {
    uint64_t acc = len * P64_1;
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += xxph3_mix16B(in + 48, 96, seed);
          acc += xxph3_mix16B(in + len - 64, 112, seed);
        }
        acc += xxph3_mix16B(in + 32, 64, seed);
        acc += xxph3_mix16B(in + len - 48, 80, seed);
      }
      acc += xxph3_mix16B(in + 16, 32, seed);
      acc += xxph3_mix16B(in + len - 32, 48, seed);
    }
    acc += xxph3_mix16B(in, 0, seed);
    acc += xxph3_mix16B(in + len - 16, 16, seed);
    return xxph3_avalanche(acc);
  }
  uint64_t acc = len * P64_1;
  for (uint32_t i = 0; i < 8; ++i) acc += xxph3_mix16B(in + 16 * i, 16 * i, seed);
  acc = xxph3_avalanche(acc);
  const uint32_t nb_rounds = len / 16;
  for (uint32_t i = 8; i < nb_rounds; ++i) acc += xxph3_mix16B(in + 16 * i, 16 * (i - 8) + 3, seed);
  acc += xxph3_mix16B(in + len - 16, 136 - 17, seed);
  return xxph3_avalanche(acc);
}

__device__ __forceinline__ uint64_t scramble_acc(uint64_t a, uint64_t key) {
  a ^= a >> 47;
  a ^= key;
  return a * P32_1;
}

// XXPH3_64bits_withSeed for len > 240, whole wave (all arguments uniform);
// every lane returns the hash.  xxph3.h:1514-1583, 1630-1637.
__device__ uint64_t wave_xxph3_long(const uint8_t* p, uint32_t len, uint64_t seed, uint32_t lane) {
  const uint32_t s = lane >> 2, pp = lane & 3;
  const uint64_t k0 = psec64(8 * s + 16 * pp, seed), k1 = psec64(8 * s + 16 * pp + 8, seed);
  const uint64_t ks0 = psec64(128 + 16 * pp, seed), ks1 = psec64(136 + 16 * pp, seed);
  // XXPH3_INIT_ACC (xxph3.h:1567)
  uint64_t acc0 = pp == 0 ? P32_3 : pp == 1 ? P64_2 : pp == 2 ? P64_4 : P64_5;
  uint64_t acc1 = pp == 0 ? P64_1 : pp == 1 ? P64_3 : pp == 2 ? P32_2 : P32_1;
  const uint32_t nb = len / 1024;
  const uint32_t nbS = (len - 1024 * nb) / 64;
  const uint32_t m = static_cast<uint32_t>(reinterpret_cast<uint64_t>(p) & 3);
  const uint8_t* q = p - m + 16 * lane;
  uint32_t g = 0;
  for (; g + 4 <= nb; g += 4) {  // 4 loads in flight per lane
    uint64_t c0[4], c1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t d0, d1;
      ld16u(q + 1024 * (g + j), m, d0, d1);
      c0[j] = d0 + mul32to64(d0 ^ k0);  // acc_64bits: acc[i] += data + lo*hi(data ^ key)
      c1[j] = d1 + mul32to64(d1 ^ k1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = scramble_acc(acc0 + stripe_sum(c0[j]), ks0);
      acc1 = scramble_acc(acc1 + stripe_sum(c1[j]), ks1);
    }
  }
  for (; g < nb; ++g) {
    uint64_t d0, d1;
    ld16u(q + 1024 * g, m, d0, d1);
    acc0 = scramble_acc(acc0 + stripe_sum(d0 + mul32to64(d0 ^ k0)), ks0);
    acc1 = scramble_acc(acc1 + stripe_sum(d1 + mul32to64(d1 ^ k1)), ks1);
  }
  {  // last partial block: stripes [0, nbS), no scramble
    uint64_t c0 = 0, c1 = 0;
    if (s < nbS) {
      uint64_t d0, d1;
      ld16u(q + 1024 * nb, m, d0, d1);
      c0 = d0 + mul32to64(d0 ^ k0);
      c1 = d1 + mul32to64(d1 ^ k1);
    }
    acc0 += stripe_sum(c0);
    acc1 += stripe_sum(c1);
  }
  if (len & 63) {  // last stripe at len - 64, secret + 192 - 64 - 7 (xxph3.h:1539-1542)
    const uint8_t* lp = p + len - 64 + 16 * pp;
    const uint32_t ml = static_cast<uint32_t>(reinterpret_cast<uint64_t>(lp) & 3);
    uint64_t d0, d1;
    ld16u(lp - ml, ml, d0, d1);
    acc0 += d0 + mul32to64(d0 ^ psec64(121 + 16 * pp, seed));
    acc1 += d1 + mul32to64(d1 ^ psec64(129 + 16 * pp, seed));
  }
  // XXPH3_mergeAccs from secret + 11 (xxph3.h:1554-1582)
  uint64_t t = mul128_fold64(acc0 ^ psec64(11 + 16 * pp, seed), acc1 ^ psec64(19 + 16 * pp, seed));
  t += quad_xor64<1>(t);
  t += quad_xor64<2>(t);
  return xxph3_avalanche(static_cast<uint64_t>(len) * P64_1 + t);
}

// The same on one 16-lane row (t = lane & 15), four fields per wave at once
// (round 5): lane t takes the 16-byte chunks at 16 t + 256 k of each 1 KiB
// block (stripe t/4 + 4k, accumulator pair t%4), and the last stripe's load
// is issued with them, so a field under 1 KiB (a value of 240..1000 bytes,
// the memtable shape) costs one round trip to memory instead of two, and
// four of them overlap.  Every lane of the row returns the hash.
__device__ uint64_t row_xxph3_long(const uint8_t* p, uint32_t len, uint64_t seed, uint32_t t) {
  const uint32_t s4 = t >> 2, pp = t & 3;
  uint64_t acc0 = pp == 0 ? P32_3 : pp == 1 ? P64_2 : pp == 2 ? P64_4 : P64_5;
  uint64_t acc1 = pp == 0 ? P64_1 : pp == 1 ? P64_3 : pp == 2 ? P32_2 : P32_1;
  const uint32_t nb = len / 1024;
  const uint32_t nbS = (len - 1024 * nb) / 64;
  const uint32_t m = static_cast<uint32_t>(reinterpret_cast<uint64_t>(p) & 3);
  const uint8_t* q = p - m + 16 * t;
  const uint64_t ks0 = psec64(128 + 16 * pp, seed), ks1 = psec64(136 + 16 * pp, seed);
  // the last stripe (xxph3.h:1539-1542), loaded up front
  uint64_t l0 = 0, l1 = 0;
  {
    const uint8_t* lp = p + len - 64 + 16 * pp;
    const uint32_t ml = static_cast<uint32_t>(reinterpret_cast<uint64_t>(lp) & 3);
    ld16u(lp - ml, ml, l0, l1);
  }
  // (rows of one wave may have different block counts: the loop runs to the
  // wave's largest, wave-uniform around the row sums)
  for (uint32_t g = 0; __ballot(g <= nb); ++g) {
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t st = s4 + 4 * k;
      if (g < nb || (g == nb && st < nbS)) {
        uint64_t d0, d1;
        ld16u(q + 1024 * g + 256 * k, m, d0, d1);
        c0 += d0 + mul32to64(d0 ^ psec64(8 * st + 16 * pp, seed));  // acc_64bits
        c1 += d1 + mul32to64(d1 ^ psec64(8 * st + 16 * pp + 8, seed));
      }
    }
    c0 += row_ror64<4>(c0);
    c1 += row_ror64<4>(c1);
    c0 += row_ror64<8>(c0);
    c1 += row_ror64<8>(c1);
    if (g <= nb) {
      acc0 += c0;
      acc1 += c1;
    }
    if (g < nb) {
      acc0 = scramble_acc(acc0, ks0);
      acc1 = scramble_acc(acc1, ks1);
    }
  }
  if (len & 63) {
    acc0 += l0 + mul32to64(l0 ^ psec64(121 + 16 * pp, seed));
    acc1 += l1 + mul32to64(l1 ^ psec64(129 + 16 * pp, seed));
  }
  uint64_t h = mul128_fold64(acc0 ^ psec64(11 + 16 * pp, seed), acc1 ^ psec64(19 + 16 * pp, seed));
  h += quad_xor64<1>(h);
  h += quad_xor64<2>(h);
  return xxph3_avalanche(static_cast<uint64_t>(len) * P64_1 + h);
}

#ifndef FORST_KV_ROWS
#define FORST_KV_ROWS 1
#endif

__device__ __forceinline__ bool in_range(uint64_t off, uint64_t len, uint64_t base_len) {
  return off <= base_len && len <= base_len - off;
}

// MODE: kKvHash (Hash64 per buffer), kKvProtect, kKvVerify
template <int MODE>
__global__ void __launch_bounds__(kThreads) kv_kernel(KvArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWaves * 64;
  for (uint64_t b0 = (static_cast<uint64_t>(blockIdx.x) * kWaves + wave) * 64; b0 < a.n;
       b0 += stride) {
    const uint64_t i = b0 + lane;
    const bool act = i < a.n;
    uint64_t ko = 0, vo = 0, co = 0, kseed = kSeedK;
    uint32_t kl = 0, vl = 0;
    bool valid = false;
    if (act) {
      ko = a.key_off[i];
      kl = a.key_len[i];
      valid = in_range(ko, kl, a.base_len);
      if (MODE == kKvHash) {
        kseed = a.seeds ? a.seeds[i] : a.seed;
      } else {
        vo = a.val_off[i];
        vl = a.val_len[i];
        valid = valid && in_range(vo, vl, a.base_len);
      }
      if (MODE == kKvVerify) {
        co = a.chk_off[i];
        valid = valid && in_range(co, a.prot_bytes, a.base_len);
      }
    }
    uint64_t h = 0;
    if (valid && kl <= 240) h ^= xxph3_short(a.base + ko, kl, kseed);
    if (MODE != kKvHash) {
      if (valid && vl <= 240) h ^= xxph3_short(a.base + vo, vl, kSeedV);
      if (valid && a.ops) {  // NPHash64(&op_type, 1, kSeedO)
        const uint32_t op = a.ops[i];
        h ^= xxph3_1to3(op, op, op, 1, kSeedO);
      }
      if (valid && a.seqs) h ^= xxph3_4to8(a.seqs[i], 8, kSeedS);  // native LE bytes
      if (valid && a.cfs) {
        const uint64_t cf = a.cfs[i];
        h ^= xxph3_4to8(cf | (cf << 32), 4, kSeedC);
      }
    }
    if (FORST_KV_ROWS) {
      // fields > 240 bytes: four at a time, one per 16-lane row (keys first)
      uint64_t lk = __ballot(valid && kl > 240);
      uint64_t lv = MODE != kKvHash ? __ballot(valid && vl > 240) : 0ull;
      const uint32_t row = lane >> 4, t = lane & 15;
      while (lk | lv) {
        uint32_t src = 64, isv = 0;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
          uint32_t sr = 64, vr = 0;
          if (lk) {
            sr = static_cast<uint32_t>(__builtin_ctzll(lk));
            lk &= lk - 1;
          } else if (lv) {
            sr = static_cast<uint32_t>(__builtin_ctzll(lv));
            lv &= lv - 1;
            vr = 1;
          }
          if (row == r) {
            src = sr;
            isv = vr;
          }
        }
        const uint32_t sl = src < 64 ? src : 0;
        // (the source lane's key and value fields, the row picks one)
        const uint32_t klo = __shfl(static_cast<uint32_t>(ko), sl);
        const uint32_t khi = __shfl(static_cast<uint32_t>(ko >> 32), sl);
        const uint32_t kln = __shfl(kl, sl);
        uint32_t vlo = 0, vhi = 0, vln = 0;
        if (MODE != kKvHash) {
          vlo = __shfl(static_cast<uint32_t>(vo), sl);
          vhi = __shfl(static_cast<uint32_t>(vo >> 32), sl);
          vln = __shfl(vl, sl);
        }
        const uint32_t flo = isv ? vlo : klo, fhi = isv ? vhi : khi, fl = isv ? vln : kln;
        const uint32_t slo = __shfl(static_cast<uint32_t>(kseed), sl);
        const uint32_t shi = __shfl(static_cast<uint32_t>(kseed >> 32), sl);
        const uint64_t o = src < 64 ? (static_cast<uint64_t>(fhi) << 32) | flo : 0ull;
        const uint64_t sd = isv ? kSeedV : (static_cast<uint64_t>(shi) << 32) | slo;
        // (a row without a field hashes the buffer's first 241 bytes, discarded: a
        // long field exists, so base_len > 240)
        const uint64_t hv = row_xxph3_long(a.base + o, src < 64 ? fl : 241u, sd, t);
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
          const uint32_t sr = readlane32(src, 16 * r);
          const uint64_t vr = readlane64(static_cast<uint32_t>(hv), static_cast<uint32_t>(hv >> 32),
                                         16 * r);
          if (lane == sr) h ^= vr;
        }
      }
    }
    // fields > 240 bytes: the whole wave hashes them one after the other
    uint64_t lk = FORST_KV_ROWS ? 0ull : __ballot(valid && kl > 240);
    while (lk) {
      const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(lk));
      lk &= lk - 1;
      const uint64_t o = readlane64(static_cast<uint32_t>(ko), static_cast<uint32_t>(ko >> 32), l);
      const uint32_t n = readlane32(kl, l);
      const uint64_t sd = readlane64(static_cast<uint32_t>(kseed), static_cast<uint32_t>(kseed >> 32), l);
      const uint64_t hv = wave_xxph3_long(a.base + o, n, sd, lane);
      h ^= lane == l ? hv : 0ull;
    }
    if (MODE != kKvHash && !FORST_KV_ROWS) {
      uint64_t lv = __ballot(valid && vl > 240);
      while (lv) {
        const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(lv));
        lv &= lv - 1;
        const uint64_t o = readlane64(static_cast<uint32_t>(vo), static_cast<uint32_t>(vo >> 32), l);
        const uint32_t n = readlane32(vl, l);
        const uint64_t hv = wave_xxph3_long(a.base + o, n, kSeedV, lane);
        h ^= lane == l ? hv : 0ull;
      }
    }
    if (!valid) h = 0;
    if (MODE == kKvVerify) {
      // ProtectionInfo<T>::Verify (kv_checksum.h:117-133): low prot_bytes bytes, LE
      uint64_t stored = 0;
      if (valid)
        for (uint32_t b = 0; b < a.prot_bytes; ++b)
          stored |= static_cast<uint64_t>(ldu8(a.base + co + b)) << (8 * b);
      const uint64_t mask = a.prot_bytes >= 8 ? ~0ull : ((1ull << (8 * a.prot_bytes)) - 1);
      const bool ok = valid && ((stored ^ h) & mask) == 0;
      if (act && a.out) a.out[i] = h;
      if (act && a.ok) a.ok[i] = ok ? 1 : 0;
      const uint64_t badm = __ballot(act && !ok);
      if (a.mismatches && badm && lane == 0)
        atomicAdd(a.mismatches, static_cast<unsigned long long>(__popcll(badm)));
    } else if (act) {
      a.out[i] = h;
    }
  }
}

}  // namespace

hipError_t launch_kv(int mode, const KvArgs& a, hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  const uint64_t per_wg = uint64_t(kWaves) * 64;
  const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
      1, std::min<uint64_t>((a.n + per_wg - 1) / per_wg, uint64_t(di.num_cus) * 8)));
  switch (mode) {
    case kKvHash:
      *name = "kv_kernel<hash64>";
      hipLaunchKernelGGL(kv_kernel<kKvHash>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    case kKvProtect:
      *name = "kv_kernel<protect>";
      hipLaunchKernelGGL(kv_kernel<kKvProtect>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
    default:
      *name = "kv_kernel<verify>";
      hipLaunchKernelGGL(kv_kernel<kKvVerify>, dim3(grid), dim3(kThreads), 0, stream, a);
      break;
  }
  return hipGetLastError();
}

}  // namespace forst
