// forst_amd/csrc/xxhash_legacy.hip -- kxxHash (XXH32) and kxxHash64 (XXH64)
// block checksums on gfx950 (table/format.cc:573-576, :603-622;
// util/xxhash.h XXH32 ~:2400-2560, XXH64 ~:2750-2990, seed 0).
//
// XXH32/XXH64 are four serial accumulator chains over 16/32-byte stripes:
// no associativity to exploit inside one message.  So a wave hashes 16
// messages at once: lane group g = lane/4 owns message g, lane k = lane%4 owns
// accumulator v(k+1) and walks its chain (one 4/8-byte word per stripe; the 4
// lanes of a group together read each stripe contiguously).  The chains are
// latency-bound (~1 multiply-rotate-multiply per step) but 16 messages per
// wave x many waves per CU keep the HBM stream busy.  The group's lane 0
// merges the four accumulators and runs the <= 31-byte tail and avalanche.
//
// Block semantics: compute mode hashes payload || compression-type byte
// (the streaming XXH32_update(data) + XXH32_update(&last, 1) of
// format.cc:603-622 equals the one-shot hash of the concatenation; the type
// byte may live only in last_bytes[], so it is spliced in virtually); verify
// mode hashes data[0 .. size+1) and compares with the trailer.
#include <cstdlib>

#include "device_common.h"
#include "engine.h"

namespace forst {
namespace {

constexpr uint32_t kWaves = 4;
constexpr uint32_t kThreads = kWaves * 64;
constexpr uint32_t kMsgsPerWave = 16;

constexpr uint32_t Q32_1 = 0x9E3779B1u, Q32_2 = 0x85EBCA77u, Q32_3 = 0xC2B2AE3Du,
                   Q32_4 = 0x27D4EB2Fu, Q32_5 = 0x165667B1u;
constexpr uint64_t Q64_1 = 0x9E3779B185EBCA87ull, Q64_2 = 0xC2B2AE3D27D4EB4Full,
                   Q64_3 = 0x165667B19E3779F9ull, Q64_4 = 0x85EBCA77C2B2AE63ull,
                   Q64_5 = 0x27D4EB2F165667C5ull;

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) {
  return (x << r) | (x >> (32 - r));
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
__device__ __forceinline__ uint32_t r32(uint32_t acc, uint32_t in) {
  return rotl32(acc + in * Q32_2, 13) * Q32_1;
}
__device__ __forceinline__ uint64_t r64(uint64_t acc, uint64_t in) {
  return rotl64(acc + in * Q64_2, 31) * Q64_1;
}

// A message = mem[0 .. nmem) followed by `nv` (0/1) virtual byte `vb`.
struct Msg {
  const uint8_t* p;
  uint32_t nmem, nv, vb;
  __device__ __forceinline__ uint32_t total() const { return nmem + nv; }
  __device__ __forceinline__ uint32_t byte(uint32_t o) const {
    return o < nmem ? ldu8(p + o) : vb;
  }
  // little-endian W-byte word at offset o (o + W <= total())
  template <int W>
  __device__ __forceinline__ uint64_t word(uint32_t o) const {
    if (o + W <= nmem) return W == 8 ? ldu64(p + o) : ldu32(p + o);
    uint64_t v = 0;  // crosses the virtual byte: assemble byte-wise
    for (int b = W - 1; b >= 0; --b) v = (v << 8) | byte(o + b);
    return v;
  }
};

template <bool X64>
__device__ __forceinline__ uint32_t group_hash(const Msg& m, bool active, uint32_t lane) {
  constexpr uint32_t S = X64 ? 32 : 16;  // stripe bytes
  constexpr uint32_t W = X64 ? 8 : 4;    // word bytes per accumulator
  const uint32_t k = lane & 3;
  const uint32_t total = active ? m.total() : 0;
  const uint32_t nstripes = total / S;
  uint64_t v;
  if (X64) {
    const uint64_t init[4] = {Q64_1 + Q64_2, Q64_2, 0, 0 - Q64_1};
    v = k == 0 ? init[0] : k == 1 ? init[1] : k == 2 ? init[2] : init[3];
  } else {
    const uint32_t init[4] = {Q32_1 + Q32_2, Q32_2, 0, 0 - Q32_1};
    v = k == 0 ? init[0] : k == 1 ? init[1] : k == 2 ? init[2] : init[3];
  }
  // the serial chain: accumulator k eats word k of every stripe
  for (uint32_t t = 0; t < nstripes; ++t) {
    const uint64_t w = m.template word<W>(t * S + k * W);
    if (X64)
      v = r64(v, w);
    else
      v = r32(static_cast<uint32_t>(v), static_cast<uint32_t>(w));
  }
  // gather v1..v4 into every lane of the group (quad broadcast)
  const uint32_t base = lane & ~3u;
  uint64_t vv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = __shfl(static_cast<uint32_t>(v), base + q);
    const uint32_t hi = X64 ? __shfl(static_cast<uint32_t>(v >> 32), base + q) : 0u;
    vv[q] = (static_cast<uint64_t>(hi) << 32) | lo;
  }
  if (!active) return 0;
  if (X64) {
    uint64_t h;
    if (total >= 32) {
      h = rotl64(vv[0], 1) + rotl64(vv[1], 7) + rotl64(vv[2], 12) + rotl64(vv[3], 18);
#pragma unroll
      for (int q = 0; q < 4; ++q) h = (h ^ r64(0, vv[q])) * Q64_1 + Q64_4;
    } else {
      h = Q64_5;
    }
    h += total;
    uint32_t o = nstripes * 32;
    while (total - o >= 8) {
      h ^= r64(0, m.template word<8>(o));
      h = rotl64(h, 27) * Q64_1 + Q64_4;
      o += 8;
    }
    if (total - o >= 4) {
      h ^= m.template word<4>(o) * Q64_1;
      h = rotl64(h, 23) * Q64_2 + Q64_3;
      o += 4;
    }
    while (o < total) {
      h ^= m.byte(o) * Q64_5;
      h = rotl64(h, 11) * Q64_1;
      ++o;
    }
    h ^= h >> 33;
    h *= Q64_2;
    h ^= h >> 29;
    h *= Q64_3;
    h ^= h >> 32;
    return static_cast<uint32_t>(h);  // Lower32of64 (format.cc:576)
  } else {
    uint32_t h;
    if (total >= 16) {
      h = rotl32(static_cast<uint32_t>(vv[0]), 1) + rotl32(static_cast<uint32_t>(vv[1]), 7) +
          rotl32(static_cast<uint32_t>(vv[2]), 12) + rotl32(static_cast<uint32_t>(vv[3]), 18);
    } else {
      h = Q32_5;
    }
    h += total;
    uint32_t o = nstripes * 16;
    while (total - o >= 4) {
      h += static_cast<uint32_t>(m.template word<4>(o)) * Q32_3;
      h = rotl32(h, 17) * Q32_4;
      o += 4;
    }
    while (o < total) {
      h += m.byte(o) * Q32_5;
      h = rotl32(h, 11) * Q32_1;
      ++o;
    }
    h ^= h >> 15;
    h *= Q32_2;
    h ^= h >> 13;
    h *= Q32_3;
    h ^= h >> 16;
    return h;
  }
}

template <int MODE, bool X64>
__global__ void __launch_bounds__(kThreads) xxhash_legacy_kernel(BlockArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t g = lane >> 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kWaves * kMsgsPerWave;
  for (uint64_t b0 = (static_cast<uint64_t>(blockIdx.x) * kWaves + wave) * kMsgsPerWave;
       b0 < a.n; b0 += stride) {
    const uint64_t i = b0 + g;
    bool active = i < a.n;
    uint64_t off = 0;
    uint32_t size = 0;
    bool valid = false;
    Msg m{a.base, 0, 0, 0};
    uint32_t stored = 0, mod = 0, last = 0;
    if (active) {
      off = a.offsets[i];
      size = a.sizes[i];
      uint64_t need = size;
      if (MODE == kModeVerify || MODE == kModeTrailer) need += 5;
      if (MODE == kModeCompute && a.last_bytes == nullptr) need += 1;
      valid = off <= a.base_len && need <= a.base_len - off;
    }
    if (valid) {
      const uint8_t* p = a.base + off;
      m.p = p;
      mod = a.modifiers ? a.modifiers[i] : 0u;
      if (MODE == kModeVerify) {
        m.nmem = size + 1;  // ComputeBuiltinChecksum(type, data, size+1)
        stored = ldu32(p + size + 1);
      } else if (MODE == kModeRaw) {
        m.nmem = size;
      } else {
        last = a.last_bytes ? a.last_bytes[i] : ldu8(p + size);
        m.nmem = size;
        m.nv = 1;
        m.vb = last;
      }
    }
    const uint32_t h = group_hash<X64>(m, valid, lane);
    if (!active || (lane & 3) != 0) continue;
    if (!valid) {
      if (a.out32) a.out32[i] = 0;
      if (MODE == kModeVerify) {
        if (a.ok_out) a.ok_out[i] = 0;
        if (a.stored_out) a.stored_out[i] = 0;
        if (a.mismatches) atomicAdd(a.mismatches, 1ull);
      }
      continue;
    }
    if (MODE == kModeRaw) {
      a.out32[i] = h;
    } else if (MODE == kModeVerify) {
      const uint32_t st = stored - mod;
      const bool ok = st == h;
      if (a.out32) a.out32[i] = h;
      if (a.stored_out) a.stored_out[i] = st;
      if (a.ok_out) a.ok_out[i] = ok ? 1 : 0;
      if (!ok && a.mismatches) atomicAdd(a.mismatches, 1ull);
    } else {
      const uint32_t c = h + mod;
      if (a.out32) a.out32[i] = c;
      if (MODE == kModeTrailer) {
        uint8_t* w = a.base_w + off + size;
        w[0] = static_cast<uint8_t>(last);
        stu32_bytes(w + 1, c);
      }
    }
  }
}

template <bool X64>
hipError_t launch_mode(int mode, const BlockArgs& a, hipStream_t stream, uint32_t grid,
                       const char** name) {
  switch (mode) {
    case kModeCompute:
      *name = X64 ? "xxhash64_block_kernel<compute>" : "xxhash32_block_kernel<compute>";
      hipLaunchKernelGGL((xxhash_legacy_kernel<kModeCompute, X64>), dim3(grid), dim3(kThreads),
                         0, stream, a);
      break;
    case kModeTrailer:
      *name = X64 ? "xxhash64_block_kernel<trailer>" : "xxhash32_block_kernel<trailer>";
      hipLaunchKernelGGL((xxhash_legacy_kernel<kModeTrailer, X64>), dim3(grid), dim3(kThreads),
                         0, stream, a);
      break;
    case kModeVerify:
      *name = X64 ? "xxhash64_block_kernel<verify>" : "xxhash32_block_kernel<verify>";
      hipLaunchKernelGGL((xxhash_legacy_kernel<kModeVerify, X64>), dim3(grid), dim3(kThreads),
                         0, stream, a);
      break;
    default:
      *name = X64 ? "xxhash64_block_kernel<raw>" : "xxhash32_block_kernel<raw>";
      hipLaunchKernelGGL((xxhash_legacy_kernel<kModeRaw, X64>), dim3(grid), dim3(kThreads), 0,
                         stream, a);
      break;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_xxhash_legacy_blocks(bool x64, int mode, const BlockArgs& a,
                                       hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  const uint64_t per_wg = uint64_t(kWaves) * kMsgsPerWave;
  const uint32_t grid = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>((a.n + per_wg - 1) / per_wg,
                                               uint64_t(di.num_cus) * 16)));
  return x64 ? launch_mode<true>(mode, a, stream, grid, name)
             : launch_mode<false>(mode, a, stream, grid, name);
}

}  // namespace forst
