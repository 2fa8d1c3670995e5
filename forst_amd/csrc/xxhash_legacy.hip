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

// ---- one message per lane (round 5) ------------------------------------------
// The group kernel above gives each accumulator its own lane: every chain
// step waits for a 4/8-byte load of its own, and the 16 messages of a wave
// cover 16 x 16 bytes per load instruction -- 0.21 (XXH32) / 0.31 (XXH64) of
// the HBM peak on 1 M x 16 KiB (bench round 5).  Here one LANE hashes one
// message with its four accumulators in registers (four independent chains),
// reading kLStep bytes per step with 16-byte loads and one realignment
// dword; a wave works on 64 messages, and a lane that is done takes the next
// message of the wave's batch at once, so no lane waits for the wave's
// longest message (batches of 64 descriptors: the first static, the rest
// claimed from a ticket).  The last < kLStep + 4 bytes (the stripes the
// steps leave, the tail and the virtual type byte of compute mode) are
// copied into the lane's LDS slot with independent loads and finished there.
constexpr uint32_t kLWaves = 4;
constexpr uint32_t kLThreads = kLWaves * 64;
// 256 bytes per message and step, one 4-wave workgroup per CU (the CU streams
// 256 messages at once).  Round 6: the step's bytes are loaded COALESCED --
// 16 lanes read one message's 256 bytes with one 16-byte load each, 4
// messages per load instruction -- and written to the owning lanes' LDS
// slots, from which each lane reads its own 256 bytes back.  Per-lane 16-byte
// loads (round 5) touched 64 lines per instruction and stopped at 0.61 of the
// HBM peak whatever the step size, occupancy or prefetch depth; the
// transposed form touches 8.  A/B, 1 M x 16 KiB, verify / trailer fraction
// of the HBM peak (profiles/ab_r06/xxhash_lane_xpose_r06bc.log,
// xxhash_lane_pf_s512_r06a.log; profiles/ab_r05/xxhash_lane_step_occupancy.log):
// round 4's group kernel 0.21 / 0.21 (XXH32), 0.32 / 0.31 (XXH64); per-lane
// loads, 64-byte steps 0.41 / 0.40, 128 B 0.56 / 0.57, 256 B 0.61 / 0.62,
// 512 B 0.58 / 0.56, 256 B with the next step loaded one iteration ahead
// 0.60 / 0.62; transposed 0.675 / 0.722 (XXH32), 0.66 / 0.716 (XXH64), with
// the prefetch as well 0.66 / 0.71, at 2 workgroups per CU 0.655 / 0.63.
#ifndef FORST_LANE_WG_PER_CU
#define FORST_LANE_WG_PER_CU 1
#endif
#ifndef FORST_LANE_TRL_STAGE
#define FORST_LANE_TRL_STAGE 1
#endif
#ifndef FORST_LANE_TRL_CAP
#define FORST_LANE_TRL_CAP 8192
#endif
constexpr uint32_t kTrlCap = FORST_LANE_TRL_CAP;  // staged trailers per workgroup (64 KiB of LDS)
struct TrlEntry {
  uint32_t i, c;  // descriptor, checksum
};
constexpr uint32_t kLStep = 256;          // bytes per message and step: 16 lanes x 16
constexpr uint32_t kLSlot = kLStep + 16;  // LDS bytes per lane: a step's row, or the
                                          // < kLStep + 11 tail bytes (16-byte multiple)

// little-endian word at byte o of a lane's slot (o + 8 <= kLSlot)
__device__ __forceinline__ uint32_t slot32(const uint8_t* sl, uint32_t o) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(sl + (o & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], o & 3u);
}
__device__ __forceinline__ uint64_t slot64(const uint8_t* sl, uint32_t o) {
  return static_cast<uint64_t>(slot32(sl, o)) | (static_cast<uint64_t>(slot32(sl, o + 4)) << 32);
}

template <int MODE, bool X64>
__global__ void __launch_bounds__(kLThreads) xxhash_lane_kernel(BlockArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t slots[kLThreads * kLSlot / 4];
  // trailer mode: (descriptor, checksum) pairs written after the loop
  __shared__ TrlEntry s_trl[FORST_LANE_TRL_STAGE && MODE == kModeTrailer ? kTrlCap : 1];
  __shared__ uint32_t s_ntrl;
  if (FORST_LANE_TRL_STAGE && MODE == kModeTrailer) {
    if (threadIdx.x == 0) s_ntrl = 0;
    __syncthreads();
  }
  constexpr uint32_t S = X64 ? 32 : 16;  // stripe bytes
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  uint8_t* sl = reinterpret_cast<uint8_t*>(slots) + threadIdx.x * kLSlot;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kLWaves;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * kLWaves + wave;
  // the wave's batch [bcur, bend) of descriptors not yet taken by a lane
  uint64_t bcur = gw * 64 < a.n ? gw * 64 : a.n;
  uint64_t bend = bcur + 64 < a.n ? bcur + 64 : a.n;
  bool more = bcur < a.n;  // (wave-uniform) batches may remain
  // per lane: its message
  bool have = false;
  uint64_t i = 0, off = 0;
  const uint8_t* pa = a.base;
  uint32_t m = 0, nmem = 0, nv = 0, vb = 0, pos = 0, vend = 0, size = 0, stored = 0, mod = 0;
  bool valid = false;
  uint64_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
  for (;;) {
    // ---- lanes without a message take the next ones of the batch
    uint64_t need = __ballot(!have);
    while (need && more) {
      const uint32_t rank = static_cast<uint32_t>(__popcll(need & ((1ull << lane) - 1)));
      const uint64_t avail = bend - bcur;
      if (!have && rank < avail) {
        i = bcur + rank;
        have = true;
        off = a.offsets[i];
        size = a.sizes[i];
        uint64_t nd = size;
        if (MODE == kModeVerify || MODE == kModeTrailer) nd += 5;
        if (MODE == kModeCompute && a.last_bytes == nullptr) nd += 1;
        valid = off <= a.base_len && nd <= a.base_len - off;
        mod = valid && a.modifiers ? a.modifiers[i] : 0u;
        const uint8_t* p = a.base + (valid ? off : 0);
        m = static_cast<uint32_t>(reinterpret_cast<uint64_t>(p) & 3u);
        pa = p - m;
        nv = 0;
        vb = 0;
        stored = 0;
        if (!valid) {
          nmem = 0;
        } else if (MODE == kModeVerify) {
          nmem = size + 1;  // ComputeBuiltinChecksum(type, data, size+1); the
                            // stored word after it is read from the tail slot
        } else if (MODE == kModeRaw) {
          nmem = size;
        } else {
          nmem = size;
          nv = 1;
          vb = a.last_bytes ? a.last_bytes[i] : ldu8(p + size);
        }
        // steps whose aligned window [pa + pos, + kLStep + 4) lies in the
        // message's own bytes, counted without m: messages of one size take
        // the same number of steps whatever their alignment, so the lanes of
        // a wave stay in step (with m in the count, verify's 16 KiB + 1 byte
        // messages took 63 or 64 steps and the wave's lanes drifted apart)
        vend = nmem >= kLStep + 4 ? ((nmem - 4) & ~(kLStep - 1)) : 0u;
        pos = 0;
        if (X64) {
          v0 = Q64_1 + Q64_2;
          v1 = Q64_2;
          v2 = 0;
          v3 = 0 - Q64_1;
        } else {
          v0 = static_cast<uint32_t>(Q32_1 + Q32_2);
          v1 = Q32_2;
          v2 = 0;
          v3 = static_cast<uint32_t>(0u - Q32_1);
        }
      }
      const uint64_t took = static_cast<uint64_t>(__popcll(need)) < avail
                                ? static_cast<uint64_t>(__popcll(need)) : avail;
      bcur += took;
      need = __ballot(!have);
      if (bcur >= bend) {  // the batch is used up: claim the next one
        uint64_t nb = 0;
        if (lane == 0) nb = nw + atomicAdd(a.ticket, 1ull);
        nb = uniform64(nb) * 64;
        if (nb >= a.n) {
          more = false;
        } else {
          bcur = nb;
          bend = nb + 64 < a.n ? nb + 64 : a.n;
        }
      }
    }
    if (!__ballot(have)) break;
    // ---- one kLStep-byte step of every lane that has one left
    const bool vec = have && pos < vend;
    const uint64_t vmask = __ballot(vec);
    if (vmask) {
      constexpr int kW = kLStep / 4;  // dwords per step
      uint32_t d[kW + 1];
      // coalesced: lane 16g + j loads chunk j of message 4k + g's step for
      // k = 0..15 into that message's row (its lane's slot); then each lane
      // reads its own row (rows 272 bytes apart: conflict-free b128 reads)
      const uint64_t qa = reinterpret_cast<uint64_t>(pa + pos);
      const uint32_t j = lane & 15;
      uint8_t* const wl = reinterpret_cast<uint8_t*>(slots) + (threadIdx.x & ~63u) * kLSlot;
      u32x4a4 x[16];
      const uint8_t* sp[16];  // message 4k + (lane >> 4)'s step address (all lanes
#pragma unroll                // take part in the shuffles: no selects around them)
      for (int k = 0; k < 16; ++k) {
        const uint32_t src = 4 * k + (lane >> 4);
        const uint32_t lo = __shfl(static_cast<uint32_t>(qa), src);
        const uint32_t hi = __shfl(static_cast<uint32_t>(qa >> 32), src);
        sp[k] = reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t src = 4 * k + (lane >> 4);
        x[k] = ld16_a4(((vmask >> src) & 1 ? sp[k] : a.base) + 16 * j + vzero());
      }
      d[kW] = ld4_a4((vec ? pa + pos : a.base) + kLStep + vzero());
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t src = 4 * k + (lane >> 4);
        *reinterpret_cast<u32x4a4*>(wl + src * kLSlot + 16 * j) = x[k];
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < kW / 4; ++k) {
        const u32x4a4 y = *reinterpret_cast<const u32x4a4*>(sl + 16 * k);
        d[4 * k] = y.x;
        d[4 * k + 1] = y.y;
        d[4 * k + 2] = y.z;
        d[4 * k + 3] = y.w;
      }
      __builtin_amdgcn_wave_barrier();
      if (vec) {
        uint32_t w[kW];
#pragma unroll
        for (int j = 0; j < kW; ++j) w[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], m);
        if (X64) {
#pragma unroll
          for (int st = 0; st < kW / 8; ++st) {
            const uint32_t* x = w + 8 * st;
            v0 = r64(v0, static_cast<uint64_t>(x[0]) | (static_cast<uint64_t>(x[1]) << 32));
            v1 = r64(v1, static_cast<uint64_t>(x[2]) | (static_cast<uint64_t>(x[3]) << 32));
            v2 = r64(v2, static_cast<uint64_t>(x[4]) | (static_cast<uint64_t>(x[5]) << 32));
            v3 = r64(v3, static_cast<uint64_t>(x[6]) | (static_cast<uint64_t>(x[7]) << 32));
          }
        } else {
#pragma unroll
          for (int st = 0; st < kW / 4; ++st) {
            v0 = r32(static_cast<uint32_t>(v0), w[4 * st]);
            v1 = r32(static_cast<uint32_t>(v1), w[4 * st + 1]);
            v2 = r32(static_cast<uint32_t>(v2), w[4 * st + 2]);
            v3 = r32(static_cast<uint32_t>(v3), w[4 * st + 3]);
          }
        }
        pos += kLStep;
      }
    }
    // ---- lanes whose steps are done: the rest from the LDS slot, then store
    const bool fin = have && pos >= vend;
    if (!__ballot(fin)) continue;
    if (fin) {
      // bytes [vend, nmem) as the dword-aligned words from pa + vend (at slot
      // byte m + x for message byte vend + x), in verify mode with the 4
      // stored checksum bytes after them; words past those are 0
      const uint32_t span = m + (nmem - vend);  // < kLStep + 7
      const uint32_t want = span + (MODE == kModeVerify ? 4u : 0u);
      const uint8_t* q = pa + vend;
      constexpr int kT = kLStep / 4 + (MODE == kModeVerify ? 3 : 2);
      uint32_t t[kT];
#pragma unroll
      for (int k = 0; k < kT; ++k) t[k] = 4u * k < want ? ld4_a4(q + 4 * k + vzero()) : 0u;
      uint32_t* sw = reinterpret_cast<uint32_t*>(sl);
#pragma unroll
      for (int k = 0; k < kT; ++k) sw[k] = t[k];
#pragma unroll
      for (int k = kT; k < static_cast<int>(kLSlot / 4); ++k) sw[k] = 0u;
      if (nv) sl[span] = static_cast<uint8_t>(vb);
      if (MODE == kModeVerify) stored = slot32(sl, span);
    }
    if (fin) {
      const uint32_t total = nmem + nv;
      const uint32_t nst = total / S;  // stripes of the whole message
      uint32_t o = vend;               // message offset; slot byte m + (o - vend)
      auto w32 = [&](uint32_t at) { return slot32(sl, m + (at - vend)); };
      auto w64 = [&](uint32_t at) { return slot64(sl, m + (at - vend)); };
      for (; o + S <= nst * S; o += S) {  // the stripes after the steps
        if (X64) {
          v0 = r64(v0, w64(o));
          v1 = r64(v1, w64(o + 8));
          v2 = r64(v2, w64(o + 16));
          v3 = r64(v3, w64(o + 24));
        } else {
          v0 = r32(static_cast<uint32_t>(v0), w32(o));
          v1 = r32(static_cast<uint32_t>(v1), w32(o + 4));
          v2 = r32(static_cast<uint32_t>(v2), w32(o + 8));
          v3 = r32(static_cast<uint32_t>(v3), w32(o + 12));
        }
      }
      uint32_t h;
      if (X64) {  // XXH64_finalize (util/xxhash.h ~:2750-2990)
        uint64_t hh;
        if (total >= 32) {
          hh = rotl64(v0, 1) + rotl64(v1, 7) + rotl64(v2, 12) + rotl64(v3, 18);
          hh = (hh ^ r64(0, v0)) * Q64_1 + Q64_4;
          hh = (hh ^ r64(0, v1)) * Q64_1 + Q64_4;
          hh = (hh ^ r64(0, v2)) * Q64_1 + Q64_4;
          hh = (hh ^ r64(0, v3)) * Q64_1 + Q64_4;
        } else {
          hh = Q64_5;
        }
        hh += total;
        for (; total - o >= 8; o += 8) {
          hh ^= r64(0, w64(o));
          hh = rotl64(hh, 27) * Q64_1 + Q64_4;
        }
        if (total - o >= 4) {
          hh ^= static_cast<uint64_t>(w32(o)) * Q64_1;
          hh = rotl64(hh, 23) * Q64_2 + Q64_3;
          o += 4;
        }
        for (; o < total; ++o) {
          hh ^= (w32(o) & 0xffu) * Q64_5;
          hh = rotl64(hh, 11) * Q64_1;
        }
        hh ^= hh >> 33;
        hh *= Q64_2;
        hh ^= hh >> 29;
        hh *= Q64_3;
        hh ^= hh >> 32;
        h = static_cast<uint32_t>(hh);  // Lower32of64 (format.cc:576)
      } else {  // XXH32_finalize
        if (total >= 16) {
          h = rotl32(static_cast<uint32_t>(v0), 1) + rotl32(static_cast<uint32_t>(v1), 7) +
              rotl32(static_cast<uint32_t>(v2), 12) + rotl32(static_cast<uint32_t>(v3), 18);
        } else {
          h = Q32_5;
        }
        h += total;
        for (; total - o >= 4; o += 4) {
          h += w32(o) * Q32_3;
          h = rotl32(h, 17) * Q32_4;
        }
        for (; o < total; ++o) {
          h += (w32(o) & 0xffu) * Q32_5;
          h = rotl32(h, 11) * Q32_1;
        }
        h ^= h >> 15;
        h *= Q32_2;
        h ^= h >> 13;
        h *= Q32_3;
        h ^= h >> 16;
      }
      if (!valid) {
        if (a.out32) a.out32[i] = 0;
        if (MODE == kModeVerify) {
          if (a.ok_out) a.ok_out[i] = 0;
          if (a.stored_out) a.stored_out[i] = 0;
          if (a.mismatches) atomicAdd(a.mismatches, 1ull);
        }
      } else if (MODE == kModeRaw) {
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
          uint32_t slot = kTrlCap;
          if (FORST_LANE_TRL_STAGE && (i >> 32) == 0) slot = atomicAdd(&s_ntrl, 1u);
          if (slot < kTrlCap) {
            s_trl[slot] = TrlEntry{static_cast<uint32_t>(i), c};
          } else {  // (the staging area is full: stored here)
            uint8_t* wp = a.base_w + off + size;
            wp[0] = static_cast<uint8_t>(vb);
            stu32_bytes(wp + 1, c);
          }
        }
      }
      have = false;
    }
  }
  if (FORST_LANE_TRL_STAGE && MODE == kModeTrailer) {
    // the staged trailers, stored once every wave of the workgroup is done
    // (stores share vmcnt with the loads: inside the loop every later step
    // waited for them); the type byte is the caller's (last_bytes) or the
    // one already in memory
    __syncthreads();
    const uint32_t m = s_ntrl < kTrlCap ? s_ntrl : kTrlCap;
    for (uint32_t j = threadIdx.x; j < m; j += kLThreads) {
      const TrlEntry e = s_trl[j];
      uint8_t* wp = a.base_w + a.offsets[e.i] + a.sizes[e.i];
      if (a.last_bytes) wp[0] = a.last_bytes[e.i];
      stu32_bytes(wp + 1, e.c);
    }
  }
}

#ifndef FORST_LEGACY_LANE
#define FORST_LEGACY_LANE 1
#endif

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

template <bool X64>
hipError_t launch_lane(int mode, const BlockArgs& a, hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  const uint64_t batches = (a.n + 63) / 64;
  const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(
      1, std::min<uint64_t>((batches + kLWaves - 1) / kLWaves,
                            uint64_t(di.num_cus) * FORST_LANE_WG_PER_CU)));
  BlockArgs b = a;
  void* t = nullptr;
  hipError_t e = scratch_alloc(&t, 256, stream);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(t, 0, 8, stream)) != hipSuccess) {
    (void)scratch_free(t, stream);
    return e;
  }
  b.ticket = static_cast<unsigned long long*>(t);
  switch (mode) {
    case kModeCompute:
      *name = X64 ? "xxhash64_lane_kernel<compute>" : "xxhash32_lane_kernel<compute>";
      hipLaunchKernelGGL((xxhash_lane_kernel<kModeCompute, X64>), dim3(grid), dim3(kLThreads), 0,
                         stream, b);
      break;
    case kModeTrailer:
      *name = X64 ? "xxhash64_lane_kernel<trailer>" : "xxhash32_lane_kernel<trailer>";
      hipLaunchKernelGGL((xxhash_lane_kernel<kModeTrailer, X64>), dim3(grid), dim3(kLThreads), 0,
                         stream, b);
      break;
    case kModeVerify:
      *name = X64 ? "xxhash64_lane_kernel<verify>" : "xxhash32_lane_kernel<verify>";
      hipLaunchKernelGGL((xxhash_lane_kernel<kModeVerify, X64>), dim3(grid), dim3(kLThreads), 0,
                         stream, b);
      break;
    default:
      *name = X64 ? "xxhash64_lane_kernel<raw>" : "xxhash32_lane_kernel<raw>";
      hipLaunchKernelGGL((xxhash_lane_kernel<kModeRaw, X64>), dim3(grid), dim3(kLThreads), 0,
                         stream, b);
      break;
  }
  e = hipGetLastError();
  const hipError_t f = scratch_free(t, stream);
  return e != hipSuccess ? e : f;
}

hipError_t launch_xxhash_legacy_blocks(bool x64, int mode, const BlockArgs& a,
                                       hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  // (the lane kernel's realignment loads read the 4 bytes in front of an
  // unaligned block start: buffers shorter than 4 KiB keep the group kernel)
  if (FORST_LEGACY_LANE && a.base_len >= 4096)
    return x64 ? launch_lane<true>(mode, a, stream, name) : launch_lane<false>(mode, a, stream, name);
  const uint64_t per_wg = uint64_t(kWaves) * kMsgsPerWave;
  const uint32_t grid = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>((a.n + per_wg - 1) / per_wg,
                                               uint64_t(di.num_cus) * 16)));
  return x64 ? launch_mode<true>(mode, a, stream, grid, name)
             : launch_mode<false>(mode, a, stream, grid, name);
}

}  // namespace forst
