// forst_amd/csrc/crc32c.hip -- CRC32C block kernels for gfx950 (CDNA4).
//
// Replaces, per block, util/crc32c.cc:1133 crc32c::Extend (SSE4.2 crc32c_3way
// on the reference's x86 path) with one 64-lane wavefront per block.
//
// Algorithm (no carry-less multiply exists on CDNA4, so CRC is table driven):
//  * A block's message is covered by R rounds of 4 KiB ending at a dword
//    boundary W_end <= end; lane l owns the 64-byte segment [64l, 64l+64) of
//    each round (4 x global_load_dwordx4 per lane).  Bytes in front of the
//    message inside round 0 are garbage: the lane holding the first message
//    dword resets its state there (injecting ~init, crc32c::Extend's
//    pre-inversion) and lanes entirely in front zero their state.
//  * Each lane runs a slicing-by-4 CRC over its segment with four 256-entry
//    tables replicated 32x in LDS (entry e of copy c at dword 32e + c, lane
//    l reads copy l&31) so every ds_read_b32 is bank-conflict free.
//  * Between rounds a lane jumps over the 4032 bytes owned by the other lanes
//    with one 4-lookup GF(2) shift (x^(8*4032) mod P).
//  * 6-level xor-butterfly over the wave combines the 64 lane states with
//    shifts x^(8*64*2^k) (the algebra of crc32c::Crc32cCombine,
//    util/crc32c.cc:1279); the <= 7 tail bytes after W_end (+ the block's
//    compression-type byte on the write side) are appended byte-wise.
// The combine constants are block-size independent, so mixed 4/16/64 KiB
// batches run in one launch.  See DESIGN.md for the roofline analysis.
#include <cstdlib>
#include <string>

#include "crc32c_tables.h"
#include "device_common.h"
#include "engine.h"

namespace forst {
namespace {

constexpr uint32_t kRB = FORST_CRC_ROUND_BYTES;  // bytes per wave-round
constexpr uint32_t kWaves = 16;                  // waves per workgroup
constexpr uint32_t kThreads = kWaves * 64;
constexpr uint32_t kRep = 32;                     // table replication
constexpr uint32_t kOffJump = 4 * 256 * kRep;     // dword offsets in LDS
constexpr uint32_t kOffTree = kOffJump + 1024;
constexpr uint32_t kLdsDwords = kOffTree + FORST_CRC_TREE_LEVELS * 1024;
constexpr uint32_t kSmall = 32;  // shorter messages take the byte-serial path

static_assert(kLdsDwords * 4 <= 160 * 1024, "CRC tables must fit in LDS");

__device__ __forceinline__ uint32_t lds_at(const uint32_t* __restrict__ L,
                                           uint32_t byte_addr) {
  return L[byte_addr >> 2];
}

// slicing-by-4 step on the replicated tables: G(v) = v * x^32 mod P
__device__ __forceinline__ uint32_t crc_g(const uint32_t* __restrict__ L,
                                          uint32_t lb, uint32_t v) {
  const uint32_t a0 = ((v & 0xffu) << 7) + lb;
  const uint32_t a1 = (((v >> 8) & 0xffu) << 7) + lb;
  const uint32_t a2 = (((v >> 16) & 0xffu) << 7) + lb;
  const uint32_t a3 = ((v >> 24) << 7) + lb;
  return L[(a0 >> 2)] ^ L[(a1 >> 2) + 8192] ^ L[(a2 >> 2) + 16384] ^
         L[(a3 >> 2) + 24576];
}

// byte-at-a-time step (table G[3] is the Sarwate table)
__device__ __forceinline__ uint32_t crc_byte(const uint32_t* __restrict__ L,
                                             uint32_t lb, uint32_t s,
                                             uint32_t byte) {
  const uint32_t a = (((s ^ byte) & 0xffu) << 7) + lb;
  return L[(a >> 2) + 24576] ^ (s >> 8);
}

// linear shift x^(8n) through an unreplicated 4x256 table at dword T
__device__ __forceinline__ uint32_t crc_shift(const uint32_t* __restrict__ L,
                                              uint32_t T, uint32_t v) {
  return L[T + (v & 0xffu)] ^ L[T + 256 + ((v >> 8) & 0xffu)] ^
         L[T + 512 + ((v >> 16) & 0xffu)] ^ L[T + 768 + (v >> 24)];
}

__device__ __forceinline__ void load_seg(uint32_t (&w)[16],
                                         const uint8_t* seg) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32x4a4 v = ld16_a4(seg + 16 * k);
    w[4 * k + 0] = v.x;
    w[4 * k + 1] = v.y;
    w[4 * k + 2] = v.z;
    w[4 * k + 3] = v.w;
  }
}

// Round-0 load for windows that start before the caller's buffer: never
// touch a dword below `lo` (those lanes' data is garbage anyway).
__device__ __forceinline__ void load_seg_checked(uint32_t (&w)[16],
                                                 const uint8_t* seg,
                                                 uint64_t lo) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint8_t* c = seg + 16 * k;
    const uint64_t ca = reinterpret_cast<uint64_t>(c);
    if (ca >= lo) {
      const u32x4a4 v = ld16_a4(c);
      w[4 * k + 0] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    } else {
#pragma unroll
      for (int d = 0; d < 4; ++d)
        w[4 * k + d] = (ca + 4 * d >= lo) ? ld4_a4(c + 4 * d) : 0u;
    }
  }
}

// crc32c::Extend(init, p, len), then extended by `nextra` (0/1) extra byte.
// All arguments are wave-uniform; every lane returns the result.  Bytes in
// [lo, p) may be read (and ignored); nothing outside [lo, p+len) is touched.
__device__ __forceinline__ uint32_t wave_crc32c(const uint32_t* __restrict__ L,
                                                uint32_t lane,
                                uint32_t lb, const uint8_t* p, uint64_t len,
                                uint32_t init, uint32_t nextra, uint32_t extra,
                                uint64_t lo) {
  uint32_t s;
  if (len < kSmall) {
    s = ~init;
    for (uint32_t i = 0; i < static_cast<uint32_t>(len); ++i)
      s = crc_byte(L, lb, s, ldu8(p + i));
  } else {
    const uint64_t A = reinterpret_cast<uint64_t>(p);
    const uint64_t E = A + len;
    const uint64_t Aal = A & ~3ull;
    const uint32_t m = static_cast<uint32_t>(A & 3);
    uint64_t Wend = E & ~3ull;
    const uint64_t D = Wend - Aal;
    uint32_t R = static_cast<uint32_t>((D + kRB - 1) / kRB);
    if (R > 1 && (D % kRB) == 4) {  // spill 4 bytes into the tail, save a round
      Wend -= 4;
      --R;
    }
    const uint64_t Wstart = Wend - static_cast<uint64_t>(R) * kRB;
    const uint32_t hA = static_cast<uint32_t>(Aal - Wstart);
    const uint32_t LA = hA >> 6;
    const uint32_t jA = (hA >> 2) & 15u;
    // pointer arithmetic from p keeps the global address space (no flat ops)
    const uint8_t* seg = p - static_cast<int64_t>(A - Wstart) + lane * 64;

    // ---- round 0: contains the head of the message ----
    uint32_t w[16];
    if (Wstart >= lo)
      load_seg(w, seg);
    else
      load_seg_checked(w, seg, lo);
    s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (static_cast<uint32_t>(j) == jA) {
        if (m == 0) {
          const uint32_t s0 = (lane == LA) ? ~init : s;
          s = crc_g(L, lb, s0 ^ w[j]);
        } else {
          const uint32_t sn = crc_g(L, lb, s ^ w[j]);
          uint32_t sb = ~init;
          uint32_t wb = w[j] >> (8 * m);
          for (uint32_t b = m; b < 4; ++b) {
            sb = crc_byte(L, lb, sb, wb & 0xffu);
            wb >>= 8;
          }
          s = (lane == LA) ? sb : sn;
        }
      } else {
        s = crc_g(L, lb, s ^ w[j]);
      }
    }
    s = (lane < LA) ? 0u : s;

    // ---- rounds 1..R-1: plain streaming ----
    for (uint32_t r = 1; r < R; ++r) {
      seg += kRB;
      load_seg(w, seg);
      s = crc_shift(L, kOffJump, s);
#pragma unroll
      for (int j = 0; j < 16; ++j) s = crc_g(L, lb, s ^ w[j]);
    }

    // ---- combine the 64 lane states (xor butterfly, all lanes end equal) --
#pragma unroll
    for (int k = 0; k < FORST_CRC_TREE_LEVELS; ++k) {
      const uint32_t other = __shfl_xor(s, 1 << k);
      const bool right = (lane >> k) & 1;
      const uint32_t left_v = right ? other : s;
      const uint32_t right_v = right ? s : other;
      s = crc_shift(L, kOffTree + 1024u * k, left_v) ^ right_v;
    }

    // ---- tail bytes [Wend, E) ----
    const uint8_t* t = p + (Wend - A);
    const uint32_t nt = static_cast<uint32_t>(E - Wend);
    for (uint32_t i = 0; i < nt; ++i) s = crc_byte(L, lb, s, ldu8(t + i));
  }
  if (nextra) s = crc_byte(L, lb, s, extra);
  return ~s;
}

__device__ __forceinline__ void fill_tables(uint32_t* L) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 4 * 256 * kRep; i += kThreads) L[i] = kCrcG[i >> 5];
  for (uint32_t i = tid; i < 1024; i += kThreads) L[kOffJump + i] = kCrcJump[i];
  for (uint32_t i = tid; i < FORST_CRC_TREE_LEVELS * 1024; i += kThreads)
    L[kOffTree + i] = kCrcTree[i];
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Pipelined block kernel: a wave walks its blocks as a stream of (block,
// round) items and issues the global loads of the NEXT item (next round of
// the same block, or round 0 of its next block, plus that block's tail and
// trailer words) before it runs the LDS-table CRC of the current item, so
// every wave keeps ~4 KiB in flight while it computes.
// ---------------------------------------------------------------------------
struct CrcJob {
  uint64_t i;         // descriptor index (>= n: no job)
  const uint8_t* p;   // message start
  const uint8_t* seg; // this lane's round-0 segment
  uint32_t R;         // rounds; 0 => short message (byte-serial path)
  uint32_t len;       // message length (short path)
  uint32_t LA, jA, m; // head lane / head dword / head misalignment
  uint32_t nt;        // tail bytes after the last round
  uint32_t tail0, tail1;
  uint32_t extra, nextra;
  uint32_t init;
  uint32_t stored;    // verify: trailer value (context not yet removed)
  uint32_t mod;
  uint32_t last;      // compute/trailer: compression type byte
  bool valid;         // descriptor inside the buffer
  bool safe;          // round-0 window inside the buffer
};

template <int MODE>
__device__ __forceinline__ CrcJob crc_job_setup(const BlockArgs& a, uint64_t i,
                                                uint32_t lane) {
  CrcJob j;
  j.i = i;
  j.R = 0;
  j.len = 0;
  j.valid = false;
  j.safe = true;
  j.LA = j.jA = j.m = j.nt = 0;
  j.tail0 = j.tail1 = 0;
  j.extra = 0;
  j.nextra = 0;
  j.init = 0;
  j.stored = 0;
  j.mod = 0;
  j.last = 0;
  j.p = a.base;
  j.seg = a.base;
  if (i >= a.n) return j;
  const uint64_t off = a.offsets[i];
  const uint32_t size = a.sizes[i];
  uint64_t need = size;
  if (MODE == kModeVerify || MODE == kModeTrailer) need += 5;
  if (MODE == kModeCompute && a.last_bytes == nullptr) need += 1;
  j.valid = off <= a.base_len && need <= a.base_len - off;
  if (!j.valid) return j;
  const uint8_t* p = a.base + off;
  j.p = p;
  j.mod = a.modifiers ? a.modifiers[i] : 0u;
  uint64_t len = size;
  if (MODE == kModeVerify) {
    len = uint64_t(size) + 1;  // reader_common.cc:36 (type byte is checksummed)
    j.stored = ldu32(p + size + 1);
  } else if (MODE == kModeRaw) {
    j.init = a.init_crcs ? a.init_crcs[i] : 0u;
  } else {
    j.last = a.last_bytes ? a.last_bytes[i] : ldu8(p + size);
    j.extra = j.last;
    j.nextra = 1;
  }
  j.len = static_cast<uint32_t>(len);
  if (len < kSmall) return j;  // R = 0
  const uint64_t A = reinterpret_cast<uint64_t>(p);
  const uint64_t E = A + len;
  const uint64_t Aal = A & ~3ull;
  j.m = static_cast<uint32_t>(A & 3);
  uint64_t Wend = E & ~3ull;
  const uint64_t D = Wend - Aal;
  uint32_t R = static_cast<uint32_t>((D + kRB - 1) / kRB);
  if (R > 1 && (D % kRB) == 4) {
    Wend -= 4;
    --R;
  }
  const uint64_t Wstart = Wend - static_cast<uint64_t>(R) * kRB;
  const uint32_t hA = static_cast<uint32_t>(Aal - Wstart);
  j.R = R;
  j.LA = hA >> 6;
  j.jA = (hA >> 2) & 15u;
  j.safe = Wstart >= reinterpret_cast<uint64_t>(a.base);
  j.seg = p - static_cast<int64_t>(A - Wstart) + lane * 64;
  j.nt = static_cast<uint32_t>(E - Wend);
  const uint8_t* t = p + (Wend - A);
  if (j.nt > 0) j.tail0 = ld4v(t);
  if (j.nt > 4) j.tail1 = ld4v(t + 4);
  return j;
}

template <int MODE>
__device__ __forceinline__ void crc_job_finish(const BlockArgs& a, const CrcJob& j,
                                               uint32_t lane, uint32_t crc) {
  if (lane != 0) return;
  if (!j.valid) {
    if (a.out32) a.out32[j.i] = 0;
    if (MODE == kModeVerify) {
      if (a.ok_out) a.ok_out[j.i] = 0;
      if (a.stored_out) a.stored_out[j.i] = 0;
      if (a.mismatches) atomicAdd(a.mismatches, 1ull);
    }
    return;
  }
  if (MODE == kModeRaw) {
    a.out32[j.i] = crc;
  } else if (MODE == kModeVerify) {
    const uint32_t computed = crc_mask(crc);
    const uint32_t stored = j.stored - j.mod;
    const bool ok = stored == computed;
    if (a.out32) a.out32[j.i] = computed;
    if (a.stored_out) a.stored_out[j.i] = stored;
    if (a.ok_out) a.ok_out[j.i] = ok ? 1 : 0;
    if (!ok && a.mismatches) atomicAdd(a.mismatches, 1ull);
  } else {
    const uint32_t c = crc_mask(crc) + j.mod;
    if (a.out32) a.out32[j.i] = c;
    if (MODE == kModeTrailer) {
      uint8_t* q = a.base_w + (j.p - a.base) + (j.len);
      q[0] = static_cast<uint8_t>(j.last);
      stu32_bytes(q + 1, c);
    }
  }
}

// byte-serial CRC of a short message (len < kSmall)
__device__ __forceinline__ uint32_t crc_short(const uint32_t* __restrict__ L, uint32_t lb,
                                              const CrcJob& j) {
  uint32_t s = ~j.init;
  for (uint32_t k = 0; k < j.len; ++k) s = crc_byte(L, lb, s, ldu8(j.p + k));
  if (j.nextra) s = crc_byte(L, lb, s, j.extra);
  return ~s;
}

// load the segment of item (job, round r) into w
__device__ __forceinline__ void crc_job_load(uint32_t (&w)[16], const CrcJob& j, uint32_t r,
                                             uint64_t lo) {
  if (j.R == 0) return;
  const uint8_t* seg = j.seg + static_cast<uint64_t>(r) * kRB;
  if (r == 0 && !j.safe)
    load_seg_checked(w, seg, lo);
  else
    load_seg(w, seg);
}

// round r of job j on data w; returns the lane state
__device__ __forceinline__ uint32_t crc_job_round(const uint32_t* __restrict__ L, uint32_t lb,
                                                  uint32_t lane, const CrcJob& j, uint32_t r,
                                                  uint32_t s, const uint32_t (&w)[16]) {
  if (r == 0) {
    s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (static_cast<uint32_t>(k) == j.jA) {
        if (j.m == 0) {
          const uint32_t s0 = (lane == j.LA) ? ~j.init : s;
          s = crc_g(L, lb, s0 ^ w[k]);
        } else {
          const uint32_t sn = crc_g(L, lb, s ^ w[k]);
          uint32_t sb = ~j.init;
          uint32_t wb = w[k] >> (8 * j.m);
          for (uint32_t b = j.m; b < 4; ++b) {
            sb = crc_byte(L, lb, sb, wb & 0xffu);
            wb >>= 8;
          }
          s = (lane == j.LA) ? sb : sn;
        }
      } else {
        s = crc_g(L, lb, s ^ w[k]);
      }
    }
    s = (lane < j.LA) ? 0u : s;
  } else {
    s = crc_shift(L, kOffJump, s);
#pragma unroll
    for (int k = 0; k < 16; ++k) s = crc_g(L, lb, s ^ w[k]);
  }
  return s;
}

// 64-lane combine + tail + extra byte; every lane returns the finalized CRC
__device__ __forceinline__ uint32_t crc_job_combine(const uint32_t* __restrict__ L, uint32_t lb,
                                                    uint32_t lane, const CrcJob& j, uint32_t s) {
#pragma unroll
  for (int k = 0; k < FORST_CRC_TREE_LEVELS; ++k) {
    const uint32_t other = __shfl_xor(s, 1 << k);
    const bool right = (lane >> k) & 1;
    const uint32_t left_v = right ? other : s;
    const uint32_t right_v = right ? s : other;
    s = crc_shift(L, kOffTree + 1024u * k, left_v) ^ right_v;
  }
  uint32_t t = j.tail0;
  for (uint32_t k = 0; k < j.nt; ++k) {
    if (k == 4) t = j.tail1;
    s = crc_byte(L, lb, s, t & 0xffu);
    t >>= 8;
  }
  if (j.nextra) s = crc_byte(L, lb, s, j.extra);
  return ~s;
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) crc32c_block_kernel(BlockArgs a) {
  __shared__ uint32_t L[kLdsDwords];
  fill_tables(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t lb = (lane & 31) << 2;
  const uint64_t lo = reinterpret_cast<uint64_t>(a.base);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;

  CrcJob cur = crc_job_setup<MODE>(a, static_cast<uint64_t>(blockIdx.x) * kWaves + wave, lane);
  uint32_t wA[16], wB[16];
  crc_job_load(wA, cur, 0, lo);
  uint32_t r = 0, s = 0;

  // one pipeline step: compute (cur, r) on `wc` while item after it is loaded into `wn`
  auto step = [&](uint32_t (&wc)[16], uint32_t (&wn)[16]) {
    const bool same = cur.valid && cur.R > 0 && r + 1 < cur.R;
    CrcJob nxt = cur;
    if (same) {
      crc_job_load(wn, cur, r + 1, lo);
    } else {
      nxt = crc_job_setup<MODE>(a, cur.i + nw, lane);
      crc_job_load(wn, nxt, 0, lo);
    }
    if (!cur.valid) {
      crc_job_finish<MODE>(a, cur, lane, 0);
    } else if (cur.R == 0) {
      crc_job_finish<MODE>(a, cur, lane, crc_short(L, lb, cur));
    } else {
      s = crc_job_round(L, lb, lane, cur, r, s, wc);
      if (!same) crc_job_finish<MODE>(a, cur, lane, crc_job_combine(L, lb, lane, cur, s));
    }
    if (same) {
      ++r;
    } else {
      cur = nxt;
      r = 0;
    }
  };
  while (cur.i < a.n) {
    step(wA, wB);
    if (cur.i >= a.n) break;
    step(wB, wA);
  }
}

template <int MODE>
__global__ void __launch_bounds__(kThreads)
    crc32c_block_kernel_simple(BlockArgs a) {
  __shared__ uint32_t L[kLdsDwords];
  fill_tables(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t lb = (lane & 31) << 2;
  const uint64_t lo = reinterpret_cast<uint64_t>(a.base);
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
    if (!inb) {  // descriptor outside the buffer: report, never read
      if (lane == 0) {
        if (a.out32) a.out32[i] = 0;
        if (MODE == kModeVerify) {
          if (a.ok_out) a.ok_out[i] = 0;
          if (a.stored_out) a.stored_out[i] = 0;
          if (a.mismatches) atomicAdd(a.mismatches, 1ull);
        }
      }
      continue;
    }
    if (MODE == kModeRaw) {
      const uint32_t init = a.init_crcs ? a.init_crcs[i] : 0u;
      const uint32_t c = wave_crc32c(L, lane, lb, p, size, init, 0, 0, lo);
      if (lane == 0) a.out32[i] = c;
    } else if (MODE == kModeVerify) {
      // reader_common.cc:36-47
      const uint32_t computed =
          crc_mask(wave_crc32c(L, lane, lb, p, uint64_t(size) + 1, 0, 0, 0, lo));
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
      // format.cc:594-600 + builder.cc:1340-1345
      const uint32_t last = a.last_bytes ? a.last_bytes[i] : ldu8(p + size);
      const uint32_t mod = a.modifiers ? a.modifiers[i] : 0u;
      const uint32_t c =
          crc_mask(wave_crc32c(L, lane, lb, p, size, 0, 1, last, lo)) + mod;
      if (lane == 0) {
        if (a.out32) a.out32[i] = c;
        if (MODE == kModeTrailer) {
          uint8_t* q = a.base_w + off + size;
          q[0] = static_cast<uint8_t>(last);
          stu32_bytes(q + 1, c);
        }
      }
    }
  }
}

}  // namespace

hipError_t launch_crc32c_blocks(int mode, const BlockArgs& a,
                                hipStream_t stream, const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  uint32_t grid = static_cast<uint32_t>(
      std::min<uint64_t>((a.n + kWaves - 1) / kWaves, di.num_cus));
  if (grid == 0) grid = 1;
#ifdef FORST_DEBUG_BOUNDS
  {
    DbgState st{};
    st.lo = reinterpret_cast<uint64_t>(a.base);
    st.hi = st.lo + a.base_len;
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_forst_dbg), &st, sizeof(st), 0,
                                          hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
  }
#endif
  // FORST_CRC_VARIANT=simple selects the unpipelined kernel (A/B reference)
  const char* variant = std::getenv("FORST_CRC_VARIANT");
  const bool simple = variant && std::string(variant) == "simple";
#define FORST_LAUNCH_CRC(M, TAG)                                                         \
  do {                                                                                   \
    if (simple) {                                                                        \
      *name = "crc32c_block_kernel_simple<" TAG ">";                                     \
      hipLaunchKernelGGL(crc32c_block_kernel_simple<M>, dim3(grid), dim3(kThreads), 0,   \
                         stream, a);                                                     \
    } else {                                                                             \
      *name = "crc32c_block_kernel<" TAG ">";                                            \
      hipLaunchKernelGGL(crc32c_block_kernel<M>, dim3(grid), dim3(kThreads), 0, stream,  \
                         a);                                                             \
    }                                                                                    \
  } while (0)
  switch (mode) {
    case kModeCompute:
      FORST_LAUNCH_CRC(kModeCompute, "compute");
      break;
    case kModeTrailer:
      FORST_LAUNCH_CRC(kModeTrailer, "trailer");
      break;
    case kModeVerify:
      FORST_LAUNCH_CRC(kModeVerify, "verify");
      break;
    default:
      FORST_LAUNCH_CRC(kModeRaw, "raw");
      break;
  }
#undef FORST_LAUNCH_CRC
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// WAL (db/log_reader.cc:450-531, db/log_writer.cc:228-263)
// ---------------------------------------------------------------------------
namespace {

constexpr uint32_t kLogBlock = 32768;  // db/log_format.h:45
constexpr uint32_t kLogHdr = 7;        // db/log_format.h:48
constexpr uint32_t kLogRHdr = 11;      // db/log_format.h:52

__device__ __forceinline__ bool is_recyclable_type(uint32_t t) {
  return (t >= 5 && t <= 8) || t == 11;
}

// One wave per 32 KiB log block; headers are walked serially (their
// positions depend on the previous length), each record's CRC is a
// wave-parallel crc32c over header[6 .. hdr+len).
__global__ void __launch_bounds__(kThreads) wal_verify_kernel(WalArgs a) {
  __shared__ uint32_t L[kLdsDwords];
  fill_tables(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t lb = (lane & 31) << 2;
  const uint64_t lo = reinterpret_cast<uint64_t>(a.log);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  for (uint64_t bi = static_cast<uint64_t>(blockIdx.x) * kWaves + wave;
       bi < a.n_blocks; bi += nw) {
    const uint64_t b = a.first_block + bi;
    const uint64_t start = b * kLogBlock;
    uint64_t end = start + kLogBlock;
    if (end > a.log_len) end = a.log_len;
    uint32_t status = 0, nrec = 0;
    uint64_t pos = start;
    while (start < end && end - pos >= kLogHdr) {
      const uint8_t* h = a.log + pos;
      const uint32_t hdr_lo = ldu32(h + 3);  // bytes 3..6
      const uint32_t length = (hdr_lo >> 8) & 0xffffu;
      const uint32_t type = hdr_lo >> 24;
      const bool recyc = is_recyclable_type(type);
      const uint32_t hs = recyc ? kLogRHdr : kLogHdr;
      if (end - pos < hs) break;  // truncated header at EOF (ReadMore)
      if (hs + length > end - pos) {
        status = 2;  // kBadRecordLen
        break;
      }
      if (recyc && ldu32(h + 7) != a.log_number) {
        status = 4;  // kOldRecord
        break;
      }
      if (type == 0 && length == 0) {
        status = 3;  // kZeroType: preallocated space, rest of block skipped
        break;
      }
      const uint32_t expected = crc_unmask(ldu32(h));
      const uint32_t actual =
          wave_crc32c(L, lane, lb, h + 6, length + hs - 6, 0, 0, 0, lo);
      if (actual != expected) {
        status = 1;  // kBadRecordChecksum: rest of block dropped
        break;
      }
      ++nrec;
      pos += hs + length;
    }
    if (lane == 0) {
      if (a.status_out) a.status_out[bi] = static_cast<uint8_t>(status);
      if (a.nrec_out) a.nrec_out[bi] = nrec;
      if (a.fail_off_out) a.fail_off_out[bi] = static_cast<uint32_t>(pos - start);
      if (a.bad_blocks && status != 0 && status != 3) atomicAdd(a.bad_blocks, 1ull);
    }
  }
}

// EmitPhysicalRecord's CRC == Mask(Value(header[6 .. hs) || payload)).
__global__ void __launch_bounds__(kThreads) wal_record_crc_kernel(WalArgs a) {
  __shared__ uint32_t L[kLdsDwords];
  fill_tables(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t lb = (lane & 31) << 2;
  const uint64_t lo = reinterpret_cast<uint64_t>(a.log);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kWaves + wave;
       i < a.n_records; i += nw) {
    const uint64_t off = a.header_offsets[i];
    uint32_t c = 0;
    bool inb = off <= a.log_len && a.log_len - off >= kLogHdr;
    uint32_t length = 0, hs = kLogHdr;
    if (inb) {
      const uint8_t* h = a.log + off;
      const uint32_t hdr_lo = ldu32(h + 3);
      length = (hdr_lo >> 8) & 0xffffu;
      hs = is_recyclable_type(hdr_lo >> 24) ? kLogRHdr : kLogHdr;
      inb = a.log_len - off >= uint64_t(hs) + length;
    }
    if (inb) {
      const uint8_t* h = a.log + off;
      c = crc_mask(wave_crc32c(L, lane, lb, h + 6, length + hs - 6, 0, 0, 0, lo));
      if (lane == 0 && a.write_in_place) stu32_bytes(a.log_w + off, c);
    }
    if (lane == 0 && a.crc_out) a.crc_out[i] = c;
  }
}

}  // namespace

hipError_t launch_wal_verify(const WalArgs& a, hipStream_t stream,
                             const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n_blocks == 0) return hipSuccess;
  uint32_t grid = static_cast<uint32_t>(
      std::min<uint64_t>((a.n_blocks + kWaves - 1) / kWaves, di.num_cus));
  *name = "wal_verify_kernel";
  hipLaunchKernelGGL(wal_verify_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_wal_record_crc(const WalArgs& a, hipStream_t stream,
                                 const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n_records == 0) return hipSuccess;
  uint32_t grid = static_cast<uint32_t>(
      std::min<uint64_t>((a.n_records + kWaves - 1) / kWaves, di.num_cus));
  *name = "wal_record_crc_kernel";
  hipLaunchKernelGGL(wal_record_crc_kernel, dim3(grid), dim3(kThreads), 0,
                     stream, a);
  return hipGetLastError();
}

}  // namespace forst

#ifdef FORST_DEBUG_BOUNDS
// diagnostics build only: first out-of-bounds access recorded by the CRC
// kernels since the last launch (line, offset from base, width, count)
extern "C" __attribute__((visibility("default"))) int forst_debug_fetch(unsigned long long* out) {
  forst::DbgState st{};
  if (hipMemcpyFromSymbol(&st, HIP_SYMBOL(forst::g_forst_dbg), sizeof(st)) != hipSuccess)
    return -3;
  for (int k = 0; k < 4; ++k) out[k] = st.rec[k];
  return 0;
}
#endif
