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
#include "stream_common.h"

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

#ifdef FORST_DIAG
// ---------------------------------------------------------------------------
// Streaming block kernel v1 (diagnostics build only: A/B reference of v2).
//
// Each wave owns a contiguous share [kbeg, kend) of the descriptors and walks
// it as a stream of (block, round) steps.  At the top of every step it issues
// the global loads of the NEXT step (next round of this block, or round 0 of
// the next block, plus that block's tail/trailer dwords), then runs the
// LDS-table CRC of the current step on the registers loaded one step earlier.
// Every load is unconditional and issued in straight-line code, so the
// compiler's s_waitcnt for the current step counts only the next step's loads
// (vmcnt(6)) and one round stays in flight per wave while it computes.  Block
// descriptors are fetched 64 at a time (lane j holds block kb+j; read with
// v_readlane into SGPRs) and results are kept in lane kk of result VGPRs and
// stored once per 64 blocks: no descriptor load or store sits between a
// prefetch and its use.
//
// Head of a message (round 0): the window [W0, Wend) ends at the last dword
// boundary Wend <= end.  Lanes wholly in front of the first message dword
// load the last window segment instead (any in-window address is safe) and
// zero their state; the lane LA holding the first message dword restarts its
// chain at dword jA with state S0 = ~init moved back over the m = A&3 bytes
// in front of the message (inverse Sarwate steps), those bytes masked to zero.
// Tail: the <= 3 bytes after Wend come from the tail dword, byte-wise.
// Blocks shorter than 64 bytes, blocks whose round-0 head lane would read in
// front of the buffer, and out-of-range descriptors take the wave_crc32c path.
// ---------------------------------------------------------------------------
constexpr uint32_t kOffTinv = kLdsDwords;  // 256-byte inverse of T3's top byte
constexpr uint32_t kLdsDwordsStream = kLdsDwords + 64;
static_assert(kLdsDwordsStream * 4 <= 160 * 1024, "stream kernel LDS");

__device__ __forceinline__ void fill_tinv(uint32_t* L) {
  // Sarwate table T = G[3]: the top byte of T[b] is a bijection of b
  uint8_t* inv = reinterpret_cast<uint8_t*>(L + kOffTinv);
  const uint32_t t = threadIdx.x;
  if (t < 256) inv[kCrcG[3 * 256 + t] >> 24] = static_cast<uint8_t>(t);
  __syncthreads();
}

// inverse of one zero-byte step s' = (s >> 8) ^ T[s & 255] (uniform value)
__device__ __forceinline__ uint32_t crc_unstep(const uint32_t* __restrict__ L, uint32_t lb,
                                               uint32_t sp) {
  const uint32_t top = sp >> 24;
  const uint32_t b = (L[kOffTinv + (top >> 2)] >> (8 * (top & 3))) & 0xffu;
  const uint32_t t = L[(((b << 7) + lb) >> 2) + 24576];
  return ((sp ^ t) << 8) | b;
}

// wave-uniform description of one block (lives in SGPRs)
struct Blk {
  uint64_t off;     // message start (offset from base)
  int64_t w0;       // round-0 window start offset (may be < 0 for slow blocks)
  uint64_t we;      // window end (dword boundary <= message end)
  uint64_t t0, t1;  // tail / trailer dword offsets (always loadable)
  uint32_t size, len, mod, extra;
  uint32_t R, LA, jA, nt, S0, bm;
  bool valid, slow;
};

template <int MODE>
__device__ __forceinline__ Blk blk_setup(const BlockArgs& a, const uint32_t* __restrict__ L,
                                         uint32_t lb, uint64_t k, uint64_t kend, uint64_t kb,
                                         const DescBatch& cb, const DescBatch& nb,
                                         const uint32_t (&kS0)[4]) {
  Blk b;
  const Desc d = batch_desc(k, kb, cb, nb);  // k may be >= kend (then invalid)
  b.off = d.off;
  b.size = d.size;
  b.mod = d.mod;
  b.extra = d.extra;

  const bool has_extra = (MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes;
  const bool mem_last = MODE == kModeVerify || ((MODE == kModeCompute || MODE == kModeTrailer) &&
                                                !a.last_bytes);
  b.valid = k < kend && desc_in_range<MODE>(a, d);
  (void)has_extra;
  b.len = b.size + (mem_last ? 1u : 0u);

  const uint64_t E = b.off + b.len;
  const uint64_t ws = b.off & ~3ull;
  b.we = E & ~3ull;
  const uint64_t d4 = b.we - ws;
  b.R = static_cast<uint32_t>((d4 + kRB - 1) / kRB);
  b.w0 = static_cast<int64_t>(b.we) - static_cast<int64_t>(b.R) * kRB;
  const uint32_t hA = static_cast<uint32_t>(static_cast<int64_t>(ws) - b.w0);
  b.LA = hA >> 6;
  b.jA = (hA >> 2) & 15u;
  b.nt = static_cast<uint32_t>(E - b.we);
  const uint32_t m = static_cast<uint32_t>(b.off & 3);
  b.bm = 0xffffffffu << (8 * m);
  b.slow = !b.valid || d4 < 64 || b.w0 + 64 * static_cast<int64_t>(b.LA) < 0;
  if (MODE == kModeRaw) {
    uint32_t s0 = ~b.extra;
    for (uint32_t q = 0; q < m; ++q) s0 = crc_unstep(L, lb, s0);
    b.S0 = s0;
  } else {
    b.S0 = m == 0 ? kS0[0] : m == 1 ? kS0[1] : m == 2 ? kS0[2] : kS0[3];
  }
  b.t0 = (b.nt > 0 || MODE == kModeVerify) ? b.we : b.we - 4;
  b.t1 = (MODE == kModeVerify && b.nt > 0) ? b.we + 4 : b.t0;
  if (b.slow) {  // loads of a slow block's step are dummies at the buffer start
    b.w0 = 0;
    b.we = 64;
    b.LA = 0;
    b.t0 = b.t1 = 0;
  }
  return b;
}

struct StepBuf {
  uint32_t w[16];
  uint32_t t0, t1;
};

__device__ __forceinline__ void issue_step(const uint8_t* __restrict__ base, uint32_t lane,
                                           int64_t w0, uint64_t we, uint32_t la, uint64_t t0,
                                           uint64_t t1, uint32_t r, StepBuf& b) {
  int64_t so = w0 + static_cast<int64_t>(r) * kRB + 64 * static_cast<int64_t>(lane);
  const uint32_t la0 = r == 0 ? la : 0u;
  so = lane < la0 ? static_cast<int64_t>(we) - 64 : so;
  const uint8_t* sp = base + so;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const u32x4a4 v = ld16_a4(sp + 16 * q);
    b.w[4 * q + 0] = v.x;
    b.w[4 * q + 1] = v.y;
    b.w[4 * q + 2] = v.z;
    b.w[4 * q + 3] = v.w;
  }
  b.t0 = ld4v(base + t0);
  b.t1 = ld4v(base + t1);
}

__device__ __forceinline__ uint32_t stream_round(const uint32_t* __restrict__ L, uint32_t lb,
                                                 uint32_t lane, const Blk& c, uint32_t r,
                                                 uint32_t s, const uint32_t (&w)[16]) {
  if (r == 0) {
    s = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      uint32_t x = s ^ w[q];
      if (static_cast<uint32_t>(q) == c.jA) {
        const uint32_t head = (w[q] & c.bm) ^ c.S0;
        x = lane == c.LA ? head : x;
      }
      s = crc_g(L, lb, x);
    }
    s = lane < c.LA ? 0u : s;
  } else {
    s = crc_shift(L, kOffJump, s);
#pragma unroll
    for (int q = 0; q < 16; ++q) s = crc_g(L, lb, s ^ w[q]);
  }
  return s;
}

template <int K>
__device__ __forceinline__ uint32_t tree_level(const uint32_t* __restrict__ L, uint32_t lane,
                                               uint32_t s) {
  const uint32_t other = static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(s), 0x110 + (1 << K), 0xf, 0xf, false));
  constexpr uint32_t keep = (2u << K) - 1u;
  if ((lane & keep) == keep) s = crc_shift(L, kOffTree + 1024u * K, other) ^ s;
  return s;
}

// combine the 64 lane states of a block (lane l = bytes [64l, 64l+64) of each
// round, the last round ending at Wend), append the tail bytes and the extra
// byte; returns ~state (the crc32c::Extend value), wave-uniform.
__device__ __forceinline__ uint32_t stream_finish(const uint32_t* __restrict__ L, uint32_t lb,
                                                  uint32_t lane, const Blk& c, uint32_t s,
                                                  uint32_t t0, bool has_extra) {
  // levels 0..3 inside 16-lane rows: lane i (low k+1 bits set) takes lane
  // i-2^k (DPP row_shr) and shifts it over its own 2^k segments
  s = tree_level<0>(L, lane, s);
  s = tree_level<1>(L, lane, s);
  s = tree_level<2>(L, lane, s);
  s = tree_level<3>(L, lane, s);
  // levels 4..5 on the row results (wave-uniform: broadcast LDS reads)
  const uint32_t g0 = readlane32(s, 15);
  const uint32_t g1 = readlane32(s, 31);
  const uint32_t g2 = readlane32(s, 47);
  const uint32_t g3 = readlane32(s, 63);
  const uint32_t t01 = crc_shift(L, kOffTree + 1024u * 4, g0) ^ g1;
  const uint32_t t23 = crc_shift(L, kOffTree + 1024u * 4, g2) ^ g3;
  uint32_t st = crc_shift(L, kOffTree + 1024u * 5, t01) ^ t23;
  uint32_t t = t0;
  for (uint32_t q = 0; q < c.nt; ++q) {
    st = crc_byte(L, lb, st, t & 0xffu);
    t >>= 8;
  }
  if (has_extra) st = crc_byte(L, lb, st, c.extra);
  return ~st;
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) crc32c_stream_kernel(BlockArgs a) {
  __shared__ uint32_t L[kLdsDwordsStream];
  fill_tables(L);
  fill_tinv(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t lb = (lane & 31) << 2;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * kWaves + wave;
  uint64_t kbeg, kend;
  wave_share(a.n, nw, gw, kbeg, kend);
  if (kbeg >= kend) return;
  const bool has_extra = (MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes;

  // S0 for init = 0 (every block mode): ~0 moved back over m = 0..3 bytes
  uint32_t kS0[4];
  kS0[0] = 0xffffffffu;
#pragma unroll
  for (int m = 1; m < 4; ++m) kS0[m] = uniform(crc_unstep(L, lb, kS0[m - 1]));

  DescBatch cb, nb;
  uint64_t kb = kbeg;
  load_batch<MODE>(a, kb, kend, lane, cb);
  load_batch<MODE>(a, kb + kBatch, kend, lane, nb);
  uint64_t k = kbeg;
  Blk C = blk_setup<MODE>(a, L, lb, k, kend, kb, cb, nb, kS0);
  Blk N = blk_setup<MODE>(a, L, lb, k + 1, kend, kb, cb, nb, kS0);
  uint32_t rOut = 0, rSt = 0, rOk = 0;
  StepBuf X, Y;
  issue_step(a.base, lane, C.w0, C.we, C.LA, C.t0, C.t1, 0, X);
  uint32_t r = 0, s = 0;

  auto flush = [&](uint32_t cnt) {
    const uint64_t i = kb + lane;
    const bool mine = lane < cnt;
    if (mine && a.out32) a.out32[i] = rOut;
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

  // one step: issue (next) into nx, compute (C, r) from cu; false when done
  auto step = [&](StepBuf& cu, StepBuf& nx) -> bool {
    const bool last = C.slow || r + 1 >= C.R;
    issue_step(a.base, lane, last ? N.w0 : C.w0, last ? N.we : C.we, last ? N.LA : C.LA,
               last ? N.t0 : C.t0, last ? N.t1 : C.t1, last ? 0u : r + 1, nx);
    if (!C.slow) s = stream_round(L, lb, lane, C, r, s, cu.w);
    if (!last) {
      ++r;
      return true;
    }
    uint32_t crc = 0, stored = 0;
    if (!C.slow) {
      crc = stream_finish(L, lb, lane, C, s, cu.t0, has_extra);
      if (MODE == kModeVerify)
        stored = C.nt ? __builtin_amdgcn_alignbyte(cu.t1, cu.t0, C.nt) : cu.t0;
    } else if (C.valid) {
      const uint8_t* p = a.base + C.off;
      const uint32_t init = MODE == kModeRaw ? C.extra : 0u;
      crc = wave_crc32c(L, lane, lb, p, C.len, init, has_extra ? 1u : 0u, C.extra,
                        reinterpret_cast<uint64_t>(a.base));
      // retire() waits for the load INSIDE this branch: a pending load
      // merging into the fast path would make hipcc drain the prefetch
      // (s_waitcnt vmcnt(0)) at every block end.
      if (MODE == kModeVerify) stored = retire(ldu32(p + C.size + 1));
      crc = retire(crc);
    }
    uint32_t out, st = 0, ok = C.valid ? 1u : 0u;
    if (MODE == kModeRaw) {
      out = crc;
    } else if (MODE == kModeVerify) {
      const uint32_t computed = crc_mask(crc);  // reader_common.cc:36-47
      st = stored - C.mod;
      ok = (C.valid && st == computed) ? 1u : 0u;
      out = computed;
    } else {
      out = crc_mask(crc) + C.mod;  // format.cc:594-600 + builder.cc:1340-1345
    }
    if (!C.valid) {
      out = 0;
      st = 0;
    }
    const uint32_t kk = static_cast<uint32_t>(k - kb);
    rOut = lane == kk ? out : rOut;
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
    N = blk_setup<MODE>(a, L, lb, k + 1, kend, kb, cb, nb, kS0);
    r = 0;
    return true;
  };
  while (step(X, Y) && step(Y, X)) {
  }
}
#endif  // FORST_DIAG

// ---------------------------------------------------------------------------
// Streaming block kernel v2: two independent CRC chains per lane.
//
// The latency of the v1 kernel is a serial chain of 17 dependent LDS table
// steps per 4 KiB round (16 dwords + the hop) plus a 6-step combine tree per
// block.  v2 halves the chain: in every 4 KiB round, chain c (0, 1) of lane l
// owns the 32-byte segment [2048c + 32l, +32) -- 8 dwords -- so a lane runs
// two independent 8-step chains whose LDS latencies overlap.  The hop to the
// next round is fused with the first dword step (s' = J2(s) ^ G(w0), J2 = shift
// by 4096 - 32 + 4 bytes).  The finish is three table steps deep instead of a
// tree: every lane moves each chain state to the end of its 16-lane row with
// A[lo] (lo = 15 - (l & 15)), the rows are XOR-reduced with DPP (no tables),
// and the 8 row values (2 chains x 4 rows) are moved to the end of the round
// with B[hi] and XORed.  The <= 3 tail bytes and the block's type byte are
// folded in ONE slicing step of k <= 4 bytes.
//
// LDS (byte addresses; the only __shared__ object, at 0):
//   [0, 64K)       G and J2, replicated 8x and interleaved: row e (256 B) holds
//                  G_t[e] copy c at dword 8t + c and J2_t[e] copy c at dword
//                  32 + 8t + c (t = 0..3 table, c = 0..7 copy).  Lane l
//                  (c = l & 7, g = (l >> 3) & 3) does the i-th lookup of a
//                  step on table i ^ g with byte i ^ g, so the 32 lanes of a
//                  ds_read_b32 bank group hit dwords 8{0,1,2,3} + c: 32
//                  distinct banks, conflict free.  The address
//                  256 * byte + 4 (8 t + c) [+ 128 for J2] is ONE v_perm_b32 of
//                  the data word and a per-lane constant.
//   [64K, 124K)    A[1..15]: shift by 32 lo bytes (unreplicated, 4 KiB each)
//   [124K, 152K)   B[1..7]: shift by 512 hi bytes
// ---------------------------------------------------------------------------
constexpr uint32_t kOffA2 = 65536;
constexpr uint32_t kOffB2 = kOffA2 + 15 * 4096;
constexpr uint32_t kLds2Bytes = kOffB2 + 7 * 4096;
static_assert(kLds2Bytes <= 160 * 1024, "v2 tables must fit in LDS");
constexpr uint32_t kRB2 = FORST_CRC_ROUND_BYTES;
constexpr uint32_t kSeg2 = FORST_CRC2_SEG_BYTES;       // 32
constexpr uint32_t kChain2 = FORST_CRC2_CHAIN_BYTES;   // 2048
static_assert(kSeg2 * 16 * 8 == 2 * kChain2, "A/B tables assume 32-byte segments, 2 chains");

__device__ __forceinline__ uint32_t lds32(const uint8_t* __restrict__ Lb, uint32_t addr) {
  return *reinterpret_cast<const uint32_t*>(Lb + addr);
}

struct Lanes2 {
  uint32_t lpack;     // byte i: 4 (8 (i^g) + c)  (G; J2 is +128, folded into the ds_read offset)
  uint32_t sel[4];    // v_perm selector: addr = {0, 0, x.b(i^g), lpack.b(i)}
};

__device__ __forceinline__ Lanes2 lanes2(uint32_t lane) {
  Lanes2 k;
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
__device__ __forceinline__ uint32_t lane_c4(uint32_t lane) { return (lane & 7) << 2; }

// replicated 4-table linear map: G (J = false) or J2 (J = true)
template <bool J>
__device__ __forceinline__ uint32_t rep_map(const uint8_t* __restrict__ Lb, const Lanes2& k,
                                            uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    r ^= lds32(Lb, __builtin_amdgcn_perm(x, k.lpack, k.sel[i]) + (J ? 128u : 0u));
  return r;
}

// k-byte slicing step (k <= 4, wave-uniform): the state after bytes y_0..y_k-1
// (little-endian in y):  (s >> 8k) ^ XOR_j G[4-k+j][(s ^ y)_j]
__device__ __forceinline__ uint32_t step_k(const uint8_t* __restrict__ Lb, const Lanes2& kk,
                                           uint32_t s, uint32_t y, uint32_t k) {
  if (k == 0) return s;
  const uint32_t x = s ^ y;
  const uint32_t c4 = lane_c4(threadIdx.x);
  uint32_t r = k == 4 ? 0u : (s >> (8 * k));
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    if (j < k) {
      const uint32_t t = 4 - k + j;
      r ^= lds32(Lb, __builtin_amdgcn_perm(x, c4, 0x0c0c0000u | ((4 + j) << 8)) + 32 * t);
    }
  }
  return r;
}

// linear shift through an unreplicated 4 x 256 table at byte offset b
__device__ __forceinline__ uint32_t shift_at(const uint8_t* __restrict__ Lb, uint32_t b,
                                             uint32_t v) {
  return lds32(Lb, b + ((v & 0xffu) << 2)) ^ lds32(Lb, b + 1024 + (((v >> 8) & 0xffu) << 2)) ^
         lds32(Lb, b + 2048 + (((v >> 16) & 0xffu) << 2)) ^ lds32(Lb, b + 3072 + ((v >> 24) << 2));
}

__device__ __forceinline__ void fill_tables2(uint32_t* L) {
  const uint32_t tid = threadIdx.x;
  // row e, dword d: d < 32 -> G_{d>>3}[e], else J2_{(d-32)>>3}[e]
  for (uint32_t i = tid; i < 16384; i += kThreads) {
    const uint32_t e = i >> 6, d = i & 63, t = (d >> 3) & 3;
    L[i] = d < 32 ? kCrcG[t * 256 + e] : kCrcJ2[t * 256 + e];
  }
  for (uint32_t i = tid; i < 15 * 1024; i += kThreads) L[kOffA2 / 4 + i] = kCrcA[i];
  for (uint32_t i = tid; i < 7 * 1024; i += kThreads) L[kOffB2 / 4 + i] = kCrcB[i];
  __syncthreads();
}

// raw mode with a per-message init: S0 = ~init moved back over m bytes
__device__ __forceinline__ uint32_t unstep_m(uint32_t v, uint32_t m) {
  if (m == 0) return v;
  const uint32_t* col = kCrcUnstep + 32 * (m - 1);
  uint32_t r = 0;
  for (uint32_t i = 0; i < 32; ++i) r ^= ((v >> i) & 1u) ? col[i] : 0u;
  return r;
}

// wave-uniform description of one block, kept compact (three live copies
// sit in SGPRs): derived quantities are recomputed where they are used
struct Blk2 {
  uint64_t off;
  uint64_t we;  // window end: last dword boundary <= message end
  uint32_t size, mod, extra, R, S0;
  uint32_t pk;  // cA:1 | lA:6 | jA:3 | q:3 | nt:2 | valid:1 | slow:1 | m:2 | xtra:1
  __device__ __forceinline__ uint32_t cA() const { return pk & 1u; }
  __device__ __forceinline__ uint32_t lA() const { return (pk >> 1) & 63u; }
  __device__ __forceinline__ uint32_t jA() const { return (pk >> 7) & 7u; }
  __device__ __forceinline__ uint32_t q() const { return (pk >> 10) & 7u; }
  __device__ __forceinline__ uint32_t nt() const { return (pk >> 13) & 3u; }
  __device__ __forceinline__ bool valid() const { return (pk >> 15) & 1u; }
  __device__ __forceinline__ bool slow() const { return (pk >> 16) & 1u; }
  __device__ __forceinline__ uint32_t bm() const { return 0xffffffffu << (8 * ((pk >> 17) & 3u)); }
  __device__ __forceinline__ bool xtra() const { return (pk >> 19) & 1u; }
  // end of the round windows: the message's last dword boundary, one dword
  // earlier for an xtra block
  __device__ __forceinline__ uint64_t wend() const { return we - (xtra() ? 4u : 0u); }
  // round-0 window start (may be < 0)
  __device__ __forceinline__ int64_t w0() const {
    return static_cast<int64_t>(wend()) - static_cast<int64_t>(R) * kRB2;
  }
};

// Rounds of a window of d4 bytes (a dword multiple).  A window exactly one
// dword longer than whole rounds -- a quarter of back-to-back 4 KiB blocks:
// 4097 checksummed bytes starting at 3 mod 4 -- ends one dword early ("xtra");
// that dword is one slicing step in the finish instead of an almost empty
// round.  (Block modes only: raw messages of arbitrary lengths rarely hit it.)
template <int MODE, uint32_t RB>
__device__ __forceinline__ void window_rounds(uint64_t d4, uint32_t& R, bool& xtra) {
  xtra = MODE != kModeRaw && (d4 & (RB - 1)) == 4 && d4 > RB;
  R = static_cast<uint32_t>(xtra ? d4 / RB : (d4 + RB - 1) / RB);
}

template <int MODE>
__device__ __forceinline__ bool mem_last_byte(const BlockArgs& a) {
  return MODE == kModeVerify || ((MODE == kModeCompute || MODE == kModeTrailer) && !a.last_bytes);
}

// scalar setup (blocks of the NEXT descriptor batch: at most two per batch,
// reached by the look-ahead cursors before the batch becomes current)
template <int MODE>
__device__ __forceinline__ Blk2 blk2_setup_scalar(const BlockArgs& a, uint64_t k, uint64_t kend,
                                                  uint64_t kb, const DescBatch& cb,
                                                  const DescBatch& nb) {
  Blk2 b;
  const Desc d = batch_desc(k, kb, cb, nb);
  b.off = d.off;
  b.size = d.size;
  b.mod = d.mod;
  b.extra = d.extra;
  const bool valid = k < kend && desc_in_range<MODE>(a, d);
  const uint64_t E = b.off + b.size + (mem_last_byte<MODE>(a) ? 1u : 0u);
  const uint64_t ws = b.off & ~3ull;
  b.we = E & ~3ull;
  const uint64_t d4 = b.we - ws;
  bool xtra;
  window_rounds<MODE, kRB2>(d4, b.R, xtra);
  b.pk = xtra ? 1u << 19 : 0u;  // w0() below needs the flag
  const uint32_t hA = static_cast<uint32_t>(static_cast<int64_t>(ws) - b.w0());
  const uint32_t cA = hA >> 11, lA = (hA >> 5) & 63u, jA = (hA >> 2) & 7u;
  // head segment starting in front of the buffer (only blocks at offset < 28):
  // it is loaded from offset 0 and shifted up by q dwords in registers
  const int64_t seg_head = static_cast<int64_t>(ws) - 4 * static_cast<int64_t>(jA);
  const uint32_t q = seg_head < 0 ? static_cast<uint32_t>(-seg_head) >> 2 : 0u;
  const uint32_t nt = static_cast<uint32_t>(E - b.we);
  const uint32_t m = static_cast<uint32_t>(b.off & 3);
  const bool slow = !valid || d4 < 64;
  b.S0 = MODE == kModeRaw && a.init_crcs ? unstep_m(~b.extra, m) : kCrcS0[m];
  if (slow) {  // the slow path loads on its own; dummy step loads at [0, 4 KiB)
    b.we = kRB2;
    b.R = 1;
    b.pk = (nt << 13) | (valid ? 1u << 15 : 0u) | (1u << 16) | (m << 17);
  } else {
    b.pk = cA | (lA << 1) | (jA << 7) | (q << 10) | (nt << 13) | (valid ? 1u << 15 : 0u) |
           (m << 17) | (xtra ? 1u << 19 : 0u);
  }
  return b;
}

// Per-lane derived block fields of the CURRENT descriptor batch (lane j <->
// block kb + j), computed once per 64 blocks in vector code so that a block's
// setup is a few v_readlane instead of ~100 scalar instructions.
struct Derived2 {
  uint32_t pk, R, S0;  // S0 only in raw mode (per-message init)
};

template <int MODE>
__device__ __forceinline__ Derived2 derive2(const BlockArgs& a, const DescBatch& cb, uint64_t kb,
                                            uint64_t kend, uint32_t lane) {
  Derived2 d;
  const uint64_t off = (static_cast<uint64_t>(cb.off_hi) << 32) | cb.off_lo;
  const Desc ds{off, cb.size, cb.mod, cb.extra};
  const bool valid = kb + lane < kend && desc_in_range<MODE>(a, ds);
  const uint64_t E = off + cb.size + (mem_last_byte<MODE>(a) ? 1u : 0u);
  const uint64_t ws = off & ~3ull;
  const uint64_t we = E & ~3ull;
  const uint64_t d4 = we - ws;
  uint32_t R;
  bool xtra;
  window_rounds<MODE, kRB2>(d4, R, xtra);
  const int64_t w0 = static_cast<int64_t>(we) - (xtra ? 4 : 0) - static_cast<int64_t>(R) * kRB2;
  const uint32_t hA = static_cast<uint32_t>(static_cast<int64_t>(ws) - w0);
  const uint32_t cA = hA >> 11, lA = (hA >> 5) & 63u, jA = (hA >> 2) & 7u;
  const int64_t seg_head = static_cast<int64_t>(ws) - 4 * static_cast<int64_t>(jA);
  const uint32_t q = seg_head < 0 ? static_cast<uint32_t>(-seg_head) >> 2 : 0u;
  const uint32_t nt = static_cast<uint32_t>(E - we);
  const uint32_t m = static_cast<uint32_t>(off & 3);
  const bool slow = !valid || d4 < 64;
  d.R = slow ? 1u : R;
  d.pk = slow ? ((nt << 13) | (valid ? 1u << 15 : 0u) | (1u << 16) | (m << 17))
              : (cA | (lA << 1) | (jA << 7) | (q << 10) | (nt << 13) | (valid ? 1u << 15 : 0u) |
                 (m << 17) | (xtra ? 1u << 19 : 0u));
  d.S0 = MODE == kModeRaw ? (a.init_crcs ? unstep_m(~cb.extra, m) : kCrcS0[m]) : 0u;
  return d;
}

template <int MODE>
__device__ __forceinline__ Blk2 blk2_setup(const BlockArgs& a, uint64_t k, uint64_t kend,
                                           uint64_t kb, const DescBatch& cb, const DescBatch& nb,
                                           const Derived2& cd) {
  if (k - kb >= kBatch) return blk2_setup_scalar<MODE>(a, k, kend, kb, cb, nb);
  const uint32_t sl = static_cast<uint32_t>(k - kb);
  Blk2 b;
  b.off = readlane64(cb.off_lo, cb.off_hi, sl);
  b.size = readlane32(cb.size, sl);
  b.mod = readlane32(cb.mod, sl);
  b.extra = readlane32(cb.extra, sl);
  b.pk = readlane32(cd.pk, sl);
  b.R = readlane32(cd.R, sl);
  b.S0 = MODE == kModeRaw ? readlane32(cd.S0, sl) : kCrcS0[(b.pk >> 17) & 3u];
  b.we = b.slow() ? kRB2 : ((b.off + b.size + (mem_last_byte<MODE>(a) ? 1u : 0u)) & ~3ull);
  return b;
}

struct StepBuf2 {
  uint32_t w[2][8];
  uint32_t t0, t1, t2;  // t2: the xtra dword
};

template <int MODE>
__device__ __forceinline__ void issue_step2(const uint8_t* __restrict__ base, uint32_t lane,
                                            const Blk2& b, uint32_t r, StepBuf2& buf) {
  const int64_t w0 = b.w0();
  const uint32_t cA = b.cA(), lA = b.lA();
#pragma unroll
  for (uint32_t c = 0; c < 2; ++c) {
    int64_t so = w0 + static_cast<int64_t>(r) * kRB2 + kChain2 * c + kSeg2 * lane;
    if (r == 0) {
      // segments wholly in front of the head: any safe in-message address
      const bool pre = c < cA || (c == cA && lane < lA);
      so = pre ? static_cast<int64_t>(b.we) - kSeg2 : so;
      so = so < 0 ? 0 : so;
    }
    const uint8_t* sp = base + so;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const u32x4a4 v = ld16_a4(sp + 16 * q);
      buf.w[c][4 * q + 0] = v.x;
      buf.w[c][4 * q + 1] = v.y;
      buf.w[c][4 * q + 2] = v.z;
      buf.w[c][4 * q + 3] = v.w;
    }
  }
  // tail dword at we (holds the <= 3 tail bytes; in verify mode the stored
  // checksum starts inside it or is the next dword); slow blocks: offset 0
  const uint32_t nt = b.nt();
  const uint64_t t0 = b.slow() ? 0 : (nt > 0 || MODE == kModeVerify) ? b.we : b.we - 4;
  buf.t0 = ld4v(base + t0);
  buf.t1 = MODE == kModeVerify ? ld4v(base + (b.slow() || nt == 0 ? t0 : t0 + 4)) : 0u;
  buf.t2 = MODE != kModeRaw ? ld4v(base + (b.xtra() ? b.we - 4 : t0)) : 0u;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// the four table reads of G(x) (J = false) or J2(x) (J = true)
template <bool J>
__device__ __forceinline__ void rep_look(const uint8_t* __restrict__ Lb, const Lanes2& k,
                                         uint32_t x, uint32_t (&l)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    l[i] = lds32(Lb, __builtin_amdgcn_perm(x, k.lpack, k.sel[i]) + (J ? 128u : 0u));
}

// G(x) ^ e: the next chain input when e is the next data word
__device__ __forceinline__ uint32_t g_then(const uint8_t* __restrict__ Lb, const Lanes2& k,
                                           uint32_t x, uint32_t e) {
  uint32_t l[4];
  rep_look<false>(Lb, k, x, l);
  return xor3(l[0], l[1], xor3(l[2], l[3], e));
}

// one round of both chains.  Chain inputs are carried as x = state ^ next word,
// so every step is 4 v_perm + 4 ds_read + 2 v_bitop3.
__device__ __forceinline__ void stream_round2(const uint8_t* __restrict__ Lb, const Lanes2& K,
                                              uint32_t lane, const Blk2& b, uint32_t r,
                                              uint32_t (&s)[2], const uint32_t (&w)[2][8]) {
  if (r == 0) {
    const uint32_t cA = b.cA(), lA = b.lA(), jA = b.jA(), q = b.q();
    const uint32_t bm = b.bm();
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c) {
      uint32_t wc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) wc[j] = w[c][j];
      if (q != 0 && c == cA) {  // head segment loaded from offset 0: shift up q dwords
        uint32_t sh[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          uint32_t v = 0;
#pragma unroll
          for (int qq = 1; qq < 8; ++qq)
            if (qq <= j) v = (q == static_cast<uint32_t>(qq)) ? wc[j - qq] : v;
          sh[j] = v;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) wc[j] = lane == lA ? sh[j] : wc[j];
      }
      // words in front of the message's first dword are zeroed (G(0) = 0, so
      // the chain state stays 0 until the head word) ...
      const uint32_t js = (c < cA || (c == cA && lane < lA)) ? 8u
                          : (c == cA && lane == lA)          ? jA
                                                             : 0u;
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) wc[j] = j < js ? 0u : wc[j];
      // ... and the head word of the head lane loses the bytes in front of
      // the message and gains S0 (uniform dynamic index jA)
      if (c == cA) {
        const uint32_t hv = wc[jA];
        wc[jA] = lane == lA ? ((hv & bm) ^ b.S0) : hv;
      }
      uint32_t x = wc[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) x = g_then(Lb, K, x, wc[j]);
      s[c] = g_then(Lb, K, x, 0u);
    }
  } else {
    // first word of each chain: J2(s) ^ G(w0) ^ w1 (hop fused with the step)
    uint32_t x[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint32_t lj[4], lg[4];
      rep_look<true>(Lb, K, s[c], lj);
      rep_look<false>(Lb, K, w[c][0], lg);
      x[c] = xor3(xor3(lj[0], lj[1], lj[2]), xor3(lj[3], lg[0], lg[1]), xor3(lg[2], lg[3], w[c][1]));
    }
#pragma unroll
    for (int j = 2; j < 8; ++j) {
      x[0] = g_then(Lb, K, x[0], w[0][j]);
      x[1] = g_then(Lb, K, x[1], w[1][j]);
    }
    s[0] = g_then(Lb, K, x[0], 0u);
    s[1] = g_then(Lb, K, x[1], 0u);
  }
}

// XOR of the 16 lanes of each row, valid in the row's last lane (DPP row_shr)
template <int N>
__device__ __forceinline__ uint32_t row_shr_xor(uint32_t v) {
  return v ^ static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x110 + N,
                                                               0xf, 0xf, false));
}

// XOR of the 16 lanes of each row, valid in every lane of the row (DPP row_ror)
template <int N>
__device__ __forceinline__ uint32_t row_ror_xor(uint32_t v) {
  return v ^ static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x120 + N,
                                                               0xf, 0xf, false));
}

// join the 2 x 64 chain states, fold in the tail bytes and the extra byte;
// returns ~state (the crc32c::Extend value), wave-uniform
template <int MODE>
__device__ __forceinline__ uint32_t stream_finish2(const uint8_t* __restrict__ Lb,
                                                   const Lanes2& K, uint32_t lane, const Blk2& b,
                                                   const uint32_t (&s)[2], uint32_t t0,
                                                   uint32_t t2, bool has_extra) {
  // chain c of lane l ends 2048 (1 - c) + 32 (63 - l) bytes before the round end
  const bool lo0 = (lane & 15) == 15;
  const uint32_t abase = kOffA2 + 4096 * (14 - (lane & 15));  // A[lo], lo = 15 - (lane & 15)
  uint32_t a0 = lo0 ? s[0] : shift_at(Lb, abase, s[0]);
  uint32_t a1 = lo0 ? s[1] : shift_at(Lb, abase, s[1]);
  a0 = row_shr_xor<1>(a0);
  a1 = row_shr_xor<1>(a1);
  a0 = row_shr_xor<2>(a0);
  a1 = row_shr_xor<2>(a1);
  a0 = row_shr_xor<4>(a0);
  a1 = row_shr_xor<4>(a1);
  a0 = row_shr_xor<8>(a0);
  a1 = row_shr_xor<8>(a1);
  // lane 16 rho + 15: chain 0 row value needs B[7 - rho], chain 1 B[3 - rho]
  uint32_t v = 0;
  if (lo0) {
    const uint32_t rho = lane >> 4;
    const uint32_t v0 = shift_at(Lb, kOffB2 + 4096 * (6 - rho), a0);
    const uint32_t v1 = rho == 3 ? a1 : shift_at(Lb, kOffB2 + 4096 * (2 - rho), a1);
    v = v0 ^ v1;
  }
  uint32_t st = readlane32(v, 15) ^ readlane32(v, 31) ^ readlane32(v, 47) ^ readlane32(v, 63);
  if (MODE != kModeRaw && b.xtra()) st = step_k(Lb, K, st, t2, 4);
  const uint32_t nt = b.nt();
  uint32_t y = nt ? (t0 & (0xffffffffu >> (32 - 8 * nt))) : 0u;
  uint32_t k = nt;
  if (has_extra) {
    y |= (b.extra & 0xffu) << (8 * k);
    ++k;
  }
  return ~step_k(Lb, K, st, y, k);
}

// short messages (< 64 bytes past the head dword): dword-serial, wave-uniform
__device__ __forceinline__ uint32_t small_crc2(const uint8_t* __restrict__ Lb, const Lanes2& K,
                                               const uint8_t* p, uint32_t len, uint32_t init,
                                               uint32_t nextra, uint32_t extra) {
  uint32_t s = ~init;
  const uint32_t m = static_cast<uint32_t>(reinterpret_cast<uint64_t>(p) & 3);
  uint32_t nh = (4 - m) & 3;
  nh = nh < len ? nh : len;
  uint32_t y = 0;
  for (uint32_t i = 0; i < nh; ++i) y |= ldu8(p + i) << (8 * i);
  s = step_k(Lb, K, s, y, nh);
  uint32_t i = nh;
  for (; i + 4 <= len; i += 4) s = rep_map<false>(Lb, K, s ^ ld4v(p + i));
  y = 0;
  const uint32_t nt = len - i;
  for (uint32_t j = 0; j < nt; ++j) y |= ldu8(p + i + j) << (8 * j);
  s = step_k(Lb, K, s, y, nt);
  if (nextra) s = step_k(Lb, K, s, extra & 0xffu, 1);
  return ~s;
}

// PROBE = 1 (diagnostics build only, FORST_CRC_VARIANT=probe_load): the same
// loads and control flow, but every data word is only XOR-folded (no table
// lookups) and every block reports ok -- the memory-side ceiling of this
// access pattern; 2 = no finish, 3 = no head handling.
template <int MODE, int PROBE>
__device__ __forceinline__ void crc32c_stream2_body(const BlockArgs& a) {
  __shared__ uint32_t L[kLds2Bytes / 4];
  fill_tables2(L);
  const uint8_t* Lb = reinterpret_cast<const uint8_t*>(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const Lanes2 K = lanes2(lane);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kWaves;
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * kWaves + wave;
  uint64_t kbeg, kend;
  wave_share(a.n, nw, gw, kbeg, kend);
  if (kbeg >= kend) return;
  const bool has_extra = (MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes;

  DescBatch cb, nb;
  uint64_t kb = kbeg;
  load_batch<MODE>(a, kb, kend, lane, cb);
  load_batch<MODE>(a, kb + kBatch, kend, lane, nb);
  Derived2 cd = derive2<MODE>(a, cb, kb, kend, lane);
  // Three cursors over the (block, round) step sequence: C is computed from
  // the buffer filled two steps ago, P1's loads are in flight, P2's are issued
  // now -- two 4 KiB steps (8 KiB) per wave stay in flight while C computes.
  uint64_t k = kbeg, k1 = 0, k2 = 0;  // blocks of C, P1, P2
  uint32_t r = 0, r1 = 0, r2 = 0;     // their rounds
  Blk2 C = blk2_setup<MODE>(a, k, kend, kb, cb, nb, cd);
  Blk2 P1, P2;
  auto advance = [&](const Blk2& b, uint64_t kk, uint32_t rr, Blk2& nbk, uint64_t& nk,
                     uint32_t& nr) {
    if (!b.slow() && rr + 1 < b.R) {
      nbk = b;
      nk = kk;
      nr = rr + 1;
    } else {
      nk = kk + 1;
      nr = 0;
      nbk = blk2_setup<MODE>(a, nk, kend, kb, cb, nb, cd);
    }
  };
  advance(C, k, 0, P1, k1, r1);
  advance(P1, k1, r1, P2, k2, r2);
  uint32_t rOut = 0, rSt = 0, rOk = 0;
  StepBuf2 X, Y, Z;
  issue_step2<MODE>(a.base, lane, C, 0, X);
  issue_step2<MODE>(a.base, lane, P1, r1, Y);
  uint32_t s[2] = {0, 0};

  auto flush = [&](uint32_t cnt) {
    const uint64_t i = kb + lane;
    const bool mine = lane < cnt;
    if (mine && a.out32) a.out32[i] = rOut;
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

  // one step: issue P2 into nx, compute C from cu; false when done
  auto step = [&](StepBuf2& cu, StepBuf2& nx) -> bool {
    issue_step2<MODE>(a.base, lane, P2, r2, nx);
    const bool last = C.slow() || r + 1 >= C.R;
    if (PROBE == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[0] ^= cu.w[0][j];
        s[1] ^= cu.w[1][j];
      }
    } else if (PROBE == 3 && !C.slow()) {
      stream_round2(Lb, K, lane, C, 1, s, cu.w);  // no head handling
    } else if (!C.slow()) {
      stream_round2(Lb, K, lane, C, r, s, cu.w);
    }
    if (last) {
      uint32_t crc = 0, stored = 0;
      if (PROBE == 2 || PROBE == 3) {  // rounds only / no head: finish cost still in 3
        const uint32_t f = PROBE == 3
                               ? stream_finish2<MODE>(Lb, K, lane, C, s, cu.t0, cu.t2, has_extra)
                                      : s[0] ^ s[1];
        stored = crc_mask(0) + C.mod;
        crc = __ballot(f == 0x9e3779b9u) ? 1u : 0u;
        s[0] = s[1] = 0;
      } else if (PROBE) {
        const uint32_t f = s[0] ^ s[1] ^ cu.t0 ^ cu.t1;
        stored = crc_mask(0) + C.mod;
        crc = __ballot(f == 0x9e3779b9u) ? 1u : 0u;
        s[0] = s[1] = 0;
      } else if (!C.slow()) {
        crc = stream_finish2<MODE>(Lb, K, lane, C, s, cu.t0, cu.t2, has_extra);
        if (MODE == kModeVerify)
          stored = C.nt() ? __builtin_amdgcn_alignbyte(cu.t1, cu.t0, C.nt()) : cu.t0;
      } else if (C.valid()) {
        const uint8_t* p = a.base + C.off;
        const uint32_t init = MODE == kModeRaw ? C.extra : 0u;
        crc = small_crc2(Lb, K, p, C.size + (mem_last_byte<MODE>(a) ? 1u : 0u), init, has_extra ? 1u : 0u, C.extra);
        // retire(): keep the slow path's loads from merging into the hot path
        if (MODE == kModeVerify) stored = retire(ldu32(p + C.size + 1));
        crc = retire(crc);
      }
      uint32_t out, st = 0, ok = C.valid() ? 1u : 0u;
      if (MODE == kModeRaw) {
        out = crc;
      } else if (MODE == kModeVerify) {
        const uint32_t computed = crc_mask(crc);  // reader_common.cc:36-47
        st = stored - C.mod;
        ok = (C.valid() && st == computed) ? 1u : 0u;
        out = computed;
      } else {
        out = crc_mask(crc) + C.mod;  // format.cc:594-600 + builder.cc:1340-1345
      }
      if (!C.valid()) {
        out = 0;
        st = 0;
      }
      const uint32_t kk = static_cast<uint32_t>(k - kb);
      rOut = lane == kk ? out : rOut;
      rSt = lane == kk ? st : rSt;
      rOk = lane == kk ? ok : rOk;
      if (k + 1 - kb == kBatch || k + 1 == kend) {
        flush(static_cast<uint32_t>(k + 1 - kb));
        if (k + 1 == kend) return false;
        kb = k + 1;
        cb = nb;
        cd = derive2<MODE>(a, cb, kb, kend, lane);
        load_batch<MODE>(a, kb + kBatch, kend, lane, nb);
      }
    }
    // rotate the cursors: C <- P1 <- P2 <- the step after P2
    C = P1;
    k = k1;
    r = r1;
    P1 = P2;
    k1 = k2;
    r1 = r2;
    advance(P1, k1, r1, P2, k2, r2);
    return true;
  };
  while (step(X, Z) && step(Y, X) && step(Z, Y)) {
  }
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) crc32c_stream2_kernel(BlockArgs a) {
  crc32c_stream2_body<MODE, 0>(a);
}

#ifdef FORST_DIAG
template <int PROBE>
__global__ void __launch_bounds__(kThreads) crc32c_stream2_probe_kernel(BlockArgs a) {
  crc32c_stream2_body<kModeVerify, PROBE>(a);
}
#endif

// ---------------------------------------------------------------------------
// CRC32C rows kernel (v3): one block per 16-lane row.
//
// In the one-block-per-wave kernels every block pays a full-wave finish
// (row-end shifts, DPP reduction, round-end shifts, tail step), a head set-up
// and a scalar block set-up; for 4 KiB blocks that is a third of the work.
// Here row r (lanes 16r..16r+15) owns a block and walks it in 1 KiB rounds:
// chain c (0, 1) of lane t owns the 32-byte segment [512c + 32t, +32) of
// every round, the hop to the next round is J3 = shift by 1024 - 32 + 4 bytes
// fused with the first dword step.  The four rows finish their blocks with
// ONE instruction stream: A[15 - t] moves each chain state to the end of the
// row, a 4-level DPP XOR reduces the row, B[1] (shift by 512) joins chain 0 to
// chain 1, and one k-byte slicing step adds the <= 3 tail bytes and the type
// byte.  Rows draw blocks dynamically from the wave's contiguous share (as in
// xxh3_rows_kernel); the head of a block is handled in round 0 of its row by
// zeroing the words in front of the message and injecting S0 into the head
// word, with rows at round 0 and rows in the middle of a block running the
// same code (J3(0) = 0).
//
// LDS: [0, 64K) G and J3 interleaved as in the v2 kernel, [64K, 124K) A[1..15],
// [124K, 128K) B[1].
// ---------------------------------------------------------------------------
// verify results staged in LDS and stored after the loop (1), or stored as
// rows finish (0): result stores in the streaming loop cost C2 verify 4.7 %
// (stores share vmcnt with the loads; profiles/ab_r04/c2_verify_stores.log)
#ifndef FORST_ROWS_STAGE
#define FORST_ROWS_STAGE 1
#endif
constexpr uint32_t kStageW = 6144;  // results per workgroup (30 KiB of LDS)
constexpr uint32_t kRowRound = 1024;
constexpr uint32_t kRowChain = 512;
constexpr uint32_t kLds3Bytes = kOffB2 + 4096;
constexpr uint32_t kNoBlk = 0xffffffffu;

// NT = the workgroup's thread count: constant trip counts, so every load of
// the fill is issued before the first LDS store waits (a loop with a
// blockDim trip count waited out one round of loads per iteration)
template <uint32_t NT>
__device__ __forceinline__ void fill_tables3(uint32_t* L) {
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t kN1 = (16384 + NT - 1) / NT, kN2 = (15 * 1024 + NT - 1) / NT,
                     kN3 = (1024 + NT - 1) / NT;
  uint32_t v1[kN1], v2[kN2], v3[kN3];
#pragma unroll
  for (uint32_t k = 0; k < kN1; ++k) {
    const uint32_t i = tid + k * NT;
    const uint32_t e = (i >> 6) & 255, d = i & 63, t = (d >> 3) & 3;
    v1[k] = i < 16384 ? (d < 32 ? kCrcG[t * 256 + e] : kCrcJ3[t * 256 + e]) : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kN2; ++k) {
    const uint32_t i = tid + k * NT;
    v2[k] = i < 15 * 1024 ? kCrcA[i] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kN3; ++k) {
    const uint32_t i = tid + k * NT;
    v3[k] = i < 1024 ? kCrcB[i] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < kN1; ++k)
    if (tid + k * NT < 16384) L[tid + k * NT] = v1[k];
#pragma unroll
  for (uint32_t k = 0; k < kN2; ++k)
    if (tid + k * NT < 15 * 1024) L[kOffA2 / 4 + tid + k * NT] = v2[k];
#pragma unroll
  for (uint32_t k = 0; k < kN3; ++k)
    if (tid + k * NT < 1024) L[kOffB2 / 4 + tid + k * NT] = v3[k];
  __syncthreads();
}

// a row's position (block of the wave share, 1 KiB round) and the block's
// window, derived once when the block is assigned; row-uniform, one copy per
// lane.  Offsets are relative to base and kept in the form the step's loads
// use, so a step issues its loads with a few adds (the per-step address
// arithmetic was a third of a 4 KiB block's VALU instructions).
struct CRowPos {
  uint32_t rp_lo, rp_hi;  // this round's window start (int64; < 0 only in round 0 near offset 0)
  uint32_t tp_lo, tp_hi;  // fast rows: the last round's finishing word t0, minus 4; slow: block offset
  uint32_t rel;           // descriptor index (kNoBlk: none)
  uint32_t rl;            // rounds left, this one included
  // cA:1 tA:4 jA:3 q:3 nt:2 m:2 valid:1 slow:1 xtra:1 d1:2 r0:1 | 24: slow rows' size:4
  // (every field a fast row needs after the derive is here: 7 VGPRs per copy)
  uint32_t pk;
  __device__ __forceinline__ int64_t rp() const {
    return static_cast<int64_t>((static_cast<uint64_t>(rp_hi) << 32) | rp_lo);
  }
  __device__ __forceinline__ uint64_t tp() const {
    return (static_cast<uint64_t>(tp_hi) << 32) | tp_lo;
  }
  __device__ __forceinline__ uint32_t cA() const { return pk & 1u; }
  __device__ __forceinline__ uint32_t tA() const { return (pk >> 1) & 15u; }
  __device__ __forceinline__ uint32_t jA() const { return (pk >> 5) & 7u; }
  __device__ __forceinline__ uint32_t q() const { return (pk >> 8) & 7u; }
  __device__ __forceinline__ uint32_t nt() const { return (pk >> 11) & 3u; }
  __device__ __forceinline__ uint32_t m() const { return (pk >> 13) & 3u; }
  __device__ __forceinline__ bool valid() const { return (pk >> 15) & 1u; }
  __device__ __forceinline__ bool slow() const { return (pk >> 16) & 1u; }
  __device__ __forceinline__ bool xtra() const { return (pk >> 17) & 1u; }
  __device__ __forceinline__ uint32_t d1() const { return (pk >> 16) & 12u; }  // bytes: 0, 4, 8
  __device__ __forceinline__ bool r0() const { return (pk >> 20) & 1u; }
  __device__ __forceinline__ uint32_t slow_size() const { return (pk >> 24) & 15u; }
  // (length-split batches) no descriptor yet, more may come: ask again
  __device__ __forceinline__ bool wait() const { return (pk >> 21) & 1u; }
  // fast rows: offset + size of the block (where a trailer goes), from the
  // window end: E - the type byte when it is in memory
  template <int MODE>
  __device__ __forceinline__ uint64_t end(bool mlb) const {
    const uint64_t t0 = tp() + 4;
    const uint64_t we = (MODE == kModeVerify || nt() > 0) ? t0 : t0 + 4;
    return we + nt() - (mlb ? 1u : 0u);
  }
};

template <int MODE>
__device__ __forceinline__ void crow_derive(const BlockArgs& a, uint64_t off, uint32_t size,
                                            CRowPos& P) {
  const bool valid = P.rel != kNoBlk && desc_in_range<MODE>(a, Desc{off, size, 0, 0});
  const uint64_t E = off + size + (mem_last_byte<MODE>(a) ? 1u : 0u);
  const uint64_t ws = off & ~3ull;
  const uint64_t we = E & ~3ull;
  const uint64_t d4 = we - ws;
  // a window one dword longer than whole rounds (1/4 of back-to-back 4 KiB
  // blocks: 4097 checksummed bytes starting at offset = 3 mod 4) ends one
  // dword early; that dword is one slicing step in the finish instead of a
  // fifth, almost empty round
  // (block modes only: raw messages of arbitrary lengths rarely hit it)
  const bool xtra = MODE != kModeRaw && (d4 & (kRowRound - 1)) == 4 && d4 > kRowRound;
  uint32_t R = static_cast<uint32_t>(xtra ? d4 / kRowRound : (d4 + kRowRound - 1) / kRowRound);
  int64_t w0 = static_cast<int64_t>(we) - (xtra ? 4 : 0) - static_cast<int64_t>(R) * kRowRound;
  const uint32_t hA = static_cast<uint32_t>(static_cast<int64_t>(ws) - w0);
  const uint32_t cA = hA >> 9, tA = (hA >> 5) & 15u, jA = (hA >> 2) & 7u;
  const int64_t seg_head = static_cast<int64_t>(ws) - 4 * static_cast<int64_t>(jA);
  const uint32_t q = seg_head < 0 ? static_cast<uint32_t>(-seg_head) >> 2 : 0u;
  const uint32_t nt = static_cast<uint32_t>(E - we);
  const uint32_t m = static_cast<uint32_t>(off & 3);
  // the finishing words: t0 = the tail dword at the window end (verify: the
  // word holding the stored checksum when nt = 0), t1 = the word after it
  // (verify, nt > 0) or the extra window dword (compute / trailer, xtra), t2
  // = the extra window dword (verify, xtra) -- loaded at tp + 4, tp + d1 and
  // tp, so t0 >= 4 (else the slow path: messages ending in the first dwords)
  const uint64_t t0 = (nt > 0 || MODE == kModeVerify) ? we : we - 4;
  const uint32_t d1 = MODE == kModeVerify ? (nt > 0 ? 8u : 4u) : (xtra && nt > 0 ? 0u : 4u);
  // messages without one whole dword take the slow path (its loads are serial
  // and unprefetched: a WAL record of 40 B through it cost a wave ~10 dependent
  // load latencies); everything else, however short, is one prefetched round
  const bool slow = !valid || d4 < 4 || t0 < 4;
  const uint64_t tp = slow ? off : t0 - 4;
  if (slow) {  // the slow path loads on its own; dummy round loads at [0, 1 KiB)
    R = 1;
    w0 = 0;
  }
  P.rl = R;
  P.rp_lo = static_cast<uint32_t>(w0);
  P.rp_hi = static_cast<uint32_t>(static_cast<uint64_t>(w0) >> 32);
  P.tp_lo = static_cast<uint32_t>(tp);
  P.tp_hi = static_cast<uint32_t>(tp >> 32);
  // a valid slow block has fewer than 12 checksummed bytes (d4 < 4 or t0 < 4)
  P.pk = (slow ? (valid ? (size & 15u) << 24 : 0u)
               : (cA | (tA << 1) | (jA << 5) | (q << 8) | (xtra ? 1u << 17 : 0u) |
                  ((d1 >> 2) << 18))) |
         (nt << 11) | (m << 13) | (valid ? 1u << 15 : 0u) | (slow ? 1u << 16 : 0u) | (1u << 20);
}

struct CRStep {
  uint32_t w[2][8];
  uint32_t t0, t1, t2, mod, extra;  // t2: the extra window dword (xtra)
};

template <int MODE, int PROBE = 0>
__device__ __forceinline__ void crow_issue(const BlockArgs& a, uint32_t lane, const CRowPos& P,
                                           uint64_t kbeg, CRStep& d) {
  const uint32_t t = lane & 15;
  if (PROBE == 3) {  // diagnostics: the same bytes as 16-B aligned, row-contiguous pieces
    const int64_t rb = (P.rp() & ~int64_t(15)) + 16 * t;
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        int64_t so = rb + 256 * (2 * c + q);
        so = so < 0 ? 0 : so;
        const u32x4a4 v = ld16_a4(a.base + so);
        d.w[c][4 * q + 0] = v.x;
        d.w[c][4 * q + 1] = v.y;
        d.w[c][4 * q + 2] = v.z;
        d.w[c][4 * q + 3] = v.w;
      }
    d.t0 = d.t1 = d.t2 = d.mod = d.extra = 0u;
    return;
  }
  // the lane's chain-0 segment; chain 1 is 512 bytes on.  Round-0 segments
  // in front of the head hold no message byte: they are loaded from where
  // they are and discarded by the head reset; only a segment in front of the
  // buffer start (a message ending in its first KiB) is loaded from 0 (the
  // head lane's is realigned by q dwords in the head step).  No branch around
  // a load: a step's loads must not depend on one, or the compiler's vmcnt
  // waits for the current step's data also wait for the step in flight.
  int64_t s0 = P.rp() + kSeg2 * t;
  int64_t s1 = s0 + kRowChain;
  if (__ballot(s0 < 0)) {  // rare (addresses only): a round in front of offset 0
    s0 = s0 < 0 ? 0 : s0;
    s1 = s1 < 0 ? 0 : s1;
  }
  // (Loading the round-0 segments in front of a raw record's head from the
  // buffer's first KiB instead, to save their HBM bytes -- 1.07x the log on
  // C5 -- measured no faster: C5 verify 0.604-0.608 vs 0.606-0.609,
  // profiles/ab_r05/raw_pre_head_redirect_C5.log.  They are mostly the
  // previous record's bytes, which its own row reads at about the same time.)
#pragma unroll
  for (uint32_t c = 0; c < 2; ++c) {
    const uint8_t* sp = a.base + (c ? s1 : s0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const u32x4a4 v = ld16_a4(sp + 16 * q);
      d.w[c][4 * q + 0] = v.x;
      d.w[c][4 * q + 1] = v.y;
      d.w[c][4 * q + 2] = v.z;
      d.w[c][4 * q + 3] = v.w;
    }
  }
  // the finishing step's words, loaded in every step (from offset 0 when not
  // needed): a step's load count must not depend on a branch (see above)
  const bool lastr = !P.slow() && P.rl <= 1;
  const uint8_t* pb = a.base + (lastr ? P.tp() : 0);
  d.t0 = ld4_a4(pb + 4);
  d.t1 = MODE == kModeRaw ? 0u : ld4_a4(pb + P.d1());
  d.t2 = MODE == kModeVerify ? ld4_a4(pb) : 0u;
  // optional arrays: (read in the ISA) a branch around these loads keeps the
  // compiler's vmcnt waits precise, a pointer select to a zero word does not
  const uint64_t idx = kbeg + (P.rel == kNoBlk ? 0 : P.rel);
  if (MODE != kModeRaw)
    d.mod = a.modifiers ? a.modifiers[idx] : 0u;
  else
    d.mod = a.expect ? a.expect[idx] : 0u;  // (raw: the expected CRC)
  if (MODE == kModeRaw)
    d.extra = a.init_crcs ? a.init_crcs[idx] : 0u;
  else if (MODE != kModeVerify)
    d.extra = a.last_bytes ? a.last_bytes[idx] : 0u;
  else
    d.extra = 0u;
}

// PROBE (diagnostics build only): 1 = same loads and row bookkeeping, no
// table work and no finish; 2 = no per-block finish.
// DEPTH 2 (diagnostics build only): two steps of loads in flight per wave
// (three step buffers, 12-wave workgroups at 3 waves/SIMD) instead of one.
constexpr uint32_t kRowsD2Waves = 12;
#ifdef FORST_DIAG
// diagnostics build only: per-wave start / end wall clock (100 MHz) of the
// last rows-kernel launch, for the tail analysis (tools/wave_tail.py)
constexpr uint32_t kDiagWaves = 8192;
__device__ unsigned long long g_wave_t0[kDiagWaves], g_wave_t1[kDiagWaves];
#endif
// Raw batches split by message length (FILT): messages shorter than
// kRawSplit bytes go to crc32c_raw_lane_kernel (one message per lane), the
// rest to the rows kernel, which drops the short ones from each descriptor
// batch as it loads it.  A short WAL record still costs a row a whole 1 KiB
// round; on C5 the records <= 512 B (40 % of them, 1.5 % of the bytes) took
// 0.69 ms of the 9.03 ms raw pass (profiles/ab_r04/c5_record_classes_raw_crc.json).
#ifndef FORST_RAW_SPLIT
#define FORST_RAW_SPLIT 256
#endif
constexpr uint32_t kRawSplit = FORST_RAW_SPLIT;

// A message goes to the rows filter kernel when it has kRawSplit bytes or
// more and its offset is below 2^58 (any larger one lies outside every
// buffer: the lane kernel reports it; batch_compact, stream_common.h).
__device__ __forceinline__ bool raw_long(uint64_t off, uint32_t size) {
  return size >= kRawSplit && (off >> 58) == 0;
}

#ifndef FORST_RAW_RING
#define FORST_RAW_RING 1
#endif
template <int MODE, int PROBE, int DEPTH, bool RAW_WG = false, bool FILT = false>
__device__ __forceinline__ void crc32c_rows_body(const BlockArgs& a) {
  static_assert(!FILT || (MODE == kModeRaw && !RAW_WG), "length split: raw global feed only");
  __shared__ uint32_t L[kLds3Bytes / 4];
  feed_init();
  fill_tables3<64 * (DEPTH == 2 ? kRowsD2Waves : kWaves)>(L);
  const uint8_t* Lb = reinterpret_cast<const uint8_t*>(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t t = lane & 15;
  const Lanes2 K = lanes2(lane);
  __shared__ uint32_t s0t[4];  // head states by start alignment (a select, not branches)
  if (threadIdx.x < 4) s0t[threadIdx.x] = kCrcS0[threadIdx.x];
  __syncthreads();
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (DEPTH == 2 ? kRowsD2Waves : kWaves);
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * (DEPTH == 2 ? kRowsD2Waves : kWaves) + wave;
  const bool has_extra = (MODE == kModeCompute || MODE == kModeTrailer) && a.last_bytes;

  // descriptor batches from the work feed: lane j <-> descriptor cg + j (cb),
  // ng + j (nb); a row's rel is the descriptor's global index (n < 2^32 - 1)
#ifdef FORST_DIAG
  if (lane == 0 && gw < kDiagWaves) {
    g_wave_t0[gw] = wall_clock64();
    g_wave_t1[gw] = 0;
  }
#endif
  BatchFeed feed;
  // block modes: the workgroup feed in 4-descriptor batches (one block per
  // row; A/B against 8: C2 verify +2.2 %, write +1.8 %, NS16 +0.9 %, C4
  // +1.4 %, profiles/ab_r03/crc_feed_batch.log; 16 was 3 % slower than 8);
  // WAL records (raw) keep the global feed (byte-balanced workgroup ranges
  // measured within noise for them, profiles/ab_r03/wal_wg_feed.log), except
  // small raw batches (RAW_WG: crc32c_rows_raw_small_kernel)
  constexpr bool kWgFeed = MODE != kModeRaw || RAW_WG;
  constexpr uint32_t kChunk = 4;
  uint64_t cg = feed_first<kWgFeed, kChunk>(a, nw, gw, lane, feed);
  // verify: results staged in LDS, stored after the loop by the whole
  // workgroup (so every wave reaches the end: no early return)
  constexpr bool kStage = FORST_ROWS_STAGE && MODE != kModeRaw && kWgFeed && DEPTH == 1 &&
                          PROBE == 0;
  __shared__ uint32_t st_out[kStage ? kStageW : 1];
  __shared__ uint8_t st_ok[kStage ? kStageW : 4];
  // raw mode: each wave's results collected in an LDS ring and stored 64 per
  // instruction when it fills and after the loop (stores share vmcnt with the
  // loads, so a store per finishing row delayed the next step's data)
  constexpr bool kRing = FORST_RAW_RING && MODE == kModeRaw && PROBE == 0 && DEPTH == 1;
  constexpr uint32_t kRingN = 224;  // per wave (16 waves: 28 KiB beside the 128 KiB of tables)
  __shared__ uint32_t ring_i[kRing ? kWaves * kRingN : 1], ring_v[kRing ? kWaves * kRingN : 1];
  uint32_t* const ri = ring_i + (kRing ? wave * kRingN : 0);
  uint32_t* const rv = ring_v + (kRing ? wave * kRingN : 0);
  uint32_t rcount = 0;  // (wave-uniform)
  auto ring_flush = [&]() {
    wave_lds_sync();
    for (uint32_t j = lane; j < rcount; j += 64) a.out32[ri[j]] = rv[j];
    wave_lds_sync();
    rcount = 0;
  };
  if (!kStage && cg >= a.n) return;
  uint32_t clen = feed.len;  // entries of cb / nb (a batch holds up to 64)
  uint64_t ng = 0;
  uint32_t nlen = 0;
  if constexpr (!FILT) {  // (FILT: claimed after cb, whose loading may claim further)
    ng = feed_next<kWgFeed, kChunk>(a, nw, lane, feed);
    nlen = feed.len;
  }
  DescBatch cb, nb;
  uint64_t kbrel = 0;  // stream position of cb's first entry
  // FILT: the batch's messages of kRawSplit bytes or more, moved to its
  // first lanes; a batch with none is skipped (the next one claimed) so a
  // batch is empty only once the feed is exhausted.  (The ballot waits for
  // the batch's loads: one load latency per 64 descriptors.)
  auto load_f = [&](uint64_t& g, uint32_t& len, DescBatch& d) {
    load_batch<MODE>(a, g, a.n, lane, d);
    if constexpr (FILT) {
      for (;;) {
        const bool keep =
            lane < len && raw_long((static_cast<uint64_t>(d.off_hi) << 32) | d.off_lo, d.size);
        const uint64_t km = __ballot(keep);
        if (km != 0 || len == 0) {
          batch_compact<false, false>(d, km, keep, lane);
          len = static_cast<uint32_t>(__popcll(km));
          break;
        }
        g = feed_next<kWgFeed, kChunk>(a, nw, lane, feed);
        len = feed.len;
        load_batch<MODE>(a, g, a.n, lane, d);
      }
    }
  };
  load_f(cg, clen, cb);
  if constexpr (FILT) {
    ng = feed_next<kWgFeed, kChunk>(a, nw, lane, feed);
    nlen = feed.len;
  }
  load_f(ng, nlen, nb);
  const uint64_t kbeg = 0;
  auto fetch = [&](uint64_t rel, CRowPos& P) {
    const BatchSlot q = batch_slot(rel, kbrel, cg, clen, ng, nlen, a.n);
    const uint32_t lo_c = __shfl(cb.off_lo, q.src), hi_c = __shfl(cb.off_hi, q.src);
    const uint32_t sz_c = __shfl(cb.size, q.src);
    const uint32_t lo_n = __shfl(nb.off_lo, q.src), hi_n = __shfl(nb.off_hi, q.src);
    const uint32_t sz_n = __shfl(nb.size, q.src);
    uint32_t hi = q.in_n ? hi_n : hi_c;
    uint64_t gi = q.gi;
    if constexpr (FILT) {  // slot k of a compacted batch: descriptor base + its lane as loaded
      gi = (q.in_n ? ng : cg) + (hi >> 26);
      hi &= 0x03ffffffu;
    }
    const uint64_t off = (static_cast<uint64_t>(hi) << 32) | (q.in_n ? lo_n : lo_c);
    const uint32_t size = q.in_n ? sz_n : sz_c;
    P.rel = q.valid ? static_cast<uint32_t>(gi) : kNoBlk;
    crow_derive<MODE>(a, off, size, P);
  };
  // A compacted batch may hold fewer descriptors than the wave has rows
  // (FILT): positions are handed out only while cb and nb have some left, and
  // a row that finds none WAITS (asks again in the next step) unless the feed
  // is exhausted -- a position handed to no row would be a descriptor never
  // computed.  (Full batches have 64: the original rule never runs short.)
  uint64_t next = 4;
  CRowPos C;
  fetch(lane >> 4, C);
  if constexpr (FILT) {
    const uint64_t avail = clen + nlen;
    if ((lane >> 4) >= avail && nlen != 0) C.pk |= 1u << 21;
    next = avail < 4 ? avail : 4;
  }
  auto advance = [&](const CRowPos& P, CRowPos& I) {
    const bool more = P.rel != kNoBlk && !P.slow() && P.rl > 1;
    const bool need = (P.rel != kNoBlk || (FILT && P.wait())) && !more;
    const uint64_t rows = __ballot(need && t == 0);  // one bit per row leader
    I = P;
    if (more) {
      I.rl = P.rl - 1;
      I.pk = P.pk & ~(1u << 20);
      const int64_t rp = P.rp() + kRowRound;
      I.rp_lo = static_cast<uint32_t>(rp);
      I.rp_hi = static_cast<uint32_t>(static_cast<uint64_t>(rp) >> 32);
    }
    // rows in the middle of their blocks (every row, 3 steps in 4 of a batch
    // of 4 KiB blocks): no descriptor work
    if (rows) {
      // rows needing one ahead of this row: rows' bits below the lane, less
      // the row's own leader bit (rows holds leader bits only) -- v_mbcnt, no
      // per-lane 64-bit mask held across the loop
      const uint32_t below = __builtin_amdgcn_mbcnt_hi(
          static_cast<uint32_t>(rows >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(rows), 0u));
      const uint32_t rank = below - (t != 0 && need ? 1u : 0u);
      CRowPos F;
      fetch(next + rank, F);
      uint64_t got = static_cast<uint64_t>(__popcll(rows));
      if constexpr (FILT) {
        const uint64_t avail = kbrel + clen + nlen - next;
        if (got > avail) got = avail;
        if (rank >= avail && nlen != 0) F.pk |= 1u << 21;
      }
      next += got;
      if (need) I = F;
      if (next >= kbrel + clen) {  // every block of cb is assigned: slide the batches
        kbrel += clen;
        clen = nlen;
        cb = nb;
#ifndef FORST_HOST_EMULATION
        // cb's copies are made here, so the batch loads below can land in
        // nb's registers directly (a load into a temporary and a move after
        // it waited for every load in flight, the step's prefetch included)
        asm volatile("" : "+v"(cb.off_lo), "+v"(cb.off_hi), "+v"(cb.size));
#endif
        cg = ng;
        ng = feed_next<kWgFeed, kChunk>(a, nw, lane, feed);
        nlen = feed.len;
        load_f(ng, nlen, nb);
      }
    }
  };
  CRowPos I, I2;
  advance(C, I);
  if (DEPTH == 2) advance(I, I2);
  CRStep X, Y, Z;
  crow_issue<MODE, PROBE>(a, lane, C, kbeg, X);
  if (DEPTH == 2) crow_issue<MODE, PROBE>(a, lane, I, kbeg, Y);
  uint32_t s[2] = {0, 0};

  // cu: the current step's data (ready); nx: the buffer that receives the
  // loads issued now (the position DEPTH steps ahead)
  auto step = [&](CRStep& cu, CRStep& nx) -> bool {

    // raw mode (WAL records, mixed sizes): no early return (see
    // xxh3_frag_kernel), both step copies issue on every path round the loop
    // and the next step's loads overlap this step's wait (C5 verify / writer
    // +1.5 %); the block modes keep the early exit, which measured better on
    // uniform blocks (A/B on one box: C2 0.600 vs 0.592)
    const bool live = __ballot(C.rel != kNoBlk || (FILT && C.wait())) != 0;
    if ((DEPTH == 2 || MODE != kModeRaw) && !live) return false;
    crow_issue<MODE, PROBE>(a, lane, DEPTH == 2 ? I2 : I, kbeg, nx);
    const bool fast = C.rel != kNoBlk && !C.slow();
    const bool r0 = C.r0();
    // ---- one 1 KiB round of every row ----
    // A row at round 0 starts its block: its chain states start at 0 (J3(0) =
    // 0), segments wholly in front of the head end the round at state 0, and
    // in the head lane the running value is RESET at the head word to
    // (word & bm) ^ S0 (the head dword without the bytes in front of the
    // message, plus the initial state moved back over them), which discards
    // whatever the words in front of it added.  Steps without a row at
    // round 0 run the plain chains.
    const bool head = PROBE == 0 && __ballot(fast && r0);
    if (PROBE == 1 || PROBE == 3) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        uint32_t x = r0 ? 0u : s[c];
#pragma unroll
        for (int j = 0; j < 8; ++j) x ^= cu.w[c][j];
        s[c] = x;
      }
    } else if (!head) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        uint32_t lj[4], lg[4];
        rep_look<true>(Lb, K, r0 ? 0u : s[c], lj);
        rep_look<false>(Lb, K, cu.w[c][0], lg);
        uint32_t x = xor3(xor3(lj[0], lj[1], lj[2]), xor3(lj[3], lg[0], lg[1]),
                          xor3(lg[2], lg[3], cu.w[c][1]));
#pragma unroll
        for (int j = 2; j < 8; ++j) x = g_then(Lb, K, x, cu.w[c][j]);
        s[c] = g_then(Lb, K, x, 0u);
      }
    } else {
      const uint32_t cA = C.cA(), tA = C.tA(), jA = C.jA(), q = C.q(), m = C.m();
      const uint32_t bm = 0xffffffffu << (8 * m);
      // raw mode with per-message inits: the GF(2) unstep; without (crc32c::Value,
      // every WAL record) S0 is the block modes' constant
      const uint32_t S0 = MODE == kModeRaw && a.init_crcs ? unstep_m(~cu.extra, m) : s0t[m];
#pragma unroll
      for (uint32_t c = 0; c < 2; ++c) {
        const bool hl = fast && r0 && c == cA && t == tA;  // the head lane of the row
        const bool pre = fast && r0 && (c < cA || (c == cA && t < tA));
        const uint32_t hj = hl ? jA : 8u;
        uint32_t wc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) wc[j] = cu.w[c][j];
        if (__ballot(hl && q != 0)) {  // head segment loaded from 0: shift up q dwords
          uint32_t sh[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            uint32_t v = 0;
#pragma unroll
            for (int qq = 1; qq < 8; ++qq)
              if (qq <= j) v = (q == static_cast<uint32_t>(qq)) ? wc[j - qq] : v;
            sh[j] = v;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) wc[j] = (hl && q != 0) ? sh[j] : wc[j];
        }
        uint32_t lj[4], lg[4];
        rep_look<true>(Lb, K, r0 ? 0u : s[c], lj);
        rep_look<false>(Lb, K, hj == 0 ? ((wc[0] & bm) ^ S0) : wc[0], lg);
        uint32_t x = xor3(xor3(lj[0], lj[1], lj[2]), xor3(lj[3], lg[0], lg[1]),
                          xor3(lg[2], lg[3], wc[1]));
        x = hj == 1 ? ((wc[1] & bm) ^ S0) : x;
#pragma unroll
        for (uint32_t j = 2; j < 8; ++j) {
          x = g_then(Lb, K, x, wc[j]);
          x = hj == j ? ((wc[j] & bm) ^ S0) : x;
        }
        s[c] = pre ? 0u : g_then(Lb, K, x, 0u);
      }
    }
    // ---- rows that finish a block in this step ----
    const bool fin = C.rel != kNoBlk && (C.slow() || C.rl <= 1);
    if (PROBE != 0 && fin && t == 15 && a.out32) a.out32[C.rel] = s[0] ^ s[1] ^ cu.t0;
    if (PROBE == 0 && __ballot(fin)) {
      // chain states to the row end (A[15 - t]), row XOR, chain 0 over chain 1
      const bool lo0 = t == 15;
      const uint32_t abase = kOffA2 + 4096 * (14 - t);
      uint32_t a0 = lo0 ? s[0] : shift_at(Lb, abase, s[0]);
      uint32_t a1 = lo0 ? s[1] : shift_at(Lb, abase, s[1]);
      a0 = row_ror_xor<1>(a0);
      a1 = row_ror_xor<1>(a1);
      a0 = row_ror_xor<2>(a0);
      a1 = row_ror_xor<2>(a1);
      a0 = row_ror_xor<4>(a0);
      a1 = row_ror_xor<4>(a1);
      a0 = row_ror_xor<8>(a0);
      a1 = row_ror_xor<8>(a1);
      uint32_t crc = 0, stored = 0;
      const uint32_t nt = C.nt();
      // lanes that finish the CRC: the row's last lane, and in trailer mode
      // lanes 11..15, which store the 5 trailer bytes with one instruction
      const bool calc = fin && (MODE == kModeTrailer ? t >= 11 : lo0);
      if (calc) {
        uint32_t st = shift_at(Lb, kOffB2, a0) ^ a1;
        if (MODE != kModeRaw && C.xtra()) st = step_k(Lb, K, st, MODE == kModeVerify ? cu.t2 : cu.t1, 4);
        uint32_t y = nt ? (cu.t0 & (0xffffffffu >> (32 - 8 * nt))) : 0u;
        uint32_t k = nt;
        if (has_extra) {
          y |= (cu.extra & 0xffu) << (8 * k);
          ++k;
        }
        crc = ~step_k(Lb, K, st, y, k);
        if (MODE == kModeVerify) stored = nt ? __builtin_amdgcn_alignbyte(cu.t1, cu.t0, nt) : cu.t0;
      }
      if (calc && C.slow() && C.valid()) {
        const uint8_t* pp = a.base + C.tp();  // slow rows: the block offset
        const uint32_t init = MODE == kModeRaw ? cu.extra : 0u;
        crc = small_crc2(Lb, K, pp, C.slow_size() + (mem_last_byte<MODE>(a) ? 1u : 0u), init,
                         has_extra ? 1u : 0u, cu.extra);
        if (MODE == kModeVerify) stored = retire(ldu32(pp + C.slow_size() + 1));
        crc = retire(crc);
      }
      const bool valid = C.valid();
      const bool mine = fin && lo0;
      const uint64_t i = kbeg + (C.rel == kNoBlk ? 0 : C.rel);
      bool ok = valid;
      if (MODE == kModeRaw) {
        // WAL writer mode: masked (log_writer.cc:263).  The in-place header
        // stores are a separate pass (wal.hip): stores share vmcnt with the
        // loads on gfx950, so scattered partial-line stores here made every
        // later step wait for them (C5 writer 9.19 -> 9.90 ms)
        const uint32_t v = a.wal_hs ? crc_mask(crc) : crc;
        const bool differs = !a.expect || !valid || v != cu.mod;
#ifdef FORST_RAW_STORE_PROBE  // timing only: the store path kept but (almost) never taken
        if (mine && differs && a.out32 && v == 0x9e3779b9u) a.out32[i] = valid ? v : 0u;
#else
        if constexpr (kRing) {
          const bool put = mine && differs && a.out32 != nullptr;
          const uint64_t pm = __ballot(put);
          if (pm) {
            const uint32_t at = rcount + __builtin_amdgcn_mbcnt_hi(
                static_cast<uint32_t>(pm >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(pm), 0u));
            if (put) {
              ri[at] = static_cast<uint32_t>(i);
              rv[at] = valid ? v : 0u;
            }
            rcount += static_cast<uint32_t>(__popcll(pm));
            if (rcount > kRingN - 64) ring_flush();
          }
        } else {
          if (mine && differs && a.out32) a.out32[i] = valid ? v : 0u;
        }
#endif
      } else if (MODE == kModeVerify) {
        const uint32_t computed = crc_mask(crc);  // reader_common.cc:36-47
        const uint32_t st = stored - cu.mod;
        ok = valid && st == computed;
        // the workgroup's first kStageW results go to LDS (written after the
        // loop), the rest (ranges longer than that) directly
        const uint64_t sj = i - feed.wlo;
        const bool staged = kStage && sj < kStageW;
        if (mine && staged) {
          st_out[sj] = valid ? computed : 0u;
          st_ok[sj] = ok ? 1 : 0;
        }
        if (mine && !staged && a.out32) a.out32[i] = valid ? computed : 0u;
        if (mine && a.stored_out) a.stored_out[i] = valid ? st : 0u;
        if (mine && !staged && a.ok_out) a.ok_out[i] = ok ? 1 : 0;
        if (staged) ok = true;  // (counted in the flush)
      } else {
        const uint32_t out = crc_mask(crc) + cu.mod;  // format.cc:594-600 + builder.cc:1340-1345
        const uint64_t sj = i - feed.wlo;
        const bool staged = kStage && sj < kStageW;  // (see verify)
        if (mine && staged) {
          st_out[sj] = valid ? out : 0u;
          st_ok[sj] = valid ? 1 : 0;
        }
        if (mine && !staged && a.out32) a.out32[i] = valid ? out : 0u;
        if (MODE == kModeTrailer) {
          // the 5 trailer bytes [type][LE32] by lanes 11..15 of the row: one
          // byte store per wave instead of five per finishing row
          const uint32_t k = t - 11;
          if (!staged && calc && valid && (k != 0 || a.last_bytes)) {
            uint8_t* pw = a.base_w + C.template end<MODE>(mem_last_byte<MODE>(a));
            pw[k] = static_cast<uint8_t>(k == 0 ? cu.extra : out >> (8 * (k - 1)));
          }
        }
      }
      if (MODE == kModeVerify) {
        const uint64_t badm = __ballot(mine && !ok);
        if (a.mismatches && badm && lane == 0)
          atomicAdd(a.mismatches, static_cast<unsigned long long>(__popcll(badm)));
      }
    }
#ifndef FORST_HOST_EMULATION
    // the finishing words are read only when a row finishes; a use on every
    // path retires their loads here (a precise wait, the next step's loads
    // are younger), so reusing their registers in the next step needs no
    // full vmcnt(0) wait on the step in flight
    asm volatile("" ::"v"(cu.t0), "v"(cu.t1), "v"(cu.t2), "v"(cu.mod), "v"(cu.extra));
#endif
    C = I;
    if (DEPTH == 2) {
      I = I2;
      advance(I, I2);
    } else {
      advance(C, I);
    }
    return live;
  };
  if (DEPTH == 2) {
    while (step(X, Z) && step(Y, X) && step(Z, Y)) {
    }
  } else {
    if (MODE == kModeRaw) {
      for (bool more = true; more;) {
        step(X, Y);
        more = step(Y, X);
      }
    } else {
      while (step(X, Y) && step(Y, X)) {
      }
    }
  }
#ifdef FORST_DIAG
  if (lane == 0 && gw < kDiagWaves) g_wave_t1[gw] = wall_clock64();
#endif
  if constexpr (kRing) {
    if (rcount) ring_flush();
  }
  if constexpr (kStage) {  // the staged results, coalesced
    __syncthreads();
    const uint64_t lo = feed.wlo, hi = feed.whi;
    const uint64_t m = hi > lo ? (hi - lo < kStageW ? hi - lo : kStageW) : 0;
    uint32_t bad = 0;
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
      const uint64_t g = lo + j;
      if (a.out32) a.out32[g] = st_out[j];
      if (MODE == kModeVerify) {
        if (a.ok_out) a.ok_out[g] = st_ok[j];
        bad += st_ok[j] ? 0u : 1u;
      }
      if (MODE == kModeTrailer && st_ok[j]) {  // [type][LE32] at offset + size
        uint8_t* pw = a.base_w + a.offsets[g] + a.sizes[g];
        const uint32_t v = st_out[j];
        if (a.last_bytes) pw[0] = a.last_bytes[g];
        pw[1] = static_cast<uint8_t>(v);
        pw[2] = static_cast<uint8_t>(v >> 8);
        pw[3] = static_cast<uint8_t>(v >> 16);
        pw[4] = static_cast<uint8_t>(v >> 24);
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

template <int MODE>
__global__ void __launch_bounds__(kThreads) crc32c_rows_kernel(BlockArgs a) {
  crc32c_rows_body<MODE, 0, 1>(a);
}
// raw batches smaller than one 64-descriptor chunk per wave of the grid (the
// records a WAL recovery's fused kernel does not cover, a WAL write of a few
// records): the global feed would hand them to a few waves in 64-descriptor
// chunks, 64 records one after another on each, while the workgroup feed
// spreads them over every wave in 4-descriptor batches
__global__ void __launch_bounds__(kThreads) crc32c_rows_raw_small_kernel(BlockArgs a) {
  crc32c_rows_body<kModeRaw, 0, 1, true>(a);
}
// the long messages of a raw batch (kRawSplit bytes or more)
__global__ void __launch_bounds__(kThreads) crc32c_rows_raw_filt_kernel(BlockArgs a) {
  crc32c_rows_body<kModeRaw, 0, 1, false, true>(a);
}

// ---- the short messages of a raw batch: one message per lane --------------
// crc32c::Value(init, p, n) of a message of n < kRawSplit bytes by lane-serial
// slicing-by-4 on the G tables (the rows kernel's layout, rows of 256 bytes,
// so each ds_read of a wave is bank-conflict free).  16-byte loads, one in
// flight ahead of the dwords being folded.  The first dword starts the chain
// at S0 (~init moved back over the m = p & 3 bytes in front of the message,
// which are masked to zero), as the rows kernel's head lane does.
constexpr uint32_t kLaneThreads = 512;
// 16-byte loads of a short message: its bytes from the dword boundary in
// front (m <= 3) plus the tail dword
constexpr uint32_t kLaneChunks = (kRawSplit + 2 + 4 + 15) / 16;
__device__ __forceinline__ uint32_t lane_raw_crc(const uint8_t* __restrict__ Lb, const Lanes2& K,
                                                 const uint8_t* base, uint64_t base_len,
                                                 uint64_t off, uint32_t n, uint32_t init,
                                                 bool has_init) {
  const uint32_t m = static_cast<uint32_t>(off & 3);
  const uint32_t tot = n + m;  // bytes from the dword boundary in front
  const uint32_t nd = tot >> 2, nt = tot & 3;
  const uint32_t nc = (nd + (nt ? 1u : 0u) + 3) >> 2;  // 16-byte loads
  // messages within their first dword, and the last bytes of the buffer:
  // dword-serial with byte loads at either end (never a byte past it)
  if (nd == 0 || (off - m) + 16ull * nc > base_len)
    return small_crc2(Lb, K, base + off, n, init, 0, 0);
  const uint8_t* q = base + (off - m);
  const uint32_t S0 = has_init ? unstep_m(~init, m)
                               : m == 0 ? 0xffffffffu : m == 1 ? 0xa942e6bcu
                               : m == 2 ? 0x2804363bu : 0x96db52a8u;  // kCrcS0
  const uint32_t bm = 0xffffffffu << (8 * m);
  const uint32_t tm = (1u << (8 * nt)) - 1u;
  uint32_t s = 0;
  // every load of the message first (one memory latency per message; a
  // chunk-by-chunk loop waited one per 16 bytes: C5's 3.4 M short records
  // took 0.42 ms that way), then the chain over them
  u32x4a4 v[kLaneChunks];
#pragma unroll
  for (uint32_t c = 0; c < kLaneChunks; ++c)
    v[c] = c < nc ? ld16_a4(q + 16 * c) : u32x4a4{0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t c = 0; c < kLaneChunks; ++c) {
    if (c < nc) {
      const uint32_t w[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t i = 4 * c + j;
        if (i < nd)
          s = rep_map<false>(Lb, K, i == 0 ? ((w[j] & bm) ^ S0) : (s ^ w[j]));
        else if (i == nd && nt)
          s = step_k(Lb, K, s, w[j] & tm, nt);
      }
    }
  }
  return ~s;
}

// every descriptor of the batch that is not raw_long (the rows filter
// kernel takes those); the same results and stores as the rows kernel's
// raw mode (wal_hs masking, expect: only differing results stored, an
// out-of-range descriptor reported as 0).  Each wave takes windows of
// kRawLaneR x 64 descriptors on its own (no workgroup barrier): it loads
// them all at once, lists the short ones' window positions in its LDS slots
// (on C5 at a 256-byte split 3 records in 10 are short) and gives them out
// one per lane, the descriptor fields moved between lanes by ds_bpermute.
// Latency bound, so waves independent: workgroup-wide windows with
// barriers, and one descriptor per thread, measured 0.36 / 0.42 ms on C5
// against this layout's.
constexpr uint32_t kRawLaneR = 4;
constexpr uint32_t kRawLaneWaves = kLaneThreads / 64;
__global__ void __launch_bounds__(kLaneThreads) crc32c_raw_lane_kernel(BlockArgs a) {
  __shared__ uint32_t L[16384];
  __shared__ uint16_t slot[kRawLaneWaves][kRawLaneR * 64];
  for (uint32_t i = threadIdx.x; i < 16384; i += kLaneThreads) {
    const uint32_t e = i >> 6, d = i & 63;
    if (d < 32) L[i] = kCrcG[((d >> 3) & 3) * 256 + e];
  }
  __syncthreads();
  const uint8_t* Lb = reinterpret_cast<const uint8_t*>(L);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const Lanes2 K = lanes2(lane);
  const uint64_t below = (1ull << lane) - 1;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * kRawLaneWaves;
  constexpr uint64_t W = uint64_t(kRawLaneR) * 64;
  uint16_t* sl = slot[wave];
  for (uint64_t w0 = (static_cast<uint64_t>(blockIdx.x) * kRawLaneWaves + wave) * W; w0 < a.n;
       w0 += nw * W) {
    uint32_t olo[kRawLaneR], ohi[kRawLaneR], sz[kRawLaneR];
#pragma unroll
    for (uint32_t r = 0; r < kRawLaneR; ++r) {  // every load first
      uint64_t i = w0 + 64 * r + lane;
      i = i < a.n ? i : a.n - 1;
      const uint64_t off = a.offsets[i];
      olo[r] = static_cast<uint32_t>(off);
      ohi[r] = static_cast<uint32_t>(off >> 32);
      sz[r] = a.sizes[i];
    }
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t r = 0; r < kRawLaneR; ++r) {
      uint64_t off = (static_cast<uint64_t>(ohi[r]) << 32) | olo[r];
      uint32_t size = sz[r];
      if (a.wal_hs) {  // (as load_batch: header offset + payload length)
        const bool ok = off <= a.base_len && a.base_len - off >= uint64_t(a.wal_hs) + size;
        off = ok ? off + 6 : ~0ull;
        size = ok ? a.wal_hs + size - 6 : 0u;
        olo[r] = static_cast<uint32_t>(off);
        ohi[r] = static_cast<uint32_t>(off >> 32);
        sz[r] = size;
      }
      const bool sh = w0 + 64 * r + lane < a.n && !raw_long(off, size);
      const uint64_t m = __ballot(sh);
      if (sh) sl[cnt + static_cast<uint32_t>(__popcll(m & below))] = static_cast<uint16_t>(64 * r + lane);
      cnt += static_cast<uint32_t>(__popcll(m));
    }
    wave_lds_sync();
    for (uint32_t j0 = 0; j0 < cnt; j0 += 64) {  // (wave-uniform: the bpermutes need every lane)
      const uint32_t j = j0 + lane;
      const uint32_t q = j < cnt ? sl[j] : 0u;
      const int src = static_cast<int>(4 * (q & 63));
      uint32_t lo = 0, hi = 0, size = 0;
#pragma unroll
      for (uint32_t r = 0; r < kRawLaneR; ++r) {
        const uint32_t vlo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(olo[r])));
        const uint32_t vhi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(ohi[r])));
        const uint32_t vsz = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sz[r])));
        if ((q >> 6) == r) {
          lo = vlo;
          hi = vhi;
          size = vsz;
        }
      }
      if (j < cnt) {
        const uint64_t i = w0 + q;
        const uint64_t off = (static_cast<uint64_t>(hi) << 32) | lo;
        const bool valid = desc_in_range<kModeRaw>(a, Desc{off, size, 0, 0});
        const uint32_t init = a.init_crcs ? a.init_crcs[i] : 0u;
        uint32_t v = 0;
        if (valid) {
          const uint32_t crc = lane_raw_crc(Lb, K, a.base, a.base_len, off, size, init,
                                            a.init_crcs != nullptr);
          v = a.wal_hs ? crc_mask(crc) : crc;
        }
        const bool differs = !a.expect || !valid || v != a.expect[i];
        if (differs && a.out32) a.out32[i] = v;
      }
    }
    wave_lds_sync();  // (the slots are rewritten by the next window)
  }
}

#ifdef FORST_DIAG
template <int PROBE>
__global__ void __launch_bounds__(kThreads) crc32c_rows_probe_kernel(BlockArgs a) {
  crc32c_rows_body<kModeVerify, PROBE, 1>(a);
}
template <int MODE>
__global__ void __launch_bounds__(64 * kRowsD2Waves) crc32c_rows_d2_kernel(BlockArgs a) {
  crc32c_rows_body<MODE, 0, 2>(a);
}
__global__ void __launch_bounds__(64 * kRowsD2Waves) crc32c_rows_d2_probe_kernel(BlockArgs a) {
  crc32c_rows_body<kModeVerify, 1, 2>(a);
}

// Access-pattern probe (diagnostics only, FORST_CRC_VARIANT=pat<G>_<C>): no
// CRC work, no work feed.  Groups of G lanes (16 = a row, 64 = the wave) walk
// their blocks (static: group k of the grid takes blocks k, k + ngroups, ...)
// in C-byte steps, one step of loads in flight ahead of an XOR of the
// current one: the memory ceiling of "C contiguous bytes per group per step"
// against the rows kernel's 1 KiB per row and the v2 kernel's 4 KiB per wave.
// The plain streaming ceiling (diagnostics only, FORST_CRC_VARIANT=stream):
// the whole buffer read once, every wave a contiguous 4 KiB per step (16 B
// per lane, 4 loads per lane in flight), grid-stride, no descriptors.
__global__ void __launch_bounds__(kThreads) crc32c_stream_probe_kernel(BlockArgs a) {
  const uint64_t nthr = static_cast<uint64_t>(gridDim.x) * kThreads;
  const uint64_t n16 = a.base_len / 16;
  uint32_t acc = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n16;
       i += 4 * nthr) {
    u32x4a4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t j = i + k * nthr;
      v[k] = ld16_a4(a.base + 16 * (j < n16 ? j : i));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (a.out32 && threadIdx.x == 0) a.out32[blockIdx.x] = acc;
}

template <int G, int C>
__global__ void __launch_bounds__(kThreads) crc32c_pattern_probe_kernel(BlockArgs a) {
  constexpr int kPer = C / G / 16;  // 16-byte loads per lane per step
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t gl = lane % G;
  const uint64_t ng = static_cast<uint64_t>(gridDim.x) * (kThreads / G);
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * (kThreads / G) + threadIdx.x / G;
  uint32_t acc = 0;
  for (uint64_t b = g0; b < a.n; b += ng) {
    const uint64_t off = a.offsets[b] & ~15ull;
    const uint32_t sz = a.sizes[b];
    const uint32_t steps = (sz + 16 + C - 1) / C;
    u32x4a4 cur[kPer], nxt[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) cur[k] = ld16_a4(a.base + off + 16 * (gl + G * k));
    for (uint32_t st = 0; st < steps; ++st) {
      const uint64_t o2 = off + static_cast<uint64_t>(st + 1 < steps ? st + 1 : st) * C;
#pragma unroll
      for (int k = 0; k < kPer; ++k) nxt[k] = ld16_a4(a.base + o2 + 16 * (gl + G * k));
#pragma unroll
      for (int k = 0; k < kPer; ++k) acc ^= cur[k].x ^ cur[k].y ^ cur[k].z ^ cur[k].w;
#pragma unroll
      for (int k = 0; k < kPer; ++k) cur[k] = nxt[k];
    }
    if (gl == 0 && a.out32) a.out32[b] = acc;
  }
}
#endif

// One wave per block, no streaming: serves buffers shorter than one 4 KiB
// round (the streaming kernels' dummy loads need that much).
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

namespace {

enum class CrcKernel {
  kSimple,  // one wave per block: buffers shorter than one 4 KiB round
  kRows,    // one block per 16-lane row (crc32c_rows_kernel)
  kV2,      // one block per wave, two chains per lane (crc32c_stream2_kernel)
#ifdef FORST_DIAG
  kV1, kRowsD2, kRowsProbeLoad, kRowsProbeNoFin, kRowsD2ProbeLoad, kRowsProbeContig, kV2ProbeLoad, kV2ProbeRounds, kV2ProbeNoHead,
  kPat16_1k, kPat16_2k, kPat16_4k, kPat64_4k, kStream,
#endif
};

hipError_t launch_kernel(void (*k)(BlockArgs), uint32_t grid, uint32_t threads, BlockArgs a,
                         hipStream_t s) {
  hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 0, s, a);
  return hipGetLastError();
}

// a rows-kernel launch with its work-feed counter (stream_common.h)
hipError_t launch_fed(void (*k)(BlockArgs), uint32_t grid, uint32_t waves, BlockArgs b,
                      hipStream_t s) {
  hipError_t e = feed_setup(b, uint64_t(grid) * waves, s);
  if (e != hipSuccess) return e;
  e = launch_kernel(k, grid, 64 * waves, b, s);
  const hipError_t f = scratch_free(b.ticket, s);
  return e != hipSuccess ? e : f;
}

const char* crc_kernel_name(CrcKernel k, int mode) {
  static const char* const kNames[][4] = {
      {"crc32c_block_kernel_simple<compute>", "crc32c_block_kernel_simple<trailer>",
       "crc32c_block_kernel_simple<verify>", "crc32c_block_kernel_simple<raw>"},
      {"crc32c_rows_kernel<compute>", "crc32c_rows_kernel<trailer>", "crc32c_rows_kernel<verify>",
       "crc32c_rows_kernel<raw>"},
      {"crc32c_stream2_kernel<compute>", "crc32c_stream2_kernel<trailer>",
       "crc32c_stream2_kernel<verify>", "crc32c_stream2_kernel<raw>"},
#ifdef FORST_DIAG
      {"crc32c_stream_kernel<compute>", "crc32c_stream_kernel<trailer>",
       "crc32c_stream_kernel<verify>", "crc32c_stream_kernel<raw>"},
      {"crc32c_rows_d2_kernel<compute>", "crc32c_rows_d2_kernel<trailer>",
       "crc32c_rows_d2_kernel<verify>", "crc32c_rows_d2_kernel<raw>"},
#endif
  };
#ifdef FORST_DIAG
  switch (k) {
    case CrcKernel::kRowsProbeLoad: return "crc32c_rows_probe_kernel<1>";
    case CrcKernel::kRowsProbeNoFin: return "crc32c_rows_probe_kernel<2>";
    case CrcKernel::kRowsD2ProbeLoad: return "crc32c_rows_d2_probe_kernel";
    case CrcKernel::kRowsProbeContig: return "crc32c_rows_probe_kernel<3>";
    case CrcKernel::kPat16_1k: return "crc32c_pattern_probe_kernel<16,1024>";
    case CrcKernel::kPat16_2k: return "crc32c_pattern_probe_kernel<16,2048>";
    case CrcKernel::kPat16_4k: return "crc32c_pattern_probe_kernel<16,4096>";
    case CrcKernel::kPat64_4k: return "crc32c_pattern_probe_kernel<64,4096>";
    case CrcKernel::kStream: return "crc32c_stream_probe_kernel";
    case CrcKernel::kV2ProbeLoad: return "crc32c_stream2_probe_kernel<1>";
    case CrcKernel::kV2ProbeRounds: return "crc32c_stream2_probe_kernel<2>";
    case CrcKernel::kV2ProbeNoHead: return "crc32c_stream2_probe_kernel<3>";
    default: break;
  }
#endif
  return kNames[static_cast<int>(k)][mode & 3];
}

#ifndef FORST_CRC_BLOCK_COST
#define FORST_CRC_BLOCK_COST 0
#endif
template <int M>
hipError_t launch_crc_mode(CrcKernel k, const BlockArgs& a, uint32_t grid, hipStream_t s) {
  switch (k) {
    case CrcKernel::kSimple:
      return launch_kernel(crc32c_block_kernel_simple<M>, grid, kThreads, a, s);
    case CrcKernel::kRows:
      // block modes: the workgroup feed (stream_common.h), no ticket counter
      if (M != kModeRaw) {
        BlockArgs b = a;
        b.wg_cost = FORST_CRC_BLOCK_COST;  // (stream_common.h wg_range)
        return launch_kernel(crc32c_rows_kernel<M>, grid, 64 * kWaves, b, s);
      }
      if (a.n < uint64_t(64) * grid * kWaves)
        return launch_kernel(crc32c_rows_raw_small_kernel, grid, 64 * kWaves, a, s);
      if constexpr (M == kModeRaw && kRawSplit > 0) {
        // short messages one per lane, then the rows kernel over the rest
        const hipError_t e = launch_kernel(crc32c_raw_lane_kernel, 2 * device_info().num_cus,
                                           kLaneThreads, a, s);
        if (e != hipSuccess) return e;
        return launch_fed(crc32c_rows_raw_filt_kernel, grid, kWaves, a, s);
      }
      return launch_fed(crc32c_rows_kernel<M>, grid, kWaves, a, s);
    case CrcKernel::kV2:
      return launch_kernel(crc32c_stream2_kernel<M>, grid, kThreads, a, s);
#ifdef FORST_DIAG
    case CrcKernel::kV1:
      return launch_kernel(crc32c_stream_kernel<M>, grid, kThreads, a, s);
    case CrcKernel::kRowsD2:
      return launch_fed(crc32c_rows_d2_kernel<M>, grid, kRowsD2Waves, a, s);
    case CrcKernel::kRowsProbeLoad:
      return launch_fed(crc32c_rows_probe_kernel<1>, grid, kWaves, a, s);
    case CrcKernel::kRowsProbeNoFin:
      return launch_fed(crc32c_rows_probe_kernel<2>, grid, kWaves, a, s);
    case CrcKernel::kRowsD2ProbeLoad:
      return launch_fed(crc32c_rows_d2_probe_kernel, grid, kRowsD2Waves, a, s);
    case CrcKernel::kRowsProbeContig:
      return launch_fed(crc32c_rows_probe_kernel<3>, grid, kWaves, a, s);
    case CrcKernel::kPat16_1k:
      hipLaunchKernelGGL((crc32c_pattern_probe_kernel<16, 1024>), dim3(grid), dim3(kThreads), 0, s, a);
      return hipGetLastError();
    case CrcKernel::kPat16_2k:
      hipLaunchKernelGGL((crc32c_pattern_probe_kernel<16, 2048>), dim3(grid), dim3(kThreads), 0, s, a);
      return hipGetLastError();
    case CrcKernel::kPat16_4k:
      hipLaunchKernelGGL((crc32c_pattern_probe_kernel<16, 4096>), dim3(grid), dim3(kThreads), 0, s, a);
      return hipGetLastError();
    case CrcKernel::kPat64_4k:
      hipLaunchKernelGGL((crc32c_pattern_probe_kernel<64, 4096>), dim3(grid), dim3(kThreads), 0, s, a);
      return hipGetLastError();
    case CrcKernel::kStream:
      hipLaunchKernelGGL(crc32c_stream_probe_kernel, dim3(4 * grid), dim3(kThreads), 0, s, a);
      return hipGetLastError();
    case CrcKernel::kV2ProbeLoad:
      return launch_kernel(crc32c_stream2_probe_kernel<1>, grid, kThreads, a, s);
    case CrcKernel::kV2ProbeRounds:
      return launch_kernel(crc32c_stream2_probe_kernel<2>, grid, kThreads, a, s);
    case CrcKernel::kV2ProbeNoHead:
      return launch_kernel(crc32c_stream2_probe_kernel<3>, grid, kThreads, a, s);
#endif
  }
  return hipErrorInvalidValue;
}

#ifdef FORST_DIAG
// diagnostics build: FORST_CRC_VARIANT overrides the kernel choice (probe
// variants only replace verify launches; their results are not checksums)
CrcKernel diag_crc_kernel(CrcKernel k, int mode) {
  const std::string v = diag_env("FORST_CRC_VARIANT");
  const bool vf = mode == kModeVerify;
  if (v == "simple") return CrcKernel::kSimple;
  if (v == "rows") return CrcKernel::kRows;
  if (v == "v2") return CrcKernel::kV2;
  if (v == "v1") return CrcKernel::kV1;
  if (v == "rows_d2") return CrcKernel::kRowsD2;
  if (v == "rows_probe_load" && vf) return CrcKernel::kRowsProbeLoad;
  if (v == "rows_probe_nofin" && vf) return CrcKernel::kRowsProbeNoFin;
  if (v == "rows_d2_probe_load" && vf) return CrcKernel::kRowsD2ProbeLoad;
  if (v == "rows_probe_contig" && vf) return CrcKernel::kRowsProbeContig;
  if (v == "pat16_1k" && vf) return CrcKernel::kPat16_1k;
  if (v == "pat16_2k" && vf) return CrcKernel::kPat16_2k;
  if (v == "pat16_4k" && vf) return CrcKernel::kPat16_4k;
  if (v == "pat64_4k" && vf) return CrcKernel::kPat64_4k;
  if (v == "stream" && vf) return CrcKernel::kStream;
  if (v == "probe_load" && vf) return CrcKernel::kV2ProbeLoad;
  if (v == "probe_rounds" && vf) return CrcKernel::kV2ProbeRounds;
  if (v == "probe_nohead" && vf) return CrcKernel::kV2ProbeNoHead;
  return k;
}
#endif

}  // namespace

// raw CRCs of messages all under kRawSplit bytes: the lane kernel alone (a
// longer one would be left out: the caller guarantees the lengths)
hipError_t launch_crc32c_raw_lanes(const BlockArgs& a, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  if (kRawSplit < 256) return hipErrorInvalidValue;
  return launch_kernel(crc32c_raw_lane_kernel, 2 * device_info().num_cus, kLaneThreads, a, stream);
}

hipError_t launch_crc32c_blocks(int mode, const BlockArgs& a, hipStream_t stream,
                                const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n == 0) return hipSuccess;
  uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((a.n + kWaves - 1) / kWaves, di.num_cus));
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
  // The rows kernel (one block per 16-lane row) for every block size.  In
  // round 1 the v2 kernel (one block per wave, two 4 KiB steps in flight)
  // won above 8-20 KiB; with the workgroup feed (stream_common.h) the rows
  // kernel matches or beats it everywhere (profiles/ab_r02_late/
  // rows_vs_v2_wgfeed.log, same box: 64 KiB 0.740 vs 0.736, the 4/16/64 KiB
  // mix 0.726 vs 0.666, 512 K x 16 KiB 0.748 vs 0.705).  v2 remains for
  // batches of 2^32 - 1 or more descriptors (the rows kernel indexes them
  // with 32 bits).  Buffers shorter than one 4 KiB round take the simple
  // kernel (the streaming kernels' dummy loads read [0, 4 KiB)).
  CrcKernel k = a.base_len < kRB ? CrcKernel::kSimple
                : (a.n < 0xffffffffull && (a.kernel_hint ? a.kernel_hint == 1 : true))
                    ? CrcKernel::kRows
                    : CrcKernel::kV2;
#ifdef FORST_DIAG
  // (never for the WAL writer mode: only the rows kernel masks its CRCs)
  if (a.base_len >= kRB && !a.wal_hs) k = diag_crc_kernel(k, mode);
  if (k == CrcKernel::kRows || k == CrcKernel::kRowsD2) {
    if (a.n >= 0xffffffffull) k = CrcKernel::kV2;
  }
#endif
  // the WAL writer mode (wal_hs: header offsets + payload lengths, masked
  // output) exists in the rows kernel only
  if (a.wal_hs && (mode != kModeRaw || k != CrcKernel::kRows)) return hipErrorInvalidValue;
  *name = crc_kernel_name(k, mode);
  if (k == CrcKernel::kRows && mode == kModeRaw)
    *name = a.n < uint64_t(64) * grid * kWaves ? "crc32c_rows_raw_small_kernel"
            : kRawSplit > 0                    ? "crc32c_rows_raw_filt_kernel"
                                               : "crc32c_rows_kernel<raw>";
  switch (mode) {
    case kModeCompute:
      return launch_crc_mode<kModeCompute>(k, a, grid, stream);
    case kModeTrailer:
      return launch_crc_mode<kModeTrailer>(k, a, grid, stream);
    case kModeVerify:
      return launch_crc_mode<kModeVerify>(k, a, grid, stream);
    default:
      return launch_crc_mode<kModeRaw>(k, a, grid, stream);
  }
}

#ifdef FORST_DIAG
// ---------------------------------------------------------------------------
// WAL, one wave per log block / record (diagnostics build only: A/B reference
// of the wal.hip pipeline; db/log_reader.cc:450-531, db/log_writer.cc:228-263)
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

hipError_t launch_wal_verify_wave(const WalArgs& a, hipStream_t stream,
                             const char** name) {
  const DeviceInfo& di = device_info();
  if (a.n_blocks == 0) return hipSuccess;
  uint32_t grid = static_cast<uint32_t>(
      std::min<uint64_t>((a.n_blocks + kWaves - 1) / kWaves, di.num_cus));
  *name = "wal_verify_kernel";
  hipLaunchKernelGGL(wal_verify_kernel, dim3(grid), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_wal_record_crc_wave(const WalArgs& a, hipStream_t stream,
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

#endif  // FORST_DIAG

}  // namespace forst

#ifdef FORST_DIAG
// diagnostics build only: per-wave start / end clocks of the last rows launch
extern "C" __attribute__((visibility("default"))) int forst_diag_wave_times(
    unsigned long long* t0, unsigned long long* t1, unsigned n) {
  if (n > forst::kDiagWaves) n = forst::kDiagWaves;
  if (hipMemcpyFromSymbol(t0, HIP_SYMBOL(forst::g_wave_t0), n * 8) != hipSuccess) return -3;
  if (hipMemcpyFromSymbol(t1, HIP_SYMBOL(forst::g_wave_t1), n * 8) != hipSuccess) return -3;
  return 0;
}
#endif

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
