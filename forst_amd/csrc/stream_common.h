// forst_amd/csrc/stream_common.h -- pieces shared by the streaming block
// kernels (crc32c.hip, xxh3.hip): per-wave contiguous shares, 64-entry
// descriptor batches held one block per lane, and v_readlane helpers.
//
// A streaming kernel keeps one step of global loads in flight while it
// computes the previous one.  That only works if no other VMEM load is
// waited for in between (s_waitcnt vmcnt counts in issue order), so block
// descriptors are fetched 64 at a time into VGPRs (lane j <-> block kb+j) and
// read back into SGPRs with v_readlane; results are collected the same way
// and stored once per batch.
#pragma once
#include "device_common.h"
#include "engine.h"

namespace forst {

constexpr uint32_t kBatch = 64;

__device__ __forceinline__ uint32_t readlane32(uint32_t v, uint32_t l) {
  // (the builtin returns int: cast before any widening, or it sign-extends)
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(l)));
}
__device__ __forceinline__ uint64_t readlane64(uint32_t lo, uint32_t hi, uint32_t l) {
  return (static_cast<uint64_t>(readlane32(hi, l)) << 32) | readlane32(lo, l);
}


// [kbeg, kend): wave gw's contiguous share of n blocks over nw waves
__device__ __forceinline__ void wave_share(uint64_t n, uint64_t nw, uint64_t gw, uint64_t& kbeg,
                                           uint64_t& kend) {
  const uint64_t q = n / nw, rem = n % nw;
  kbeg = gw * q + (gw < rem ? gw : rem);
  kend = kbeg + q + (gw < rem ? 1 : 0);
}

// Global work feed of the rows kernels (WG = false): a wave consumes a stream
// of 64-descriptor batches -- first its static share [gw * share1, (gw + 1) * share1)
// (share1 a multiple of 64, nw * share1 <= n), then 64-descriptor chunks
// starting at nw * share1 + 64 * t, t claimed from a.ticket (one atomic per
// chunk; a wave whose blocks ran long simply claims fewer chunks), or dealt
// round-robin (t = gw, gw + nw, ...) when the launch has no ticket counter
// (a.ticket points at 64 counters, [0] zeroed per launch).
// Chunks never straddle a batch, so a batch is one contiguous run
// [g, g + 64) of descriptors (entries >= n are empty).  Once a batch starts
// at >= n every later one does too and the feed stops claiming.
struct BatchFeed {
  uint64_t g;    // start of the last batch handed out
  uint64_t lim;  // end of the static share / chunk it belongs to
  uint64_t rr;   // round-robin ticket (no counter)
  uint64_t wlo, whi;  // workgroup feed: this workgroup's descriptor range
  uint32_t len;  // entries of the last batch handed out (0 once exhausted)
};

__device__ __forceinline__ void feed_set_len(const BlockArgs& a, BatchFeed& f) {
  const uint64_t e = f.lim < a.n ? f.lim : a.n;
  const uint64_t l = f.g < e ? e - f.g : 0;
  f.len = static_cast<uint32_t>(l < kBatch ? l : kBatch);
}

__device__ __forceinline__ uint64_t feed_claim_global(const BlockArgs& a, uint64_t nw,
                                                      uint32_t lane, BatchFeed& f) {
  uint64_t t;
  if (a.ticket) {
    // the whole wave issues the atomic (no divergent branch in the hot loop):
    // lane 0 claims on ticket[0], the other lanes add 0 to their own slots
    // (the address is formed here, not hoisted out of the kernel's loop: a
    // loop-invariant VGPR pair the register allocator would have to keep)
    const uint32_t l = lane + vzero();
    const unsigned long long v = atomicAdd(a.ticket + l, l == 0 ? 1ull : 0ull);
    t = uniform64(v);
  } else {
    t = f.rr;
    f.rr += nw;
  }
  f.g = nw * a.share1 + static_cast<uint64_t>(kBatch) * t;
  f.lim = f.g + kBatch;
  feed_set_len(a, f);
  return f.g;
}

// Workgroup feed (WG = true; the rows kernels' block modes): workgroup b owns
// a contiguous descriptor range [L(b), L(b + 1)) of about 1/G of the batch's
// BYTES (wg_range below), and its waves take CHUNK-descriptor batches of it
// from an LDS counter.
// - An LDS atomic waits on lgkmcnt only, so a claim does not drain the
//   wave's loads in flight (a global claim does: vmcnt(0)).
// - The small grain lets the fast and slow waves of a SIMD finish together.
//   The four waves of a SIMD progress at different rates (age-ordered), and
//   the global feed's last 64-descriptor chunk left them idle for 7-13 % of a
//   C2 launch (tools/wave_tail.py).
// - Ranges by bytes, not by count (round 3): a batch sorted or clustered by
//   block size (64 KiB blocks, then 4 KiB; an arena of SST files with
//   different block sizes) would otherwise give some workgroups many times
//   the bytes of others.
constexpr uint32_t kWgChunk = 16;
__device__ __forceinline__ uint32_t* feed_lds_ctr() {
  __shared__ uint32_t ctr;
  return &ctr;
}
// zeroes the workgroup counter: before the kernel's first __syncthreads
__device__ __forceinline__ void feed_init() {
  if (threadIdx.x == 0) *feed_lds_ctr() = 0;
}

// off0 + floor(span * b / G) without 128-bit arithmetic
__device__ __forceinline__ uint64_t frac_point(uint64_t off0, uint64_t span, uint64_t b,
                                               uint64_t G) {
  return off0 + (span / G) * b + ((span % G) * b) / G;
}

// L(b): the number of descriptors "before" byte target t, by a 64-ary
// COUNTING search over offsets[] -- at each level the next segment is chosen
// by how many of the 63 probes lie below t, which is non-decreasing in t for
// any order of the array.  So L is monotone in b and [L(b), L(b+1)) tiles
// [0, n) exactly whatever the descriptors; when they are in file order (an
// SST, an arena of SSTs) it is lower_bound and the ranges are byte-balanced.
// Both bounds of the workgroup are searched together (their loads overlap):
// ceil(log64 n) dependent rounds, 4 for 1 M descriptors.
__device__ __forceinline__ void wg_range(const BlockArgs& a, uint32_t lane, uint64_t* lo_out,
                                         uint64_t* hi_out) {
  const uint64_t n = a.n, G = gridDim.x, b = blockIdx.x;
  // key of descriptor i: offsets[i] + c i -- each block weighs its bytes plus
  // c bytes for its per-block work (set-up, finish), so a range of small
  // blocks gets fewer bytes than a range of large ones
  const uint64_t c = a.wg_cost;
  const uint64_t off0 = a.offsets[0];
  const uint64_t last = a.offsets[n - 1] + a.sizes[n - 1] + c * (n - 1);
  if (last <= off0 || G == 1) {  // no byte span to split: by count
    const uint64_t W = (n + G - 1) / G;
    *lo_out = b * W < n ? b * W : n;
    *hi_out = (b + 1) * W < n ? (b + 1) * W : n;
    return;
  }
  const uint64_t span = last - off0;
  const uint64_t t0 = frac_point(off0, span, b, G), t1 = frac_point(off0, span, b + 1, G);
  uint64_t lo0 = 0, len0 = n, lo1 = 0, len1 = n;
  while (len0 > 64 || len1 > 64) {
    const uint64_t st0 = (len0 + 63) / 64, st1 = (len1 + 63) / 64;
    const uint64_t q0 = lo0 + lane * st0, q1 = lo1 + lane * st1;
    const bool v0 = len0 > 64 && lane > 0 && q0 < lo0 + len0;
    const bool v1 = len1 > 64 && lane > 0 && q1 < lo1 + len1;
    const uint64_t k0 = a.offsets[v0 ? q0 : 0] + c * q0, k1 = a.offsets[v1 ? q1 : 0] + c * q1;
    const uint64_t c0 = static_cast<uint64_t>(__popcll(__ballot(v0 && k0 < t0)));
    const uint64_t c1 = static_cast<uint64_t>(__popcll(__ballot(v1 && k1 < t1)));
    if (len0 > 64) {
      const uint64_t e = lo0 + len0;
      lo0 += c0 * st0;
      len0 = e - lo0 < st0 ? e - lo0 : st0;
    }
    if (len1 > 64) {
      const uint64_t e = lo1 + len1;
      lo1 += c1 * st1;
      len1 = e - lo1 < st1 ? e - lo1 : st1;
    }
  }
  const bool f0 = lane < len0, f1 = lane < len1;
  const uint64_t k0 = a.offsets[f0 ? lo0 + lane : 0] + c * (lo0 + lane),
                 k1 = a.offsets[f1 ? lo1 + lane : 0] + c * (lo1 + lane);
  const uint64_t L0 = lo0 + static_cast<uint64_t>(__popcll(__ballot(f0 && k0 < t0)));
  const uint64_t L1 = lo1 + static_cast<uint64_t>(__popcll(__ballot(f1 && k1 < t1)));
  *lo_out = b == 0 ? 0 : uniform64(L0);
  *hi_out = b + 1 == G ? n : uniform64(L1);
}

template <uint32_t CHUNK>
__device__ __forceinline__ uint64_t feed_claim_wg(const BlockArgs& a, uint32_t lane,
                                                  BatchFeed& f) {
  uint32_t p = 0;
  if (lane == 0) p = atomicAdd(feed_lds_ctr(), CHUNK);
  p = readlane32(p, 0);
  f.g = f.wlo + p;
  if (f.g >= f.whi) {
    f.g = a.n;  // exhausted (stays so)
    f.len = 0;
  } else {
    f.len = static_cast<uint32_t>(f.whi - f.g < CHUNK ? f.whi - f.g : CHUNK);
  }
  f.lim = f.g + f.len;
  return f.g;
}

// WG: the workgroup feed in CHUNK-descriptor batches (16 for blocks of KiBs;
// items of a few hundred bytes take 64: fewer batch loads per byte)
template <bool WG, uint32_t CHUNK = kWgChunk>
__device__ __forceinline__ uint64_t feed_first(const BlockArgs& a, uint64_t nw, uint64_t gw,
                                               uint32_t lane, BatchFeed& f) {
  f.rr = gw;
  if (WG) {
    wg_range(a, lane, &f.wlo, &f.whi);
    return feed_claim_wg<CHUNK>(a, lane, f);
  }
  if (a.share1 == 0) return feed_claim_global(a, nw, lane, f);
  f.g = gw * a.share1;
  f.lim = f.g + a.share1;
  feed_set_len(a, f);
  return f.g;
}

template <bool WG, uint32_t CHUNK = kWgChunk>
__device__ __forceinline__ uint64_t feed_next(const BlockArgs& a, uint64_t nw, uint32_t lane,
                                              BatchFeed& f) {
  if (f.g >= a.n) {  // exhausted: stays exhausted, no more claims
    f.len = 0;
    return f.g;
  }
  if (WG) return feed_claim_wg<CHUNK>(a, lane, f);
  f.g += kBatch;
  if (f.g < f.lim) {
    feed_set_len(a, f);
    return f.g;
  }
  return feed_claim_global(a, nw, lane, f);
}

// where stream position rel lies in the (current, next) batch pair of
// lengths clen / nlen: the source lane, which batch, the descriptor index and
// whether it exists
struct BatchSlot {
  int src;
  bool in_n, valid;
  uint64_t gi;
};
__device__ __forceinline__ BatchSlot batch_slot(uint64_t rel, uint64_t kbrel, uint64_t cg,
                                                uint32_t clen, uint64_t ng, uint32_t nlen,
                                                uint64_t n) {
  const uint32_t j = static_cast<uint32_t>(rel - kbrel);
  BatchSlot b;
  b.in_n = j >= clen;
  const uint32_t k = b.in_n ? j - clen : j;
  b.src = static_cast<int>(k & 63u);
  b.gi = (b.in_n ? ng : cg) + k;
  b.valid = k < (b.in_n ? nlen : clen) && b.gi < n;
  return b;
}

// per-lane descriptor batch (lane j <-> block kb + j)
struct DescBatch {
  uint32_t off_lo, off_hi, size, mod, extra;  // extra: last byte, or init (raw CRC)
};

template <int MODE>
__device__ __forceinline__ void load_batch(const BlockArgs& a, uint64_t kb, uint64_t kend,
                                           uint32_t lane, DescBatch& d) {
  uint64_t i = kb + lane;
  i = i < kend ? i : kend - 1;  // clamped: the loads are unconditional
  uint64_t off = a.offsets[i];
  uint32_t size = a.sizes[i];
  if (MODE == kModeRaw && a.wal_hs) {  // WAL writer mode: header offset + payload length
    const bool ok = off <= a.base_len && a.base_len - off >= uint64_t(a.wal_hs) + size;
    off = ok ? off + 6 : ~0ull;  // (out of range: reported, never read)
    size = ok ? a.wal_hs + size - 6 : 0u;
  }
  d.off_lo = static_cast<uint32_t>(off);
  d.off_hi = static_cast<uint32_t>(off >> 32);
  d.size = size;
  const uint32_t* mp = a.modifiers ? a.modifiers : a.sizes;
  const uint32_t mv = mp[i];
  d.mod = a.modifiers ? mv : 0u;
  if (MODE == kModeRaw) {
    const uint32_t* ip = a.init_crcs ? a.init_crcs : a.sizes;
    const uint32_t iv = ip[i];
    d.extra = a.init_crcs ? iv : 0u;
  } else {
    const uint8_t* lp = a.last_bytes ? a.last_bytes : reinterpret_cast<const uint8_t*>(a.sizes);
    d.extra = lp[i];
  }
}

// Length-split batches (the raw CRC rows kernel, the fragment XXH3 kernel):
// the descriptors a kernel keeps move to the batch's first lanes, in lane
// order (the others after them), by one ds_permute per field; each kept
// descriptor's lane in the batch as loaded rides in the top 6 bits of off_hi,
// so only offsets below 2^58 may be kept (any larger one lies outside every
// buffer).  EXTRA / MOD: the fields the kernel reads besides offset and size.
__device__ __forceinline__ bool below_2p58(const DescBatch& d) { return (d.off_hi >> 26) == 0; }
template <bool EXTRA, bool MOD>
__device__ __forceinline__ void batch_compact(DescBatch& d, uint64_t km, bool keep,
                                              uint32_t lane) {
  const uint64_t below = (1ull << lane) - 1;
  const uint32_t nk = static_cast<uint32_t>(__popcll(km));
  const uint32_t dst = keep ? static_cast<uint32_t>(__popcll(km & below))
                            : nk + static_cast<uint32_t>(__popcll(~km & below));
  const int ad = static_cast<int>(4 * dst);
  auto perm = [&](uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_permute(ad, static_cast<int>(v)));
  };
  d.off_lo = perm(d.off_lo);
  d.off_hi = perm((d.off_hi & 0x03ffffffu) | (lane << 26));
  d.size = perm(d.size);
  if (EXTRA) d.extra = perm(d.extra);
  if (MOD) d.mod = perm(d.mod);
}

// descriptor k (kb <= k < kb + 128) from the current / next batch, uniform
struct Desc {
  uint64_t off;
  uint32_t size, mod, extra;
};
__device__ __forceinline__ Desc batch_desc(uint64_t k, uint64_t kb, const DescBatch& cb,
                                           const DescBatch& nb) {
  const uint32_t kk = static_cast<uint32_t>(k - kb);
  const uint32_t sl = kk & 63u;
  const bool in_n = kk >= 64;
  Desc d;
  const uint64_t off_c = readlane64(cb.off_lo, cb.off_hi, sl);
  const uint64_t off_n = readlane64(nb.off_lo, nb.off_hi, sl);
  d.off = in_n ? off_n : off_c;
  const uint32_t size_c = readlane32(cb.size, sl), size_n = readlane32(nb.size, sl);
  d.size = in_n ? size_n : size_c;
  const uint32_t mod_c = readlane32(cb.mod, sl), mod_n = readlane32(nb.mod, sl);
  d.mod = in_n ? mod_n : mod_c;
  const uint32_t ex_c = readlane32(cb.extra, sl), ex_n = readlane32(nb.extra, sl);
  d.extra = in_n ? ex_n : ex_c;
  return d;
}

// bytes a block of this mode must have inside the buffer (reader / builder)
template <int MODE>
__device__ __forceinline__ bool desc_in_range(const BlockArgs& a, const Desc& d) {
  uint64_t need = d.size;
  if (MODE == kModeVerify || MODE == kModeTrailer) need += 5;
  if (MODE == kModeCompute && !a.last_bytes) need += 1;
  return d.off <= a.base_len && need <= a.base_len - d.off;
}

}  // namespace forst
