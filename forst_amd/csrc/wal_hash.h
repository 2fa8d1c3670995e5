// forst_amd/csrc/wal_hash.h -- XXH3_64bits of WAL logical records
// (log::Reader::ReadRecord's record checksum, db/log_reader.cc:95-165), shared
// by forst_wal_record_xxh3_batch (wal.hip) and forst_wal_recover_batch
// (wal_recover.hip).
//
// A logical record is a run of physical records (fragments).  Records laid
// out the way log::Writer::AddRecord writes them (db/log_writer.cc:65-160:
// every fragment but the last fills its log block, the next one starts right
// after the next block's header) are hashed IN PLACE by xxh3_frag_kernel
// (xxh3.hip), which reads across the header holes; only the rest -- records
// of <= 240 bytes that span a block boundary, records whose last fragment is
// under 64 bytes (the last stripe would straddle), fragment runs a writer
// never produces -- are gathered into scratch (one workgroup per record) and
// hashed there, as one compact batch.  The accessor F describes a
// pipeline's fragments:
//   F::begin(j), F::end(j)   fragment range of logical record j
//   F::header(q)             log offset of fragment q's header
//   F::hs(q), F::len(q)      its header size (7 / 11) and payload length, from
//                            the pipeline's own per-fragment arrays (no
//                            further reads of the header bytes)
//   F::use(q)                false: fragment q is not part of the record (the
//                            record is then gathered without it)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "engine.h"
#include "scan_common.h"

namespace forst {
namespace {

constexpr uint32_t kWhBlock = 32768;  // db/log_format.h:45
constexpr uint32_t kWhLanes = 256;

// per logical record: in-place descriptor (p0, len, info = hs | j_last << 8)
// for the frag kernel, or glen = len when it must be gathered (its frag
// descriptor then has length 0)
// Packed form (n < 2^24 records, a log under 2^40 bytes): glen[j] = bytes |
// 1 << 40 for a gathered record, so ONE exclusive scan gives both its scratch
// offset (low 40 bits) and its list position (the high bits) -- one scan and
// the flag pass fewer than two scans.
constexpr uint32_t kWhPackShift = 40;
constexpr uint64_t kWhPackMask = (uint64_t(1) << kWhPackShift) - 1;
__device__ __forceinline__ uint64_t wh_goff(const uint64_t* go, uint64_t j, bool packed) {
  return packed ? go[j] & kWhPackMask : go[j];
}

template <class F>
__global__ void __launch_bounds__(kWhLanes) wh_prep_kernel(const uint8_t* log, uint64_t log_len,
                                                           F f, uint64_t n,
                                                           uint64_t* p0, uint32_t* len,
                                                           uint32_t* info, uint64_t* glen,
                                                           bool packed) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kWhLanes + threadIdx.x;
  if (j >= n) return;
  const uint64_t b = f.begin(j), e = f.end(j);
  uint64_t total = 0;
  bool regular = true;
  uint64_t start = 0;   // payload offset of the first non-empty fragment
  uint32_t hs0 = 0, nz = 0, last_len = 0;
  uint64_t prev_end = 0;
  for (uint64_t q = b; q < e; ++q) {
    if (!f.use(q)) {
      regular = false;
      continue;
    }
    const uint64_t h = f.header(q);
    const uint32_t hs = f.hs(q), l = f.len(q);
    if (q > b && (h != prev_end || (h & (kWhBlock - 1)) != 0)) regular = false;
    if (q + 1 < e && ((h + hs + l) & (kWhBlock - 1)) != 0) regular = false;  // fills its block
    if (q == b) hs0 = hs;
    if (hs != hs0) regular = false;
    if (l && !nz++) start = h + hs;
    total += l;
    last_len = l;
    prev_end = h + hs + l;
  }
  const bool multi = nz > 1;
  if (multi && (total <= 240 || last_len < 64)) regular = false;
  if (total > 0xffffffffull) regular = false;
  // the frag kernel loads whole 1 KiB windows, and 32 bytes from a short
  // record's chunk (engine.h kFragTail)
  if (prev_end + kFragTail > log_len) regular = false;
  if (nz == 0) start = e > b && f.use(b) ? f.header(b) + f.hs(b) : 0;
  p0[j] = start;
  len[j] = regular ? static_cast<uint32_t>(total) : 0u;
  info[j] = multi ? (hs0 | ((nz - 1) << 8)) : 0u;
  glen[j] = regular ? 0 : packed ? total | (uint64_t(1) << kWhPackShift) : total;
}

__global__ void __launch_bounds__(kWhLanes) wh_flag_kernel(const uint64_t* glen, uint64_t n,
                                                           uint64_t* flag) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kWhLanes + threadIdx.x;
  if (j < n) flag[j] = glen[j] ? 1u : 0u;
}

// the gathered records' compact list: list[gpos[j]] = j, with their scratch
// offsets and lengths as descriptors of one XXH3 batch
__global__ void __launch_bounds__(kWhLanes) wh_list_kernel(const uint64_t* glen,
                                                           const uint64_t* goff,
                                                           const uint64_t* gpos, uint64_t n,
                                                           uint64_t* list, uint64_t* boff,
                                                           uint32_t* blen, bool packed) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kWhLanes + threadIdx.x;
  if (j >= n || glen[j] == 0) return;
  const uint64_t i = packed ? goff[j] >> kWhPackShift : gpos[j];
  list[i] = j;
  boff[i] = wh_goff(goff, j, packed);
  blen[i] = static_cast<uint32_t>(packed ? glen[j] & kWhPackMask : glen[j]);
}

// one workgroup per gathered record: its fragments back to back at dst + boff[i]
template <class F>
__global__ void __launch_bounds__(kWhLanes) wh_gather_kernel(const uint8_t* log, F f,
                                                             const uint64_t* list,
                                                             const uint64_t* boff, uint64_t ng,
                                                             uint8_t* dst) {
  for (uint64_t i = blockIdx.x; i < ng; i += gridDim.x) {
    const uint64_t j = list[i];
    uint8_t* d = dst + boff[i];
    for (uint64_t q = f.begin(j); q < f.end(j); ++q) {
      if (!f.use(q)) continue;
      const uint64_t h = f.header(q);
      const uint8_t* src = log + h + f.hs(q);
      const uint32_t l = f.len(q);
      // whole destination dwords from (unaligned) 4-byte source reads; the
      // <= 3 bytes at either end (shared with the neighbouring fragments'
      // dwords) byte by byte
      const uint32_t head = static_cast<uint32_t>((4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
      const uint32_t hb = head < l ? head : l;
      const uint32_t nw = (l - hb) >> 2;
      const uint32_t tb = hb + 4 * nw;
      if (threadIdx.x < hb) d[threadIdx.x] = src[threadIdx.x];
      if (threadIdx.x < l - tb) d[tb + threadIdx.x] = src[tb + threadIdx.x];
      uint32_t* dw = reinterpret_cast<uint32_t*>(d + hb);
      // 16 destination bytes per thread from a dword-aligned 16-byte load and
      // the dword after it (realigned), four groups per thread in flight; a
      // group's fifth source dword stays inside the fragment (n16), the
      // dwords after the last group one by one
      const uint8_t* s0 = src + hb;
      const uint32_t m = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(s0) & 3);
      const uint8_t* sa = s0 - m;
      const uint32_t n16 = nw >= 5 ? (nw - 1) >> 2 : 0u;
      for (uint32_t g0 = threadIdx.x; g0 < n16; g0 += 4 * kWhLanes) {
        u32x4a4 v[4];
        uint32_t nx[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {  // (unconditional loads: a group past n16 reads g0's)
          const uint32_t g = g0 + k * kWhLanes < n16 ? g0 + k * kWhLanes : g0;
          v[k] = ld16_a4(sa + 16 * g);
          nx[k] = ld4_a4(sa + 16 * g + 16);
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t g = g0 + k * kWhLanes;
          if (g < n16) {
            const u32x4a4 o{__builtin_amdgcn_alignbyte(v[k].y, v[k].x, m),
                            __builtin_amdgcn_alignbyte(v[k].z, v[k].y, m),
                            __builtin_amdgcn_alignbyte(v[k].w, v[k].z, m),
                            __builtin_amdgcn_alignbyte(nx[k], v[k].w, m)};
            *reinterpret_cast<u32x4a4*>(dw + 4 * g) = o;
          }
        }
      }
      for (uint32_t x = 4 * n16 + threadIdx.x; x < nw; x += kWhLanes) dw[x] = ldu32(src + hb + 4 * x);
      d += l;
    }
  }
}

// the frag kernel wrote every record's slot of out (a gathered record's
// descriptor has length 0): the gathered records' hashes over theirs
__global__ void __launch_bounds__(kWhLanes) wh_patch_kernel(const uint64_t* list,
                                                            const uint64_t* hb, uint64_t ng,
                                                            uint64_t* out) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kWhLanes + threadIdx.x;
  if (i < ng) out[list[i]] = hb[i];
}

// The gathered records' branch (list, gather, their XXH3) does not depend on
// the in-place frag kernel, so it runs on a second stream beside it and fills
// the frag kernel's launch tail (a14 9.66 -> 9.52 ms, A/B in
// profiles/ab_r04/a14_gather_overlap.log).  The recovery's remainder batch
// keeps one stream: there the fork and join cost more than the overlap gains
// (C5 recovery +0.06..0.1 ms in the same A/B).
// The second stream and its fork / join events come from the per-device pool
// of engine.h (aux_acquire: the device of the caller's stream), held for the
// call only; any failure there falls back to the caller's stream alone.
#ifndef FORST_WH_OVERLAP
#define FORST_WH_OVERLAP 1
#endif
// holds a pool entry for one call (given back on every exit)
struct AuxHold {
  AuxStream* a = nullptr;
  AuxHold() = default;
  AuxHold(const AuxHold&) = delete;
  AuxHold& operator=(const AuxHold&) = delete;
  ~AuxHold() { aux_release(a); }
};

inline size_t wh_up256(size_t b) { return (b + 255) & ~size_t(255); }
inline dim3 wh_grid(uint64_t n) {
  const uint64_t g = (n + kWhLanes - 1) / kWhLanes;
  return dim3(static_cast<uint32_t>(g ? g : 1));
}

// out[j] = XXH3_64bits of logical record j (device array).  Waits once on the
// host for the gathered byte total (it sizes the scratch): behind the queued
// frag kernel when the second stream is used, else a stream synchronisation.
template <class F>
hipError_t hash_logical_records(const uint8_t* log, uint64_t log_len, const F& f, uint64_t n,
                                uint64_t* out, hipStream_t st, const char** name,
                                bool overlap = true) {
  if (n == 0) return hipSuccess;
  // (FORST_WH_UNPACKED: the emulator test build forces the unpacked form, so
  // the branch beyond 2^24 records / 2^40 bytes runs under test too)
#ifdef FORST_WH_UNPACKED
  const bool packed = false;
#else
  const bool packed = n < (uint64_t(1) << 24) && log_len < (uint64_t(1) << kWhPackShift);
#endif
  const uint64_t nt = n / kScanTile + 2;
  const size_t s8 = wh_up256(8 * n), s4 = wh_up256(4 * n), st8 = wh_up256(8 * nt);
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, 7 * s8 + 3 * s4 + 2 * st8, st);
  if (e != hipSuccess) return e;
  uint8_t* p = static_cast<uint8_t*>(scratch);
  uint64_t* p0 = reinterpret_cast<uint64_t*>(p);
  uint64_t* glen = reinterpret_cast<uint64_t*>(p + s8);
  uint64_t* goff = reinterpret_cast<uint64_t*>(p + 2 * s8);
  uint64_t* gpos = reinterpret_cast<uint64_t*>(p + 3 * s8);  // (unpacked form only)
  uint64_t* hb = reinterpret_cast<uint64_t*>(p + 4 * s8);
  uint64_t* list = reinterpret_cast<uint64_t*>(p + 5 * s8);
  uint64_t* boff = reinterpret_cast<uint64_t*>(p + 6 * s8);  // (reused as the flags)
  uint32_t* len = reinterpret_cast<uint32_t*>(p + 7 * s8);
  uint32_t* info = reinterpret_cast<uint32_t*>(p + 7 * s8 + s4);
  uint32_t* blen = reinterpret_cast<uint32_t*>(p + 7 * s8 + 2 * s4);
  uint64_t* tiles = reinterpret_cast<uint64_t*>(p + 7 * s8 + 3 * s4);
  uint64_t* tiles2 = reinterpret_cast<uint64_t*>(p + 7 * s8 + 3 * s4 + st8);
  hipLaunchKernelGGL(wh_prep_kernel<F>, wh_grid(n), dim3(kWhLanes), 0, st, log, log_len, f, n,
                     p0, len, info, glen, packed);
  scan_u64(glen, n, tiles, goff, st);
  if (!packed) {
    hipLaunchKernelGGL(wh_flag_kernel, wh_grid(n), dim3(kWhLanes), 0, st, glen, n, boff);
    scan_u64(boff, n, tiles2, gpos, st);
  }
  uint64_t tot[2] = {0, 0};  // gathered bytes, gathered records (packed: both in tot[0])
  const uint64_t ntl = (n + kScanTile - 1) / kScanTile;
  // in place across the fragments, straight into out (every record; the
  // gathered ones have length 0 and are patched below)
  BlockArgs fa{};
  fa.base = log;
  fa.base_len = log_len;
  fa.offsets = p0;
  fa.sizes = len;
  fa.init_crcs = info;
  fa.out64 = out;
  fa.n = n;
  auto frag = [&]() {
    return log_len >= 4096 ? launch_xxh3_frag(fa, st, name)
                           : launch_xxh3_blocks(kModeRaw, fa, st, name);
  };
  if ((e = hipMemcpyAsync(&tot[0], tiles + ntl, 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (!packed &&
       (e = hipMemcpyAsync(&tot[1], tiles2 + ntl, 8, hipMemcpyDeviceToHost, st)) != hipSuccess)) {
    (void)scratch_free(scratch, st);
    return e;
  }
  // With the second stream the frag kernel is queued before the host waits
  // for the totals (on an event behind their copies), so the GPU does not
  // idle through the host's turnaround, and the gathered branch starts on the
  // second stream while the frag kernel runs.
  AuxHold hold;
  if (FORST_WH_OVERLAP && overlap) hold.a = aux_acquire(st);
  AuxStream* aux = hold.a;
  if (aux && hipEventRecord(aux->fork, st) != hipSuccess) {
    (void)hipGetLastError();
    aux = nullptr;
  }
  if (aux) {
    e = frag();
    const hipError_t w = hipEventSynchronize(aux->fork);
    if (e == hipSuccess) e = w;
  } else {
    e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = frag();
  }
  if (e != hipSuccess) {
    (void)scratch_free(scratch, st);
    return e;
  }
  const uint64_t gtotal = packed ? tot[0] & kWhPackMask : tot[0];
  const uint64_t ng = packed ? tot[0] >> kWhPackShift : tot[1];
  void* gbuf = nullptr;
  if (ng) {
    hipStream_t gs = st;
    const bool forked = aux && hipStreamWaitEvent(aux->s, aux->fork, 0) == hipSuccess;
    if (forked) gs = aux->s;
    e = scratch_alloc(&gbuf, wh_up256(gtotal + 4096), gs);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(wh_list_kernel, wh_grid(n), dim3(kWhLanes), 0, gs, glen, goff, gpos, n,
                         list, boff, blen, packed);
      const uint32_t gg = static_cast<uint32_t>(ng < 65536 ? ng : 65536);
      hipLaunchKernelGGL(wh_gather_kernel<F>, dim3(gg), dim3(kWhLanes), 0, gs, log, f, list,
                         boff, ng, static_cast<uint8_t*>(gbuf));
      BlockArgs ga{};
      ga.base = static_cast<uint8_t*>(gbuf);
      ga.base_len = wh_up256(gtotal + 4096);
      ga.offsets = boff;
      ga.sizes = blen;
      ga.out64 = hb;
      ga.n = ng;
      ga.kernel_hint = 3;  // few records (C5: 22 K of 10 M), long ones: one per wave
      const char* gname = nullptr;
      e = launch_xxh3_blocks(kModeRaw, ga, gs, &gname);
    }
    // join (also on failure: st must not run ahead of work queued on gs,
    // which reads the scratch freed on st below)
    if (forked && (hipEventRecord(aux->join, gs) != hipSuccess ||
                   hipStreamWaitEvent(st, aux->join, 0) != hipSuccess)) {
      if (e == hipSuccess) e = hipErrorUnknown;
      (void)hipStreamSynchronize(gs);
    }
    if (e == hipSuccess) {  // behind the frag kernel (st) and the join
      hipLaunchKernelGGL(wh_patch_kernel, wh_grid(ng), dim3(kWhLanes), 0, st, list, hb, ng, out);
      e = hipGetLastError();
    }
  }
  const hipError_t f1 = scratch_free(gbuf, st), f2 = scratch_free(scratch, st);
  return e != hipSuccess ? e : f1 != hipSuccess ? f1 : f2;
}

}  // namespace
}  // namespace forst
