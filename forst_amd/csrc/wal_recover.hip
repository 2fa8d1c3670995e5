// forst_amd/csrc/wal_recover.hip -- the fused WAL recovery pass (SURVEY.md
// §8f-2): log::Reader::ReadRecord (db/log_reader.cc:69-320) over a whole log
// image as called by DBImpl::RecoverLogFiles (db/db_impl/db_impl_open.cc:1210),
// with record boundaries discovered on the device.
//
// The serial reader interleaves three things: the header chain inside each
// 32 KiB log block (ReadPhysicalRecord :450-531, ReadMore :404-448), the CRC
// of every physical record, and a small state machine that assembles
// fragments into logical records, reports corruption and hashes each logical
// record with XXH3 (:95-165).  Records never straddle a log block
// (log_writer.cc:86-102), so the first two are per-block; the state machine is
// a left-to-right scan whose state only resets at "head" tokens, which makes
// it a segmented scan:
//
//   walk     lane per log block: the header chain with the reader's checks in
//            its order (truncated header, bad length, old record -- skipped in
//            kSkipAnyCorruptedRecords --, zero type) -> item count + the
//            block's terminal event                       (one sync: item total)
//   fill     re-walk: header offset + kind of every item, CRC descriptors
//   crc      crc32c rows kernel over every record (raw mode)
//   block    lane per block: first CRC mismatch truncates the block
//            (kBadRecordChecksum, rest of block dropped); reader position at
//            block exit; the first block whose event ends reading
//   tokens   per block: one token per consumed physical record (Full / First /
//            Middle / Last / unknown type / skipped old record) and one for
//            the block's event; a final EOF token
//   fsm      heads = tokens that reset the reader's fragment state (Full,
//            First, unknown type, bad record, checksum / length errors,
//            stops); segment = scan of head flags; the first Last of a
//            segment headed by First completes a logical record; every other
//            Middle / Last is reported as missing its start; a head after an
//            unfinished First segment reports what the reader reports there
//   emit     logical records (first fragment = segment head) and reports in
//            reader order                               (one sync: counts)
//   hash     XXH3_64bits of every logical record (wal_hash.h): in place
//            across the fragment headers when laid out as a writer lays them
//            out, else from a gathered copy             (one sync: gathered bytes)
//
// The reader's behaviour is reproduced to the letter, as its compiled code
// shows it (tests/golden/gen_wal_golden.py pins this file to the reference's
// own log::Reader): a type byte is read through `const char*` into an
// unsigned int (log_reader.cc:469), so 0x80..0xFF sign-extend; types 12..17
// with a valid CRC are the reader's own results kEof .. kBadRecordChecksum
// (log_reader.h:173-186), consumed without clearing the buffer; the XXH3
// state is reset only when ReadRecord starts and at "partial record without
// end(2)" (:73-79, :119-124), so a fragmented record's checksum covers the
// fragments of records aborted since (use() of the fragment accessor); and
// kSetCompressionType / timestamp-size records (types 9-11, :167-213) clear
// scratch but keep in_fragmented_record, so a segment they head inherits
// the previous segment's state (rw_live).  Their decode / duplicate checks
// depend on state kept across the whole log (compression record seen,
// recorded column families): the few such records are read back and
// decided on the host, in reader order (ctl_* below).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../../include/forst_checksum.h"
#include "crc32c_tables.h"
#include "device_common.h"
#include "engine.h"
#include "scan_common.h"
#include "wal_hash.h"

#ifndef FORST_REC_OVERLAP
#define FORST_REC_OVERLAP 1
#endif

namespace forst {
namespace {

constexpr uint32_t kLogBlock = 32768;  // db/log_format.h:45
constexpr uint32_t kLogHdr = 7;        // :48
constexpr uint32_t kLogRHdr = 11;      // :52
constexpr uint32_t kLanes = 256;
constexpr uint32_t kCtlRep = 3;        // host-decided reports per control record (at most)

// block terminal events (the reader's result when it leaves the block)
enum : uint32_t {
  kEvNone = 0,     // block consumed (trailer < header size skipped)
  kEvChecksum,     // kBadRecordChecksum: rest of block dropped
  kEvBadLen,       // kBadRecordLen, not at EOF: as a checksum error
  kEvZero,         // kZeroType, length 0 -> kBadRecord
  kEvOldStop,      // kOldRecord (not skip mode): reading ends
  kEvBadHeader,    // truncated header at EOF (kBadHeader): reading ends
  kEvBadLenEof,    // kBadRecordLen at EOF: reading ends
  kEvPseudo,       // a record of type 12..17 that ends reading (its own token)
};

// token kinds
enum : uint8_t {
  kTkFull = 1, kTkFirst, kTkMiddle, kTkLast, kTkUnknown, kTkOldSkip, kTkZero, kTkChecksum,
  kTkBadLen, kTkStopHeader, kTkStopBadLenEof, kTkStopOld, kTkStopRecycled, kTkStopEof,
  kTkCtlComp,  // kSetCompressionType (9)
  kTkCtlTs,    // kUserDefinedTimestampSizeType (10) / its recyclable form (11)
  // records whose type is one of the reader's own results (log_reader.h:173-186)
  kTkPEof,     // 12 kEof
  kTkPOld,     // 15 kOldRecord, not kSkipAnyCorruptedRecords: as kEof
  kTkPBad,     // 13 kBadRecord (and 15 in kSkipAnyCorruptedRecords)
  kTkPHeader,  // 14 kBadHeader, drop 0
  kTkPLenEof,  // 16 kBadRecordLen while eof_, drop 0
  kTkPLen,     // 16 kBadRecordLen, drop 0, buffer kept
  kTkPCrc,     // 17 kBadRecordChecksum, drop 0, buffer kept
};

struct RecoverArgs {
  const uint8_t* log;
  uint64_t log_len;
  uint64_t n_blocks;
  uint32_t log_number;
  int mode;  // WALRecoveryMode
  int fuse;  // candidates through the fused CRC + XXH3 kernel
};

__device__ __forceinline__ bool recyclable_type(uint32_t t) {  // log_format.h:20-41
  return (t >= 5 && t <= 8) || t == 11;
}
__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
         (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}
__device__ __forceinline__ uint32_t unmask(uint32_t m) {  // util/crc32c.h:39
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}
__device__ __forceinline__ bool eof_block(const RecoverArgs& a, uint64_t b) {
  return a.log_len - b * kLogBlock < kLogBlock;  // ReadMore read short: eof_
}
// a record of type 12..17 with a valid CRC that ends reading (ReadRecord
// :236-305 reached through the aliased result)
__device__ __forceinline__ bool pseudo_stops(uint32_t ty, bool eofb, uint32_t recycled, int mode) {
  return ty == 12 || ty == 14 || (ty == 15 && mode != 3) ||
         (ty == 16 && (eofb || (recycled && mode == 0))) || (ty == 17 && recycled && mode == 0);
}

// ---- walk -------------------------------------------------------------------
// items: header offsets of the physical records the reader parses in block b
// (REC: CRC to check; OLD: skipped old record, kSkipAnyCorruptedRecords);
// emit(n, header offset, old, unmasked stored CRC, packed length | type << 16
// | recyclable << 24) for each
template <class Emit>
__device__ uint32_t rw_walk_block(const RecoverArgs& a, uint64_t b, uint32_t* ev, uint32_t* ev_pos,
                                  Emit emit) {
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  const bool eofb = end - start < kLogBlock;
  uint64_t pos = start;
  uint32_t n = 0, e = kEvNone;
  while (true) {
    const uint64_t rem = end - pos;
    if (rem < kLogHdr) {  // trailer skipped, or a truncated header at EOF
      if (rem > 0 && eofb) e = kEvBadHeader;
      break;
    }
    const WalHdr h = load_wal_header(a.log, a.log_len, pos);
    const uint32_t length = h.length;
    const uint32_t type = h.type;  // the byte; sign extension matters only in reports
    const bool recyc = recyclable_type(type);
    const uint32_t hs = recyc ? kLogRHdr : kLogHdr;
    if (rem < hs) {
      if (eofb) e = kEvBadHeader;
      break;
    }
    if (hs + length > rem) {
      e = eofb ? kEvBadLenEof : kEvBadLen;
      break;
    }
    const uint32_t pk = length | (type << 16) | (recyc ? 1u << 24 : 0u);
    if (recyc && h.lognum != a.log_number) {
      if (a.mode != 3) {  // not kSkipAnyCorruptedRecords: reading ends here
        e = kEvOldStop;
        break;
      }
      emit(n, pos, true, 0u, pk);
      ++n;
      pos += hs + length;
      continue;
    }
    if (type == 0 && length == 0) {
      e = kEvZero;
      break;
    }
    emit(n, pos, false, unmask(h.crc), pk);  // log_reader.cc:522-523
    ++n;
    pos += hs + length;
  }
  *ev = e;
  *ev_pos = static_cast<uint32_t>(pos - start);
  return n;
}

__global__ void __launch_bounds__(kLanes) rw_count_kernel(RecoverArgs a, uint64_t* cnt) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (b >= a.n_blocks) return;
  uint32_t ev, ep;
  cnt[b] = rw_walk_block(a, b, &ev, &ep, [](uint32_t, uint64_t, bool, uint32_t, uint32_t) {});
}

// The items of a workgroup's 256 log blocks are one contiguous run of the
// per-item arrays: staged in LDS by the lane-per-block walks and stored
// coalesced (the walks' own stores are one partial line per item and array:
// 4.5 GB of traffic for C5's 11.4 M items); a run over the cap is stored
// directly.  crc_off / crc_len follow from the offset and the packed word.
constexpr uint32_t kRwFillCap = 2560;  // 17 B per item: 42.5 KiB of LDS
__global__ void __launch_bounds__(kLanes) rw_fill_kernel(RecoverArgs a, const uint64_t* base,
                                                         const uint64_t* cnt,
                                                         uint64_t* it_off, uint8_t* it_old,
                                                         uint64_t* crc_off, uint32_t* crc_len,
                                                         uint32_t* crc_stored, uint32_t* ipack,
                                                         uint32_t* ev, uint32_t* ev_pos) {
  __shared__ uint64_t l_off[kRwFillCap];
  __shared__ uint32_t l_st[kRwFillCap], l_pk[kRwFillCap];
  __shared__ uint8_t l_old[kRwFillCap];
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * kLanes;
  const uint64_t b = b0 + threadIdx.x;
  const uint64_t bl = (b0 + kLanes < a.n_blocks ? b0 + kLanes : a.n_blocks) - 1;  // last block
  const uint64_t wg_base = base[b0];
  const uint64_t tot = base[bl] + cnt[bl] - wg_base;
  const bool staged = tot <= kRwFillCap;  // workgroup-uniform
  if (b < a.n_blocks) {
    const uint64_t mine = base[b];
    auto direct = [&](uint32_t n, uint64_t pos, bool old, uint32_t st, uint32_t pk) {
      const uint64_t i = mine + n;
      it_off[i] = pos;
      it_old[i] = old ? 1 : 0;
      crc_off[i] = old ? 0 : pos + 6;
      crc_len[i] = old ? 0 : ((pk >> 24) ? kLogRHdr : kLogHdr) + (pk & 0xffffu) - 6;
      if (!old) crc_stored[i] = st;
      ipack[i] = pk;
    };
    auto stage = [&](uint32_t n, uint64_t pos, bool old, uint32_t st, uint32_t pk) {
      const uint64_t i = mine - wg_base + n;
      l_off[i] = pos;
      l_old[i] = old ? 1 : 0;
      l_st[i] = st;
      l_pk[i] = pk;
    };
    if (staged)
      rw_walk_block(a, b, &ev[b], &ev_pos[b], stage);
    else
      rw_walk_block(a, b, &ev[b], &ev_pos[b], direct);
  }
  if (staged) {
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < tot; k += kLanes) {
      const uint64_t i = wg_base + k;
      const uint64_t pos = l_off[k];
      const bool old = l_old[k] != 0;
      const uint32_t pk = l_pk[k];
      it_off[i] = pos;
      it_old[i] = old ? 1 : 0;
      crc_off[i] = old ? 0 : pos + 6;
      crc_len[i] = old ? 0 : ((pk >> 24) ? kLogRHdr : kLogHdr) + (pk & 0xffffu) - 6;
      if (!old) crc_stored[i] = l_st[k];
      ipack[i] = pk;
    }
  }
}

// ---- candidates: records laid out as log::Writer lays them out ---------------
// The reader's records are only known after the CRCs (the state machine
// below), but a log written by log::Writer::AddRecord (log_writer.cc:65-160)
// is a run of such records: a Full, or a First whose fragments fill their
// blocks, the next one right after the next block's header, up to a Last.
// Every such run is a CANDIDATE: one pass of the fragment kernel with the
// fused CRC (xxh3.hip xxh3_frag_kernel<3, true>) reads its bytes ONCE for both
// the XXH3 record checksum and the CRC32C of each physical record.  Records
// the state machine emits that are exactly a candidate (same first and last
// physical record, XXH3 state reset at its head) take the candidate's hash;
// everything else -- corrupted, re-typed, recycled or zero-filled logs -- is
// CRC'd by the rows kernel (raw) and hashed by hash_logical_records.
__device__ __forceinline__ uint32_t ct_shift(const uint32_t* T, uint32_t v) {  // 4 x 256 table
  return T[v & 0xffu] ^ T[256 + ((v >> 8) & 0xffu)] ^ T[512 + ((v >> 16) & 0xffu)] ^
         T[768 + (v >> 24)];
}
// v * x^(8n) mod P (raw CRC32C state moved over n zero bytes), n <= 1024
__device__ __forceinline__ uint32_t crc_shift_bytes(uint32_t v, uint32_t n) {
  const uint32_t a6 = n >> 6, b4 = (n >> 2) & 15u, r = n & 3u;
  if (a6) v = ct_shift(kCrcS64 + 1024 * (a6 - 1), v);
  if (b4) v = ct_shift(kCrcS4 + 1024 * (b4 - 1), v);
  for (uint32_t i = 0; i < r; ++i) v = (v >> 8) ^ kCrcG[3 * 256 + (v & 0xffu)];  // Sarwate
  return v;
}
// the CRC32C state after header bytes [6, hs) from ~0 (log_writer.cc:240-258)
__device__ __forceinline__ uint32_t crc_header_state(const uint8_t* h, uint32_t hs) {
  uint32_t v = 0xffffffffu;
  for (uint32_t i = 6; i < hs; ++i) v = (v >> 8) ^ kCrcG[3 * 256 + ((v ^ h[i]) & 0xffu)];
  return v;
}
// the same two with the tables in LDS (rw_cand_kernel): S64 / S4 / byte table
struct ShiftLds {
  const uint32_t* s64;
  const uint32_t* s4;
  const uint32_t* g3;
  __device__ __forceinline__ uint32_t shift(uint32_t v, uint32_t n) const {  // n <= 1024
    const uint32_t a6 = n >> 6, b4 = (n >> 2) & 15u, r = n & 3u;
    if (a6) v = ct_shift(s64 + 1024 * (a6 - 1), v);
    if (b4) v = ct_shift(s4 + 1024 * (b4 - 1), v);
    for (uint32_t i = 0; i < r; ++i) v = (v >> 8) ^ g3[v & 0xffu];
    return v;
  }
  // n <= 2048 (a window of the fragment kernel)
  __device__ __forceinline__ uint32_t shift_w(uint32_t v, uint32_t n) const {
    if (n > 1024) {
      v = shift(v, 1024);
      n -= 1024;
    }
    return shift(v, n);
  }
  // the CRC state after header[6..hs): the type byte, then (recyclable) the
  // log number -- both known from the walk (the packed word; a non-old
  // recyclable record carries the reader's log number), so no header read
  __device__ __forceinline__ uint32_t header_state(uint32_t type, uint32_t lognum,
                                                   uint32_t hs) const {
    uint32_t v = 0xffffffffu;
    v = (v >> 8) ^ g3[(v ^ type) & 0xffu];
    if (hs == kLogRHdr)
      for (uint32_t k = 0; k < 4; ++k) v = (v >> 8) ^ g3[(v ^ (lognum >> (8 * k))) & 0xffu];
    return v;
  }
};

struct Cand {
  uint8_t* head;       // per item: 1 = a candidate starts here
  uint8_t* fused;      // per item: its CRC comes from the fused kernel
  uint64_t* ez;        // per item: E | Z << 32
  uint64_t* p0;        // per item (heads): payload start of the first non-empty fragment
  uint32_t* len;       //   logical length
  uint32_t* info;      //   hs | j_last << 8 (0: one fragment)
  uint32_t* first;     //   item of the first non-empty fragment
  uint32_t* last;      //   last item
};

// one candidate head per item; a persistent grid with the shift tables in
// LDS (E / Z are chains of table reads: from global memory they made this
// pass 0.6-0.7 ms on C5).  head[] and fused[] are zeroed before the launch
// (a head marks the fragments of its run: no other thread writes them).
constexpr uint32_t kCandThreads = 1024;
__device__ __forceinline__ void cand_one(const RecoverArgs& a, uint64_t ni, uint64_t i,
                                         const uint64_t* it_off, const uint8_t* it_old,
                                         const uint32_t* ipack, const uint32_t* crc_stored,
                                         const Cand& c, const ShiftLds& T) {
  auto ltype = [&](uint64_t q) {  // legacy type of item q (0: none of Full..Last)
    const uint32_t ty = (ipack[q] >> 16) & 0xffu;
    const uint32_t nt = (ty >= 5 && ty <= 8) ? ty - 4 : ty;
    return it_old[q] || nt < 1 || nt > 4 ? 0u : nt;
  };
  const uint32_t t0 = ltype(i);
  if (t0 != 1 && t0 != 2) return;
  const uint32_t pk0 = ipack[i];
  const uint32_t rec0 = (pk0 >> 24) & 1u;
  const uint32_t hs = rec0 ? kLogRHdr : kLogHdr;
  uint64_t q = i, prev_end = 0, total = 0, start = 0, first = i;
  uint32_t nz = 0, last_len = 0;
  bool ok = true;
  for (;; ++q) {  // the run i .. q (wh_prep_kernel's regularity, wal_hash.h)
    if (q >= ni) {
      ok = false;
      break;
    }
    const uint32_t tq = ltype(q);
    const uint32_t pk = ipack[q];
    const uint64_t h = it_off[q];
    const uint32_t l = pk & 0xffffu;
    if (q > i && (tq != 3 && tq != 4)) {
      ok = false;
      break;
    }
    if (((pk >> 24) & 1u) != rec0) ok = false;
    if (q > i && (h != prev_end || (h & (kLogBlock - 1)) != 0)) ok = false;
    if (l && nz && last_len == 0) ok = false;  // (an empty fragment only first)
    if (l) {
      if (!nz) {
        start = h + hs;
        first = q;
      }
      ++nz;
    }
    total += l;
    last_len = l;
    prev_end = h + hs + l;
    if (t0 == 1 || tq == 4) break;
    if ((prev_end & (kLogBlock - 1)) != 0) ok = false;  // a First / Middle fills its block
    if (!ok) break;
  }
  const bool multi = nz > 1;
  if (multi && (total <= 240 || last_len < 64)) ok = false;
  if (total > 0xffffffffull) ok = false;
  // (the fused kernel loads whole 1 KiB windows, and 32 bytes from a short
  // record's chunk: engine.h kFragTail)
  if (prev_end + kFragTail > a.log_len) ok = false;
  // with the short path the fused kernel takes records over 240 B only: a
  // shorter run of several items (an empty First, then one fragment) is left
  // to the raw path and hash_logical_records
  if (FORST_REC_SHORT && total <= 240 && t0 != 1) ok = false;
  if (!ok) return;
  if (nz == 0) start = it_off[i] + hs;
  // a short candidate (head 2, a Full record): its CRC by the lane kernel,
  // its hash by xxh3_short_rows_kernel into ez[i] (no E / Z: the fused kernel
  // never sees it), both from the short list (rw_cand_flags_kernel)
  const bool shrt = FORST_REC_SHORT && total <= 240;
  const bool one = FORST_REC_MED && t0 == 1 && total <= kFragWinFused;  // one window
  c.head[i] = shrt ? 2 : one ? 3 : 1;
  c.p0[i] = start;
  c.len[i] = static_cast<uint32_t>(total);
  c.info[i] = multi ? (hs | ((nz - 1) << 8)) : 0u;
  c.first[i] = static_cast<uint32_t>(first);
  c.last[i] = static_cast<uint32_t>(q);
  if (shrt) return;
  // E / Z of every non-empty fragment (xxh3.hip, the fused CRC): E = H moved
  // from the fragment start to the end of its first window, Z = ~stored moved
  // from the fragment end to the end of its last window (windows of kFragWinFused)
  uint32_t b = 0;
  for (uint64_t r = first; r <= q; ++r) {
    const uint32_t l = ipack[r] & 0xffffu;
    if (l == 0) continue;  // (an empty trailing fragment: the rows kernel's CRC)
    const uint32_t H = T.header_state((ipack[r] >> 16) & 0xffu, a.log_number, hs);
    const uint32_t e = b + l;
    const uint32_t ws = b >> kFragWinFusedShift, we = (e - 1) >> kFragWinFusedShift;
    const uint32_t E = T.shift_w(H, kFragWinFused * (ws + 1) - b);
    const uint32_t Z = T.shift_w(~crc_stored[r], kFragWinFused * (we + 1) - e);
    c.ez[r] = static_cast<uint64_t>(E) | (static_cast<uint64_t>(Z) << 32);
    c.fused[r] = 1;
    b = e;
  }
}

__global__ void __launch_bounds__(kCandThreads) rw_cand_kernel(RecoverArgs a, uint64_t ni,
                                                               const uint64_t* it_off,
                                                               const uint8_t* it_old,
                                                               const uint32_t* ipack,
                                                               const uint32_t* crc_stored, Cand c) {
  __shared__ uint32_t s64[16 * 1024], s4[15 * 1024], g3[256];
  if (!a.fuse) return;  // (logs under 4 KiB: the rows kernels' dummy loads need 4 KiB)
  for (uint32_t k = threadIdx.x; k < 16 * 1024; k += kCandThreads) s64[k] = kCrcS64[k];
  for (uint32_t k = threadIdx.x; k < 15 * 1024; k += kCandThreads) s4[k] = kCrcS4[k];
  if (threadIdx.x < 256) g3[threadIdx.x] = kCrcG[3 * 256 + threadIdx.x];
  __syncthreads();
  const ShiftLds T{s64, s4, g3};
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kCandThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kCandThreads + threadIdx.x; i < ni;
       i += stride)
    cand_one(a, ni, i, it_off, it_old, ipack, crc_stored, c, T);
}

// the short candidates' list (item order): the CRC'd bytes (header[6..hs) +
// payload) for the lane CRC kernel, the payload for the one-per-lane XXH3
struct ShortList {
  uint64_t* item;
  uint64_t* off;
  uint32_t* len;
  uint64_t* p0;
  uint32_t* plen;
  uint32_t* computed;
};

// compact lists, item order: the fused kernel's candidates -- long ones
// (head 1) and one-window Full records (head 3, FORST_REC_MED), launched
// apart -- the short candidates (head 2) and the physical records the rows
// kernel CRCs.  Candidates exist only when ni < 2^32 (RecoverArgs::fuse), so
// two packed scans give all four positions: fc = long | one-window << 32,
// fr = short | raw << 32 (else fr = raw alone, 64-bit)
__global__ void __launch_bounds__(kLanes) rw_cand_flags_kernel(const Cand c, uint64_t ni,
                                                               const uint8_t* it_old, int packed,
                                                               uint64_t* fc, uint64_t* fr) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= ni) return;
  const uint8_t hd = c.head[i];
  const uint64_t sh = hd == 2 ? 1u : 0u;
  // (skipped old records need no CRC; short candidates take the lane kernel's)
  const uint64_t r = c.fused[i] || it_old[i] || sh ? 0u : 1u;
  if (packed) {
    fc[i] = (hd == 1 ? 1u : 0u) | (static_cast<uint64_t>(hd == 3 ? 1u : 0u) << 32);
    fr[i] = sh | (r << 32);
  } else {
    fr[i] = r;
  }
}

__global__ void __launch_bounds__(kLanes) rw_cand_list_kernel(const Cand c, uint64_t ni,
                                                              const uint8_t* it_old, int packed,
                                                              uint64_t n_long,
                                                              const uint64_t* cpos,
                                                              const uint64_t* rpos,
                                                              const uint64_t* crc_off,
                                                              const uint32_t* crc_len,
                                                              uint64_t* l_p0, uint32_t* l_len,
                                                              uint32_t* l_info, uint32_t* l_first,
                                                              uint64_t* r_off, uint32_t* r_len,
                                                              uint64_t* r_item, ShortList sl) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= ni) return;
  const uint8_t hd = packed ? c.head[i] : 0;
  if (hd == 1 || hd == 3) {  // the one-window records after the long ones
    const uint64_t k = hd == 1 ? (cpos[i] & 0xffffffffu) : n_long + (cpos[i] >> 32);
    l_p0[k] = c.p0[i];
    l_len[k] = c.len[i];
    l_info[k] = c.info[i];
    l_first[k] = c.first[i];
  } else if (hd == 2) {
    const uint64_t k = rpos[i] & 0xffffffffu;
    sl.item[k] = i;
    sl.off[k] = crc_off[i];
    sl.len[k] = crc_len[i];
    sl.p0[k] = c.p0[i];
    sl.plen[k] = c.len[i];
  }
  if (!c.fused[i] && !it_old[i] && hd != 2) {
    const uint64_t k = packed ? rpos[i] >> 32 : rpos[i];
    r_off[k] = crc_off[i];
    r_len[k] = crc_len[i];
    r_item[k] = i;
  }
}

// the rows kernel's CRCs -> the verdicts of the non-fused records
__global__ void __launch_bounds__(kLanes) rw_raw_ok_kernel(const uint64_t* r_item,
                                                           const uint32_t* computed, uint64_t nr,
                                                           const uint32_t* crc_stored,
                                                           uint8_t* crc_ok) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (k >= nr) return;
  const uint64_t i = r_item[k];
  crc_ok[i] = computed[k] == crc_stored[i] ? 1 : 0;
}

// ---- per block: CRC truncation, reader position, stop -------------------------
// acc[b] = items consumed before the first CRC mismatch (a stopping pseudo
// record included); the event becomes kEvChecksum at a mismatch, kEvPseudo
// at a stopping pseudo record; rp_end[b] = reader position when leaving the
// block (end of the last consumed record, or the block end after a
// buffer-clearing event)
// the first item of each block that stops its block's reading: a CRC
// mismatch, or a record whose valid CRC ends reading (pseudo_stops); item-
// parallel, so the per-block pass below reads O(1) items per block instead of
// walking them (rw_block was a lane-per-block loop: 0.27 ms on C5)
__global__ void __launch_bounds__(kLanes) rw_block_bad_kernel(RecoverArgs a, uint64_t ni,
                                                              const uint64_t* it_off,
                                                              const uint8_t* it_old,
                                                              const uint32_t* ipack,
                                                              const uint8_t* crc_ok,
                                                              const uint64_t* base,
                                                              const uint32_t* recycled_d,
                                                              uint32_t* first_bad) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= ni || it_old[i]) return;
  const uint64_t b = it_off[i] / kLogBlock;
  if (crc_ok[i] && !pseudo_stops((ipack[i] >> 16) & 0xffu, eof_block(a, b), *recycled_d, a.mode))
    return;
  atomicMin(first_bad + b, static_cast<uint32_t>(i - base[b]));
}

// block b's reading (the loop of log_reader.cc:236-305 over the block's
// items): consumed items up to the first stopping one, the block's event and
// where the reader stands after it
__global__ void __launch_bounds__(kLanes) rw_block_kernel(RecoverArgs a, const uint64_t* cnt,
                                                          const uint64_t* base,
                                                          const uint64_t* it_off,
                                                          const uint8_t* it_old,
                                                          const uint64_t* crc_off,
                                                          const uint32_t* crc_len,
                                                          const uint32_t* ipack,
                                                          const uint8_t* crc_ok,
                                                          const uint32_t* first_bad, uint32_t* ev,
                                                          uint32_t* ev_pos, uint64_t* acc,
                                                          uint64_t* rp_end,
                                                          unsigned long long* first_stop,
                                                          const uint32_t* recycled_d) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (b >= a.n_blocks) return;
  const uint32_t recycled = *recycled_d;
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  const uint64_t n = cnt[b], i0 = base[b];
  const uint64_t fb = first_bad[b];
  uint64_t k = fb < n ? fb : n;
  auto item_end = [&](uint64_t j) {
    return it_old[j] ? it_off[j] + ((ipack[j] >> 24) & 1u ? kLogRHdr : kLogHdr) + (ipack[j] & 0xffffu)
                     : crc_off[j] + crc_len[j];
  };
  uint64_t last_end = k ? item_end(i0 + k - 1) : start;
  uint32_t e = ev[b], ep = ev_pos[b];
  if (fb < n) {
    const uint64_t j = i0 + fb;
    if (!crc_ok[j]) {
      e = kEvChecksum;
      ep = static_cast<uint32_t>(crc_off[j] - 6 - start);
    } else {  // a valid record that ends reading: consumed
      k = fb + 1;
      last_end = crc_off[j] + crc_len[j];
      e = kEvPseudo;
      ep = static_cast<uint32_t>(last_end - start);
    }
  }
  acc[b] = k;
  ev[b] = e;
  ev_pos[b] = ep;
  // events that clear the buffer leave the reader at the block end
  const bool clears = e == kEvChecksum || e == kEvBadLen || e == kEvZero || e == kEvBadHeader ||
                      e == kEvBadLenEof;
  rp_end[b] = clears ? end : (e == kEvOldStop ? start + ep : last_end);
  // recycled log + kTolerateCorruptedTailRecords: a checksum / length error
  // ends reading silently (log_reader.cc:288-291)
  const bool stop = e == kEvOldStop || e == kEvBadHeader || e == kEvBadLenEof || e == kEvPseudo ||
                    ((e == kEvChecksum || e == kEvBadLen) && recycled && a.mode == 0);
  if (stop) atomicMin(first_stop, static_cast<unsigned long long>(b));
}

__device__ __forceinline__ bool event_token(uint32_t e) { return e != kEvNone && e != kEvPseudo; }

__global__ void __launch_bounds__(kLanes) rw_ntok_kernel(RecoverArgs a, const uint64_t* acc,
                                                         const uint32_t* ev,
                                                         const unsigned long long* first_stop,
                                                         uint64_t* ntok) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (b > a.n_blocks) return;
  if (b == a.n_blocks) {  // the final EOF token, unless a block stopped reading
    ntok[b] = *first_stop == ~0ull ? 1 : 0;
    return;
  }
  ntok[b] = b > *first_stop ? 0 : acc[b] + (event_token(ev[b]) ? 1 : 0);
}

// tokens: kind, item (physical record index; events: block), payload length
// (events: dropped bytes), reader position (physical_record_offset of the
// reference, end_of_buffer_offset_ - buffer_.size() before the read), type
// byte (sign-extended where reported)
struct Tokens {
  uint8_t* kind;
  uint64_t* item;
  uint32_t* len;
  uint64_t* pos;
  uint8_t* type;
};

__device__ __forceinline__ uint8_t record_kind(uint32_t type, bool eofb, uint32_t recycled, int mode) {
  const uint32_t nt = (type >= 5 && type <= 8) ? type - 4 : type;  // recyclable -> legacy
  switch (nt) {
    case 1: return kTkFull;
    case 2: return kTkFirst;
    case 3: return kTkMiddle;
    case 4: return kTkLast;
    case 9: return kTkCtlComp;
    case 10:
    case 11: return kTkCtlTs;
    case 12: return kTkPEof;
    case 13: return kTkPBad;
    case 14: return kTkPHeader;
    case 15: return mode == 3 ? kTkPBad : kTkPOld;
    case 16: return eofb ? kTkPLenEof : (recycled && mode == 0 ? kTkStopRecycled : kTkPLen);
    case 17: return recycled && mode == 0 ? kTkStopRecycled : kTkPCrc;
    default: return kTkUnknown;
  }
}

// exclusive scan of one value per lane over a kLanes-thread workgroup
__device__ __forceinline__ uint32_t rw_wg_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (uint32_t d = 1; d < kLanes; d <<= 1) {
    const uint32_t add = t >= d ? sh[t - d] : 0u;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const uint32_t incl = sh[t];
  *total = sh[kLanes - 1];
  __syncthreads();
  return incl - v;
}

// One token per consumed physical record and per block event, in reader
// order.  A workgroup's 256 log blocks own contiguous runs of the item and
// token arrays; the record tokens are made item-parallel (each lane finds its
// item's block by a binary search over the workgroup's prefix in LDS, so the
// item reads and token stores are coalesced), the event tokens by the lane of
// their block.  A record token's reader position is the end of the item
// before it in its block (or the position entering the block).
__global__ void __launch_bounds__(kLanes) rw_token_kernel(RecoverArgs a, const uint64_t* base,
                                                          const uint64_t* it_off,
                                                          const uint8_t* it_old,
                                                          const uint32_t* ipack,
                                                          const uint64_t* acc, const uint32_t* ev,
                                                          const uint32_t* ev_pos,
                                                          const uint64_t* rp_end,
                                                          const uint64_t* tok_base,
                                                          const unsigned long long* first_stop,
                                                          const uint32_t* recycled_d, Tokens t,
                                                          uint64_t* ctl_list, uint64_t ctl_cap,
                                                          unsigned long long* ctl_n) {
  __shared__ uint32_t sh[kLanes];
  __shared__ uint32_t s_loc[kLanes];
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * kLanes;
  const uint64_t b = b0 + threadIdx.x;
  const uint32_t recycled = *recycled_d;
  const uint64_t fs = *first_stop;
  if (b == a.n_blocks && fs == ~0ull) {  // kEof at the reader position after the last block
    const uint64_t o = tok_base[b];
    t.kind[o] = kTkStopEof;
    t.item[o] = b;
    t.len[o] = 0;
    t.pos[o] = b == 0 ? 0 : rp_end[b - 1];
    t.type[o] = 0;
  }
  const bool live = b < a.n_blocks && b <= fs;
  const uint32_t n = live ? static_cast<uint32_t>(acc[b]) : 0u;  // <= items of one 32 KiB block
  uint32_t tot;
  const uint32_t loc = rw_wg_scan(n, sh, &tot);
  s_loc[threadIdx.x] = loc;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < tot; k += kLanes) {
    uint32_t lo = 0, hi = kLanes;  // the last block j with s_loc[j] <= k
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_loc[mid] <= k) lo = mid; else hi = mid;
    }
    const uint64_t bj = b0 + lo, kk = k - s_loc[lo];
    const uint64_t i = base[bj] + kk, o = tok_base[bj] + kk;
    const uint32_t pk = ipack[i];  // the fill's header fields (no header re-read)
    const uint32_t length = pk & 0xffffu;
    const uint32_t type = (pk >> 16) & 0xffu;
    uint64_t rp;
    if (kk == 0) {
      rp = bj == 0 ? 0 : rp_end[bj - 1];
    } else {
      const uint32_t pp = ipack[i - 1];
      rp = it_off[i - 1] + ((pp >> 24) & 1u ? kLogRHdr : kLogHdr) + (pp & 0xffffu);
    }
    const uint8_t kind = it_old[i] ? kTkOldSkip : record_kind(type, eof_block(a, bj), recycled, a.mode);
    if (kind == kTkCtlComp || kind == kTkCtlTs) {  // decided on the host, in reader order
      const unsigned long long c = atomicAdd(ctl_n, 1ull);
      if (c < ctl_cap) ctl_list[c] = o;
    }
    t.kind[o] = kind;
    t.item[o] = i;
    t.len[o] = length;
    t.pos[o] = rp;
    t.type[o] = static_cast<uint8_t>(type);
  }
  if (!live) return;
  const uint32_t e = ev[b];
  if (!event_token(e)) return;
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  uint64_t rp = b == 0 ? 0 : rp_end[b - 1];  // reader position after the consumed items
  if (n) {
    const uint64_t il = base[b] + n - 1;
    const uint32_t pp = ipack[il];
    rp = it_off[il] + ((pp >> 24) & 1u ? kLogRHdr : kLogHdr) + (pp & 0xffffu);
  }
  const bool recyc_stop = (e == kEvChecksum || e == kEvBadLen) && recycled && a.mode == 0;
  uint8_t kind = e == kEvChecksum   ? kTkChecksum
                 : e == kEvBadLen   ? kTkBadLen
                 : e == kEvZero     ? kTkZero
                 : e == kEvOldStop  ? kTkStopOld
                 : e == kEvBadHeader ? kTkStopHeader
                                     : kTkStopBadLenEof;
  if (recyc_stop) kind = kTkStopRecycled;
  const uint64_t o = tok_base[b] + n;
  t.kind[o] = kind;
  t.item[o] = b;
  t.len[o] = static_cast<uint32_t>(end - (start + ev_pos[b]));  // drop_size: rest of the buffer
  t.pos[o] = rp;
  t.type[o] = 0;
}

__device__ __forceinline__ bool is_head(uint8_t k) { return k != kTkMiddle && k != kTkLast; }
__device__ __forceinline__ bool is_ctl(uint8_t k) { return k == kTkCtlComp || k == kTkCtlTs; }
__device__ __forceinline__ bool is_payload(uint8_t k) {
  return k == kTkFull || k == kTkFirst || k == kTkMiddle || k == kTkLast;
}

__global__ void __launch_bounds__(kLanes) rw_head_kernel(Tokens t, uint64_t n, uint64_t* head,
                                                         uint64_t* plen) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= n) return;
  head[i] = is_head(t.kind[i]) ? 1 : 0;
  plen[i] = is_payload(t.kind[i]) ? t.len[i] : 0;
}

// seg[i] = inclusive count of heads (0 = before the first head); per segment:
// head token, and the first Last (atomicMin)
__global__ void __launch_bounds__(kLanes) rw_seg_kernel(Tokens t, uint64_t n, const uint64_t* head,
                                                        uint64_t* seg, uint64_t* seg_head,
                                                        unsigned long long* seg_first_last) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= n) return;
  const uint64_t s = seg[i] + head[i];  // exclusive scan + own flag
  seg[i] = s;
  if (head[i]) seg_head[s] = i;
  if (t.kind[i] == kTkLast && s > 0) atomicMin(seg_first_last + s, static_cast<unsigned long long>(i));
}

// live[s]: in_fragmented_record holds inside segment s.  A First starts a
// fragmented record; a control record (types 9-11) keeps the state it finds
// (log_reader.cc:167-213), i.e. that of the segment before it -- a run of
// control-headed segments is resolved by walking back to the segment that
// decides; every other head clears it.  A segment is TRANSPARENT when its
// head is a control record and no record completes in it: the walk passes
// those and stops at the first other one.  The walk is capped at kLiveWalk
// segments (log::Writer writes at most a few control records in a row, so the
// cap is never reached by a writer's log); a head whose walk hits the cap is
// counted in *over and decided by the linear pass below instead (a crafted
// log of long control runs would otherwise cost O(run^2)).
constexpr uint32_t kLiveWalk = 64;
__global__ void __launch_bounds__(kLanes) rw_live_kernel(Tokens t, uint64_t n, const uint64_t* head,
                                                         const uint64_t* seg,
                                                         const uint64_t* seg_head,
                                                         const unsigned long long* seg_fl,
                                                         uint8_t* live, unsigned long long* over) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= n || !head[i]) return;
  const uint8_t k = t.kind[i];
  uint8_t l = k == kTkFirst ? 1 : 0;
  if (is_ctl(k)) {
    uint32_t steps = 0;
    for (uint64_t x = seg[i] - 1; x > 0; --x) {
      if (++steps > kLiveWalk) {
        atomicAdd(over, 1ull);
        break;
      }
      if (seg_fl[x] != ~0ull) break;  // a record completed there: not in a fragmented record
      const uint8_t kx = t.kind[seg_head[x]];
      if (kx == kTkFirst) {
        l = 1;
        break;
      }
      if (!is_ctl(kx)) break;
    }
  }
  live[seg[i]] = l;
}

// The linear form (runs only when a walk above hit its cap): nt[s] = 1 for the
// segments that are not transparent (segment 0, before the first head, is
// not); cnt = exclusive scan of nt; pos[cnt[x] + 1] = x for each such x; the
// segment that decides a control-headed segment s is pos[cnt[s]], the last
// non-transparent one before s -- what the walk finds.
__global__ void __launch_bounds__(kLanes) rw_live_nt_kernel(Tokens t, uint64_t n,
                                                            const uint64_t* head,
                                                            const uint64_t* seg,
                                                            const unsigned long long* seg_fl,
                                                            uint64_t* nt) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= n || !head[i]) return;
  const uint64_t s = seg[i];
  nt[s] = is_ctl(t.kind[i]) && seg_fl[s] == ~0ull ? 0 : 1;
}
__global__ void __launch_bounds__(kLanes) rw_live_pos_kernel(uint64_t ns, const uint64_t* nt,
                                                             const uint64_t* cnt, uint64_t* pos) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (s < ns && nt[s]) pos[cnt[s] + 1] = s;
}
__global__ void __launch_bounds__(kLanes) rw_live_fix_kernel(Tokens t, uint64_t n,
                                                             const uint64_t* head,
                                                             const uint64_t* seg,
                                                             const uint64_t* seg_head,
                                                             const unsigned long long* seg_fl,
                                                             const uint64_t* cnt,
                                                             const uint64_t* pos, uint8_t* live) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= n || !head[i] || !is_ctl(t.kind[i])) return;
  const uint64_t s = seg[i];
  const uint64_t x = pos[cnt[s]];
  live[s] = x >= 1 && seg_fl[x] == ~0ull && t.kind[seg_head[x]] == kTkFirst ? 1 : 0;
}

// reasons (forst_wal_report.reason)
enum : uint32_t {
  kRpPartial1 = 1, kRpPartial2, kRpMissing1, kRpMissing2, kRpMiddle, kRpChecksum, kRpBadLen,
  kRpTruncHeader, kRpTrailing, kRpTruncBody, kRpUnknown, kRpCompMultiple, kRpCompNotFirst,
  kRpCompDecode, kRpTsInterspersed, kRpTsDecode, kRpTsZero, kRpTsDuplicate,
};

struct Fsm {
  const uint64_t* seg;
  const uint64_t* seg_head;
  const unsigned long long* seg_first_last;
  const uint8_t* live;
  const uint64_t* pl;  // exclusive prefix of payload lengths
  const uint64_t* plen;
};

// the reader's fragment state entering head token i: in_fragmented_record
// and the size of scratch (the previous segment's payload since its head;
// control heads carry no payload)
__device__ __forceinline__ void prev_state(const Fsm& f, uint64_t i, bool* in_frag,
                                           uint64_t* scratch) {
  const uint64_t s = f.seg[i];
  *in_frag = false;
  *scratch = 0;
  if (s < 2) return;
  if (!f.live[s - 1] || f.seg_first_last[s - 1] != ~0ull) return;
  *in_frag = true;
  *scratch = f.pl[i] - f.pl[f.seg_head[s - 1]];
}

// host-decided reports of the control records (ctl_list sorted by token)
struct CtlReps {
  const uint64_t* tok;
  uint64_t n;
  const uint32_t* cnt;
  const uint32_t* reason;  // [n][kCtlRep]
  const uint64_t* bytes;
  __device__ uint64_t find(uint64_t i) const {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) / 2;
      if (tok[mid] < i) lo = mid + 1; else hi = mid;
    }
    return lo;
  }
};

// where the XXH3 state feeding a record was last reset: the log start, the
// token after an emitted record, or a First that starts over a partial
// record ("partial record without end(2)")
__device__ __forceinline__ bool hb_start(const Tokens& t, const Fsm& f, const uint64_t* n_emit,
                                         uint64_t p) {
  if (p == 0 || n_emit[p - 1]) return true;
  if (t.kind[p] != kTkFirst) return false;
  bool in_frag;
  uint64_t scratch;
  prev_state(f, p, &in_frag, &scratch);
  return in_frag && scratch;
}
constexpr uint32_t kHashWalk = 64;
__global__ void __launch_bounds__(kLanes) rw_hb_flag_kernel(Tokens t, Fsm f, uint64_t n,
                                                            const uint64_t* n_emit, uint64_t* fl) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i < n) fl[i] = hb_start(t, f, n_emit, i) ? 1u : 0u;
}
__global__ void __launch_bounds__(kLanes) rw_hb_pos_kernel(const uint64_t* fl, const uint64_t* cnt,
                                                           uint64_t n, uint64_t* pos) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i < n && fl[i]) pos[cnt[i]] = i;
}

// per token: emitted logical records (0/1) and reports -- or, with WRITE,
// the records and reports themselves at their scanned positions
template <bool WRITE>
__global__ void __launch_bounds__(kLanes) rw_emit_kernel(Tokens t, uint64_t n, Fsm f, int mode,
                                                         uint64_t* n_emit, uint64_t* n_rep,
                                                         const uint64_t* emit_at,
                                                         const uint64_t* rep_at, CtlReps cr,
                                                         forst_wal_records recs, uint64_t rec_cap,
                                                         forst_wal_reports reps, uint64_t rep_cap,
                                                         uint64_t* rec_hash_begin,
                                                         uint64_t* rec_last_tok,
                                                         const uint64_t* hb_cnt,
                                                         const uint64_t* hb_pos,
                                                         unsigned long long* hb_over) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (i >= n) return;
  const uint8_t k = t.kind[i];
  const bool strict = mode == 1 || mode == 2;  // kAbsoluteConsistency, kPointInTimeRecovery
  uint32_t reason[2] = {0, 0};
  uint64_t bytes[2] = {0, 0};
  int nr = 0;
  bool emit = false;
  uint64_t first = i;
  auto rep = [&](uint32_t r, uint64_t nb) {
    reason[nr] = r;
    bytes[nr] = nb;
    ++nr;
  };
  const uint64_t s = f.seg[i];
  if (k == kTkMiddle || k == kTkLast) {
    const bool live = s && f.live[s];
    const unsigned long long fl = s ? f.seg_first_last[s] : ~0ull;
    if (k == kTkMiddle) {
      if (!(live && (fl == ~0ull || i < fl))) rep(kRpMissing1, t.len[i]);
    } else if (live && fl == i) {
      emit = true;
      first = f.seg_head[s];
    } else {
      rep(kRpMissing2, t.len[i]);
    }
  } else {
    bool in_frag;
    uint64_t scratch;
    prev_state(f, i, &in_frag, &scratch);
    switch (k) {
      case kTkFull:
        if (in_frag && scratch) rep(kRpPartial1, scratch);
        emit = true;
        break;
      case kTkFirst:
        if (in_frag && scratch) rep(kRpPartial2, scratch);
        break;
      case kTkUnknown:
        rep(kRpUnknown, t.len[i] + (in_frag ? scratch : 0));
        break;
      case kTkOldSkip:
      case kTkZero:
      case kTkPBad:
        if (in_frag) rep(kRpMiddle, scratch);
        break;
      case kTkChecksum:
      case kTkBadLen:
        rep(k == kTkChecksum ? kRpChecksum : kRpBadLen, t.len[i]);
        if (in_frag) rep(kRpMiddle, scratch);
        break;
      case kTkPLen:
      case kTkPCrc:
        rep(k == kTkPCrc ? kRpChecksum : kRpBadLen, 0);
        if (in_frag) rep(kRpMiddle, scratch);
        break;
      case kTkStopHeader:
      case kTkPHeader:
        if (strict) rep(kRpTruncHeader, k == kTkPHeader ? 0 : t.len[i]);
        if (strict && in_frag) rep(kRpTrailing, scratch);
        break;
      case kTkStopEof:
      case kTkStopOld:
      case kTkPEof:
      case kTkPOld:
        if (strict && in_frag) rep(kRpTrailing, scratch);
        break;
      case kTkStopBadLenEof:
      case kTkPLenEof:
        if (strict) rep(kRpTruncBody, k == kTkPLenEof ? 0 : t.len[i]);
        break;
      case kTkCtlTs:
        if (in_frag && scratch) rep(kRpTsInterspersed, scratch);
        break;
      default:  // kTkStopRecycled: scratch cleared, no report; kTkCtlComp: host reports
        break;
    }
  }
  uint64_t xj = 0;
  uint32_t nx = 0;  // host-decided reports after the device's
  if (is_ctl(k) && cr.n) {
    xj = cr.find(i);
    if (xj < cr.n && cr.tok[xj] == i) nx = cr.cnt[xj];
  }
  if (!WRITE) {
    n_emit[i] = emit ? 1 : 0;
    n_rep[i] = static_cast<uint64_t>(nr) + nx;
    return;
  }
  if (emit) {
    const uint64_t j = emit_at[i];
    // the XXH3 state feeding this record was last reset where ReadRecord
    // started (the token after the previous emitted record) or at a
    // "partial record without end(2)" First; a Full record is hashed alone
    uint64_t hb = i;
    if (k == kTkLast && hb_pos) {  // the linear form (rw_hb_flag_kernel): the last start <= first
      hb = hb_pos[hb_cnt[first] + hb_start(t, f, n_emit, first) - 1];
    } else if (k == kTkLast) {
      // walk back over the tokens no record was emitted for, at most
      // kHashWalk of them (a crafted log of long non-emitting runs made this
      // O(run) on one thread); beyond that the host runs the linear form
      hb = first;
      uint32_t steps = 0;
      while (!hb_start(t, f, n_emit, hb)) {
        if (++steps > kHashWalk) {
          atomicAdd(hb_over, 1ull);
          break;
        }
        --hb;
      }
    }
    rec_hash_begin[j] = hb;
    rec_last_tok[j] = i;
    if (j < rec_cap) {
      recs.offset[j] = t.pos[first];  // Reader::LastRecordOffset
      recs.length[j] = f.pl[i] + f.plen[i] - f.pl[first];
      recs.n_fragments[j] = static_cast<uint32_t>(i - first + 1 - (is_ctl(t.kind[first]) ? 1 : 0));
    }
  }
  // unknown record type %u: the type byte as the reader's unsigned int
  const uint32_t ty = static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(t.type[i])));
  for (int r = 0; r < nr + static_cast<int>(nx); ++r) {
    const uint64_t j = rep_at[i] + r;
    if (j < rep_cap) {
      const bool dev = r < nr;
      if (reps.offset) reps.offset[j] = t.pos[i];
      if (reps.bytes) reps.bytes[j] = dev ? bytes[r] : cr.bytes[xj * kCtlRep + (r - nr)];
      if (reps.reason) reps.reason[j] = dev ? reason[r] : cr.reason[xj * kCtlRep + (r - nr)];
      if (reps.type) reps.type[j] = ty;
    }
  }
}

// control records' fields for the host: token, kind, payload offset and
// length, records emitted before it (first_record_read_)
struct CtlInfo {
  uint64_t tok;
  uint64_t payload;
  uint64_t emitted_before;
  uint32_t len;
  uint32_t kind;
};
__global__ void __launch_bounds__(kLanes) rw_ctl_info_kernel(Tokens t, const uint64_t* it_off,
                                                             const uint32_t* ipack,
                                                             const uint64_t* list, uint64_t n,
                                                             const uint64_t* emit_at,
                                                             CtlInfo* info) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (j >= n) return;
  const uint64_t q = list[j];
  const uint64_t it = t.item[q];
  const uint32_t pk = ipack[it];
  CtlInfo c;
  c.tok = q;
  c.payload = it_off[it] + ((pk >> 24) & 1u ? kLogRHdr : kLogHdr);
  c.emitted_before = emit_at[q];
  c.len = pk & 0xffffu;
  c.kind = t.kind[q];
  info[j] = c;
}

__global__ void __launch_bounds__(kLanes) rw_ctl_add_kernel(const uint64_t* tok, const uint32_t* cnt,
                                                            uint64_t n, uint64_t* n_rep) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (j < n) n_rep[tok[j]] += cnt[j];
}

// ---- hashing (wal_hash.h): record j = tokens hash_begin[j] .. last_tok[j],
// the fragments the XXH3 state was fed (use) -----------------------------------
struct RecFrags {
  const uint64_t* hash_begin;
  const uint64_t* last_tok;
  const uint8_t* kind;
  const uint64_t* item;
  const uint64_t* it_off;
  const uint32_t* ipack;  // item: length | type << 16 | recyclable << 24 (rw_fill)
  const uint64_t* seg;
  const uint8_t* live;
  const unsigned long long* seg_fl;
  __device__ uint64_t begin(uint64_t j) const { return hash_begin[j]; }
  __device__ uint64_t end(uint64_t j) const { return last_tok[j] + 1; }
  __device__ uint64_t header(uint64_t q) const { return it_off[item[q]]; }
  __device__ uint32_t hs(uint64_t q) const { return (ipack[item[q]] >> 24) & 1u ? kLogRHdr : kLogHdr; }
  __device__ uint32_t len(uint64_t q) const { return ipack[item[q]] & 0xffffu; }
  // fed to XXH3_64bits_update: a First always; a Middle / Last while
  // in_fragmented_record (log_reader.cc:119-157); a Full is hashed alone
  __device__ bool use(uint64_t q) const {
    const uint8_t k = kind[q];
    if (k == kTkFull || k == kTkFirst) return true;
    if (k != kTkMiddle && k != kTkLast) return false;
    const uint64_t s = seg[q];
    return s && live[s] && (seg_fl[s] == ~0ull || q <= seg_fl[s]);
  }
};

// an emitted record that is exactly a candidate takes the fused kernel's hash;
// need[j] = 1 for the others (hashed by hash_logical_records)
__global__ void __launch_bounds__(kLanes) rw_match_kernel(Tokens t, Fsm f, const uint64_t* hb,
                                                          const uint64_t* lt, uint64_t nr,
                                                          const Cand c, const uint64_t* cpos,
                                                          uint64_t n_long,
                                                          const uint64_t* cand_hash,
                                                          uint64_t* hash_out, uint64_t* need) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (j >= nr) return;
  const uint64_t i = lt[j];
  const uint64_t h = t.kind[i] == kTkFull ? i : f.seg_head[f.seg[i]];
  bool m = c.head != nullptr && hb[j] == h && (t.kind[h] == kTkFull || t.kind[h] == kTkFirst);
  if (m) {
    const uint64_t ih = t.item[h];
    const uint8_t hd = c.head[ih];
    m = hd && c.last[ih] == t.item[i];
    // (cpos: long | one-window positions; a short candidate's hash is in its ez)
    if (m)
      hash_out[j] = hd == 1   ? cand_hash[cpos[ih] & 0xffffffffu]
                    : hd == 3 ? cand_hash[n_long + (cpos[ih] >> 32)]
                              : c.ez[ih];
  }
  need[j] = m ? 0u : 1u;
}

__global__ void __launch_bounds__(kLanes) rw_need_list_kernel(const uint64_t* need,
                                                              const uint64_t* npos, uint64_t nr,
                                                              uint64_t* sub) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (j < nr && need[j]) sub[npos[j]] = j;
}

__global__ void __launch_bounds__(kLanes) rw_scatter_kernel(const uint64_t* sub, const uint64_t* h,
                                                            uint64_t n, uint64_t* out) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (k < n) out[sub[k]] = h[k];
}

// RecFrags over a sub-list of the records (the ones no candidate covers)
struct RecFragsSub {
  RecFrags r;
  const uint64_t* sub;
  __device__ uint64_t begin(uint64_t j) const { return r.begin(sub[j]); }
  __device__ uint64_t end(uint64_t j) const { return r.end(sub[j]); }
  __device__ uint64_t header(uint64_t q) const { return r.header(q); }
  __device__ uint32_t hs(uint64_t q) const { return r.hs(q); }
  __device__ uint32_t len(uint64_t q) const { return r.len(q); }
  __device__ bool use(uint64_t q) const { return r.use(q); }
};

__global__ void rw_recycled_kernel(RecoverArgs a, uint32_t* flag) {
  // Reader::recycled_: the first header of the file has a recyclable type
  // (log_reader.cc:480-483)
  *flag = a.log_len >= kLogHdr && recyclable_type(a.log[6]) ? 1u : 0u;
}

// the count pass's scalars gathered on the device, read back with ONE copy
// (six 8-byte copies to the host cost ~20 us each: round 6's recovery trace)
__global__ void rw_pick_kernel(uint64_t* o, const uint64_t* v) { *o = *v; }
__global__ void rw_counts_kernel(uint64_t* o, const uint64_t* rep_total,
                                 const unsigned long long* ctl_n,
                                 const unsigned long long* live_over, const uint8_t* last_kind,
                                 const uint64_t* last_pos) {
  o[1] = *rep_total;
  o[2] = *ctl_n;
  o[3] = *live_over;
  o[4] = last_kind ? *last_kind : 0u;
  o[5] = last_pos ? *last_pos : 0u;
}

size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

dim3 grid_for(uint64_t n) { return dim3(static_cast<uint32_t>((n + kLanes - 1) / kLanes ? (n + kLanes - 1) / kLanes : 1)); }

// a bump allocator over one scratch allocation; with p == nullptr it only
// measures (the same sequence of takes sizes the allocation)
struct Arena {
  uint8_t* p;
  size_t used;
  template <typename T>
  T* take(uint64_t count) {
    T* r = reinterpret_cast<T*>(p + used);
    used += up256(sizeof(T) * (count ? count : 1));
    return r;
  }
};

// phase-1 arrays (per log block)
struct P1 {
  uint64_t *cnt, *ibase, *acc, *rp_end, *tiles;
  uint32_t *ev, *ev_pos, *recycled;
  unsigned long long *first_stop, *ctl_n;
  void take(Arena& A, uint64_t nb) {
    cnt = A.take<uint64_t>(nb + 1);
    ibase = A.take<uint64_t>(nb + 1);
    acc = A.take<uint64_t>(nb + 1);
    rp_end = A.take<uint64_t>(nb + 1);
    tiles = A.take<uint64_t>((nb + 1) / kScanTile + 2);
    ev = A.take<uint32_t>(nb + 1);
    ev_pos = A.take<uint32_t>(nb + 1);
    recycled = A.take<uint32_t>(1);
    first_stop = A.take<unsigned long long>(1);
    ctl_n = A.take<unsigned long long>(1);
  }
};

constexpr uint64_t kCtlCap = 4096;
constexpr uint64_t kRawFirst = 65536;  // raw list entries that go ahead of the fused kernel

// phase-2 arrays (per item / token)
struct P2 {
  uint64_t *it_off, *crc_off;
  uint8_t* it_old;
  uint32_t *crc_len, *crc_stored, *ipack, *computed;
  // candidates (fused CRC + XXH3) and the rows kernel's list
  uint8_t* crc_ok;
  Cand c;
  uint64_t *fc, *fr, *cpos, *rpos, *l_p0, *cand_hash, *r_off, *r_item;
  uint32_t *l_len, *l_info, *l_first, *r_len;
  ShortList sl;

  Tokens t;
  uint64_t *ntok, *tok_base, *head, *plen, *pl, *seg, *seg_head, *n_emit, *n_rep, *emit_at, *rep_at,
      *tiles2, *ctl_list;
  unsigned long long *seg_fl, *live_over;
  uint8_t* live;
  void take(Arena& A, uint64_t ni, uint64_t nb, uint64_t nt) {
    it_off = A.take<uint64_t>(ni);
    it_old = A.take<uint8_t>(ni);
    crc_off = A.take<uint64_t>(ni);
    crc_len = A.take<uint32_t>(ni);
    crc_stored = A.take<uint32_t>(ni);
    ipack = A.take<uint32_t>(ni);
    computed = A.take<uint32_t>(ni);
    crc_ok = A.take<uint8_t>(ni);
    c.head = A.take<uint8_t>(ni);
    c.fused = A.take<uint8_t>(ni);
    c.ez = A.take<uint64_t>(ni + 1);  // (+1: the fused kernel loads entries i, i + 1)
    c.p0 = A.take<uint64_t>(ni);
    c.len = A.take<uint32_t>(ni);
    c.info = A.take<uint32_t>(ni);
    c.first = A.take<uint32_t>(ni);
    c.last = A.take<uint32_t>(ni);
    fc = A.take<uint64_t>(ni);
    fr = A.take<uint64_t>(ni);
    cpos = A.take<uint64_t>(ni);
    rpos = A.take<uint64_t>(ni);
    l_p0 = A.take<uint64_t>(ni);
    cand_hash = A.take<uint64_t>(ni);
    r_off = A.take<uint64_t>(ni);
    r_item = A.take<uint64_t>(ni);
    l_len = A.take<uint32_t>(ni);
    l_info = A.take<uint32_t>(ni);
    l_first = A.take<uint32_t>(ni);
    r_len = A.take<uint32_t>(ni);
    sl.item = A.take<uint64_t>(ni);
    sl.off = A.take<uint64_t>(ni);
    sl.len = A.take<uint32_t>(ni);
    sl.p0 = A.take<uint64_t>(ni);
    sl.plen = A.take<uint32_t>(ni);
    sl.computed = A.take<uint32_t>(ni);
    t.kind = A.take<uint8_t>(nt);
    t.item = A.take<uint64_t>(nt);
    t.len = A.take<uint32_t>(nt);
    t.pos = A.take<uint64_t>(nt);
    t.type = A.take<uint8_t>(nt);
    ntok = A.take<uint64_t>(nb + 2);
    tok_base = A.take<uint64_t>(nb + 2);
    head = A.take<uint64_t>(nt);
    plen = A.take<uint64_t>(nt);
    pl = A.take<uint64_t>(nt);
    seg = A.take<uint64_t>(nt);
    seg_head = A.take<uint64_t>(nt + 1);
    seg_fl = A.take<unsigned long long>(nt + 1);
    live = A.take<uint8_t>(nt + 1);
    n_emit = A.take<uint64_t>(nt);
    n_rep = A.take<uint64_t>(nt);
    emit_at = A.take<uint64_t>(nt);
    rep_at = A.take<uint64_t>(nt);
    tiles2 = A.take<uint64_t>(nt / kScanTile + 2);
    ctl_list = A.take<uint64_t>(kCtlCap);
    live_over = A.take<unsigned long long>(1);
  }
};

// the kSetCompressionType / timestamp-size records' reports, in reader
// order, from the state the reader keeps across the log
// (log_reader.cc:167-213, UpdateRecordedTimestampSize)
struct CtlHost {
  std::vector<uint64_t> tok;
  std::vector<uint32_t> cnt, reason;
  std::vector<uint64_t> bytes;
  bool unsupported = false;
};

void decide_controls(const std::vector<CtlInfo>& info, const std::vector<uint8_t>& payload,
                     const std::vector<uint64_t>& at, CtlHost* h) {
  bool comp_read = false;                      // compression_type_record_read_
  std::unordered_map<uint32_t, uint32_t> ts;   // recorded_cf_to_ts_sz_
  const size_t n = info.size();
  h->tok.resize(n);
  h->cnt.assign(n, 0);
  h->reason.assign(n * kCtlRep, 0);
  h->bytes.assign(n * kCtlRep, 0);
  for (size_t j = 0; j < n; ++j) {
    const CtlInfo& c = info[j];
    const uint8_t* p = payload.data() + at[j];
    h->tok[j] = c.tok;
    auto rep = [&](uint32_t r, uint64_t b) {
      h->reason[j * kCtlRep + h->cnt[j]] = r;
      h->bytes[j * kCtlRep + h->cnt[j]] = b;
      ++h->cnt[j];
    };
    if (c.kind == kTkCtlComp) {
      if (comp_read) rep(kRpCompMultiple, c.len);
      if (c.emitted_before) rep(kRpCompNotFirst, c.len);
      // CompressionTypeRecord::DecodeFrom (util/compression.h:1716): GetFixed32
      // consumes 4 bytes; CompressionType is an 8-bit enum (low byte)
      if (c.len < 4) {
        rep(kRpCompDecode, c.len);
      } else if (p[0] == 0x7) {  // kZSTD: a compressed WAL, not replayed here
        h->unsupported = true;
      } else if (p[0] != 0) {
        rep(kRpCompDecode, c.len - 4);
      } else {
        comp_read = true;  // InitCompression(kNoCompression): no decoder
      }
    } else {
      // UserDefinedTimestampSizeRecord::DecodeFrom (util/udt_util.h:46)
      if (c.len % 6) {
        rep(kRpTsDecode, c.len);
        continue;
      }
      for (uint32_t x = 0; x < c.len; x += 6) {
        const uint32_t cf = static_cast<uint32_t>(p[x]) | (static_cast<uint32_t>(p[x + 1]) << 8) |
                            (static_cast<uint32_t>(p[x + 2]) << 16) |
                            (static_cast<uint32_t>(p[x + 3]) << 24);
        const uint32_t sz = static_cast<uint32_t>(p[x + 4]) | (static_cast<uint32_t>(p[x + 5]) << 8);
        if (sz == 0) {
          rep(kRpTsZero, 0);
          break;
        }
        if (ts.count(cf)) {
          rep(kRpTsDuplicate, 0);
          break;
        }
        ts.emplace(cf, sz);
      }
    }
  }
}

}  // namespace

hipError_t launch_wal_recover(const uint8_t* log, uint64_t log_len, uint32_t log_number, int mode,
                              forst_wal_records recs, uint64_t rec_cap, forst_wal_reports reps,
                              uint64_t rep_cap, forst_wal_recover_result* res, hipStream_t st,
                              const char** name) {
  std::memset(res, 0, sizeof(*res));
  RecoverArgs a{log, log_len, (log_len + kLogBlock - 1) / kLogBlock, log_number, mode, 0};
  const uint64_t nb = a.n_blocks;
  *name = "rw_walk";
  hipError_t e;
  std::vector<void*> held;  // scratch allocations, freed stream-ordered on every exit
  auto fail = [&](hipError_t x) {
    for (auto it = held.rbegin(); it != held.rend(); ++it) (void)scratch_free(*it, st);
    return x;
  };
  auto alloc = [&](size_t bytes, void** p) {
    const hipError_t x = scratch_alloc(p, bytes, st);
    if (x == hipSuccess) held.push_back(*p);
    return x;
  };
  // phase 1: per-block item counts -> item total (sync 1)
  P1 q1;
  Arena M1{nullptr, 0};
  q1.take(M1, nb);
  void* s1 = nullptr;
  if ((e = alloc(M1.used, &s1)) != hipSuccess) return fail(e);
  Arena A1{static_cast<uint8_t*>(s1), 0};
  q1.take(A1, nb);
  uint64_t n_items = 0;
  if (nb) {
    hipLaunchKernelGGL(rw_count_kernel, grid_for(nb), dim3(kLanes), 0, st, a, q1.cnt);
    scan_u64(q1.cnt, nb, q1.tiles, q1.ibase, st);
  }
  hipLaunchKernelGGL(rw_recycled_kernel, dim3(1), dim3(1), 0, st, a, q1.recycled);
  if ((e = hipMemsetAsync(q1.first_stop, 0xff, 8, st)) != hipSuccess ||
      (e = hipMemsetAsync(q1.ctl_n, 0, 8, st)) != hipSuccess ||
      (nb && (e = hipMemcpyAsync(&n_items, q1.tiles + (nb + kScanTile - 1) / kScanTile, 8,
                                 hipMemcpyDeviceToHost, st)) != hipSuccess) ||
      (e = hipStreamSynchronize(st)) != hipSuccess)
    return fail(e);
  // phase 2: items, CRCs, block truncation, tokens, state machine; sized by
  // the same sequence of takes that lays the arrays out
  const uint64_t ni = n_items, nt_max = n_items + nb + 1;
  a.fuse = log_len >= 4096 && ni < 0xffffffffull ? 1 : 0;
  P2 q;
  Arena M2{nullptr, 0};
  q.take(M2, ni, nb, nt_max);
  void* s2 = nullptr;
  if ((e = alloc(M2.used, &s2)) != hipSuccess) return fail(e);
  Arena A{static_cast<uint8_t*>(s2), 0};
  q.take(A, ni, nb, nt_max);
  const Tokens& t = q.t;
  uint64_t n_cand = 0;
  AuxHold raw_hold;  // second stream of the raw CRC (beside the fused kernel)
  AuxStream* raw_aux = nullptr;
  uint64_t n_long = 0;  // candidates [0, n_long) long, then the one-window ones
  if (nb) {
    hipLaunchKernelGGL(rw_fill_kernel, grid_for(nb), dim3(kLanes), 0, st, a, q1.ibase, q1.cnt,
                       q.it_off,
                       q.it_old, q.crc_off, q.crc_len, q.crc_stored, q.ipack, q1.ev, q1.ev_pos);
    if (ni) {
      // candidates: the records a writer lays out, CRC'd and hashed by ONE
      // read of their bytes (the fused kernel); the other physical records
      // go to the rows kernel's CRC (sync: the two list sizes)
      (void)hipMemsetAsync(q.c.head, 0, ni, st);
      (void)hipMemsetAsync(q.c.fused, 0, ni, st);
      const uint64_t cg = (ni + kCandThreads - 1) / kCandThreads;
      const uint32_t ncu = static_cast<uint32_t>(device_info().num_cus);
      hipLaunchKernelGGL(rw_cand_kernel, dim3(static_cast<uint32_t>(cg < ncu ? cg : ncu)),
                         dim3(kCandThreads), 0, st, a, ni, q.it_off, q.it_old, q.ipack,
                         q.crc_stored, q.c);
      const bool packed = ni < (uint64_t(1) << 32);  // (a.fuse implies it)
      hipLaunchKernelGGL(rw_cand_flags_kernel, grid_for(ni), dim3(kLanes), 0, st, q.c, ni,
                         q.it_old, packed ? 1 : 0, q.fc, q.fr);
      const uint64_t nti = (ni + kScanTile - 1) / kScanTile;
      uint64_t cnt2[2] = {0, 0};
      if (packed) {
        scan_u64(q.fc, ni, q.tiles2, q.cpos, st);
        e = hipMemcpyAsync(&cnt2[0], q.tiles2 + nti, 8, hipMemcpyDeviceToHost, st);
      }
      scan_u64(q.fr, ni, q.tiles2, q.rpos, st);
      if (e == hipSuccess) e = hipMemcpyAsync(&cnt2[1], q.tiles2 + nti, 8, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e != hipSuccess) return fail(e);
      n_long = packed ? cnt2[0] & 0xffffffffu : 0;
      const uint64_t n_one = packed ? cnt2[0] >> 32 : 0;
      const uint64_t n_short = packed ? cnt2[1] & 0xffffffffu : 0;
      const uint64_t n_raw = packed ? cnt2[1] >> 32 : cnt2[1];
      n_cand = n_long + n_one;
      hipLaunchKernelGGL(rw_cand_list_kernel, grid_for(ni), dim3(kLanes), 0, st, q.c, ni, q.it_old,
                         packed ? 1 : 0, n_long, q.cpos, q.rpos, q.crc_off, q.crc_len, q.l_p0,
                         q.l_len, q.l_info, q.l_first, q.r_off, q.r_len, q.r_item, q.sl);
      // the raw path: the CRCs of the physical records the fused kernel does
      // not check (the rows kernels' raw mode, then their verdicts), and the
      // short candidates' XXH3 (their hash into ez[item])
      auto raw_path = [&](hipStream_t rs) -> hipError_t {
        BlockArgs cb{};
        cb.base = log;
        cb.base_len = log_len;
        cb.offsets = q.r_off;
        cb.sizes = q.r_len;
        cb.out32 = q.computed;
        cb.n = n_raw;
        const char* crc_name = nullptr;
        hipError_t r = launch_crc32c_blocks(kModeRaw, cb, rs, &crc_name);
        if (r != hipSuccess) return r;
        hipLaunchKernelGGL(rw_raw_ok_kernel, grid_for(n_raw), dim3(kLanes), 0, rs, q.r_item,
                           q.computed, n_raw, q.crc_stored, q.crc_ok);
        return hipGetLastError();
      };
      // crc_ok pre-filled with 0 (fail-closed): the fused kernel, the short
      // list and the raw path store every verdict
      if ((n_cand || n_raw || n_short) && (e = hipMemsetAsync(q.crc_ok, 0, ni, st)) != hipSuccess)
        return fail(e);
      // the short candidates (C5: 2.9 M Full records <= 240 B): CRC and XXH3
      // one per lane, ahead of the fused kernel on its stream (on a second
      // stream they would wait for the fused kernel's workgroups, which hold
      // all of the CUs' LDS, and run in its tail)
      if (n_short) {
#if FORST_REC_SHORT_ROWS
        // both on 16-lane rows, one pass over the list (xxh3.hip)
        if ((e = launch_wal_short_rows(log, log_len, q.sl.off, q.sl.len, q.sl.p0, q.sl.plen,
                                       q.sl.item, n_short, q.crc_stored, q.crc_ok, q.c.ez, st)) !=
            hipSuccess)
          return fail(e);
#else
        BlockArgs sb{};
        sb.base = log;
        sb.base_len = log_len;
        sb.offsets = q.sl.off;
        sb.sizes = q.sl.len;
        sb.out32 = q.sl.computed;
        sb.n = n_short;
        if ((e = launch_crc32c_raw_lanes(sb, st)) != hipSuccess) return fail(e);
        hipLaunchKernelGGL(rw_raw_ok_kernel, grid_for(n_short), dim3(kLanes), 0, st, q.sl.item,
                           q.sl.computed, n_short, q.crc_stored, q.crc_ok);
        if ((e = launch_xxh3_short_rows(log, log_len, q.sl.p0, q.sl.plen, n_short, q.sl.item,
                                        q.c.ez, st)) != hipSuccess)
          return fail(e);
#endif
      }
      // a long raw list (corrupted or re-typed logs) goes ahead of the fused
      // kernel too, for the same reason
      const bool raw_first = n_raw >= kRawFirst;
      if (raw_first && (e = raw_path(st)) != hipSuccess) return fail(e);
      if (n_cand) {
        BlockArgs fa{};
        fa.base = log;
        fa.base_len = log_len;
        fa.offsets = q.l_p0;
        fa.sizes = q.l_len;
        fa.init_crcs = q.l_info;
        fa.modifiers = q.l_first;
        fa.crc_ez = q.c.ez;
        fa.crc_ok = q.crc_ok;
        fa.out64 = q.cand_hash;
        fa.n = n_long;
        // a short raw list does not depend on the fused kernel (disjoint
        // items of crc_ok and ez): on a second stream, forked after the
        // memset, it runs in the fused kernel's launch tail
        if (FORST_REC_OVERLAP && n_raw && !raw_first &&
            (raw_aux = raw_hold.a = aux_acquire(st)) != nullptr &&
            (hipEventRecord(raw_aux->fork, st) != hipSuccess ||
             hipStreamWaitEvent(raw_aux->s, raw_aux->fork, 0) != hipSuccess)) {
          (void)hipGetLastError();
          raw_aux = nullptr;
        }
        const char* fname = nullptr;
        // the one-window records in a launch of their own: every row then
        // finishes its record in every step, where among long records a
        // finishing row costs the whole wave the finish code
        if (n_one) {
          BlockArgs fo = fa;
          fo.offsets = q.l_p0 + n_long;
          fo.sizes = q.l_len + n_long;
          fo.init_crcs = q.l_info + n_long;
          fo.modifiers = q.l_first + n_long;
          fo.out64 = q.cand_hash + n_long;
          fo.n = n_one;
          if ((e = launch_xxh3_frag_crc(fo, st, &fname)) != hipSuccess) return fail(e);
        }
        if ((e = launch_xxh3_frag_crc(fa, st, &fname)) != hipSuccess) return fail(e);
      }
      if (n_raw && !raw_first) {
        const hipStream_t rs = raw_aux ? raw_aux->s : st;
        e = raw_path(rs);
        // join (also on failure: the scratch is freed on st)
        if (raw_aux && (hipEventRecord(raw_aux->join, rs) != hipSuccess ||
                        hipStreamWaitEvent(st, raw_aux->join, 0) != hipSuccess)) {
          if (e == hipSuccess) e = hipErrorUnknown;
          (void)hipStreamSynchronize(rs);
        }
        if (e != hipSuccess) return fail(e);
      }
    }
    void* fbv = nullptr;
    if ((e = alloc(4 * nb, &fbv)) != hipSuccess) return fail(e);
    uint32_t* first_bad = static_cast<uint32_t*>(fbv);
    (void)hipMemsetAsync(first_bad, 0xff, 4 * nb, st);
    if (ni)
      hipLaunchKernelGGL(rw_block_bad_kernel, grid_for(ni), dim3(kLanes), 0, st, a, ni, q.it_off,
                         q.it_old, q.ipack, q.crc_ok, q1.ibase, q1.recycled, first_bad);
    hipLaunchKernelGGL(rw_block_kernel, grid_for(nb), dim3(kLanes), 0, st, a, q1.cnt, q1.ibase,
                       q.it_off, q.it_old, q.crc_off, q.crc_len, q.ipack, q.crc_ok, first_bad,
                       q1.ev, q1.ev_pos, q1.acc, q1.rp_end, q1.first_stop, q1.recycled);
  }
  hipLaunchKernelGGL(rw_ntok_kernel, grid_for(nb + 1), dim3(kLanes), 0, st, a, q1.acc, q1.ev,
                     q1.first_stop, q.ntok);
  scan_u64(q.ntok, nb + 1, q1.tiles, q.tok_base, st);
  uint64_t n_tok = 0;
  if ((e = hipMemcpyAsync(&n_tok, q1.tiles + (nb + 1 + kScanTile - 1) / kScanTile, 8,
                          hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (e = hipStreamSynchronize(st)) != hipSuccess)
    return fail(e);
  hipLaunchKernelGGL(rw_token_kernel, grid_for(nb + 1), dim3(kLanes), 0, st, a, q1.ibase, q.it_off,
                     q.it_old, q.ipack, q1.acc, q1.ev, q1.ev_pos, q1.rp_end, q.tok_base,
                     q1.first_stop, q1.recycled, t, q.ctl_list, kCtlCap, q1.ctl_n);
  const dim3 tg = grid_for(n_tok);
  hipLaunchKernelGGL(rw_head_kernel, tg, dim3(kLanes), 0, st, t, n_tok, q.head, q.plen);
  scan_u64(q.head, n_tok, q.tiles2, q.seg, st);
  scan_u64(q.plen, n_tok, q.tiles2, q.pl, st);
  (void)hipMemsetAsync(q.seg_fl, 0xff, 8 * (n_tok + 1), st);
  (void)hipMemsetAsync(q.live, 0, n_tok + 1, st);
  (void)hipMemsetAsync(q.live_over, 0, 8, st);
  hipLaunchKernelGGL(rw_seg_kernel, tg, dim3(kLanes), 0, st, t, n_tok, q.head, q.seg, q.seg_head,
                     q.seg_fl);
  hipLaunchKernelGGL(rw_live_kernel, tg, dim3(kLanes), 0, st, t, n_tok, q.head, q.seg, q.seg_head,
                     q.seg_fl, q.live, q.live_over);
  const Fsm f{q.seg, q.seg_head, q.seg_fl, q.live, q.pl, q.plen};
  forst_wal_records no_recs{};
  forst_wal_reports no_reps{};
  CtlReps cr{};
  uint64_t tot[2] = {0, 0};
  unsigned long long n_ctl = 0, live_over = 0;
  const uint64_t ntl = (n_tok + kScanTile - 1) / kScanTile;
  uint8_t last_kind = 0;
  uint64_t last_pos = 0;
  // the state machine's counts (emitted records, reports), the control-record
  // count and the stop token (one sync)
  void* cov = nullptr;
  if ((e = alloc(256, &cov)) != hipSuccess) return fail(e);
  uint64_t* counts = static_cast<uint64_t*>(cov);
  auto count_pass = [&]() -> hipError_t {
    hipLaunchKernelGGL(rw_emit_kernel<false>, tg, dim3(kLanes), 0, st, t, n_tok, f, mode, q.n_emit,
                       q.n_rep, nullptr, nullptr, cr, no_recs, 0, no_reps, 0, nullptr, nullptr,
                       nullptr, nullptr, nullptr);
    scan_u64(q.n_emit, n_tok, q.tiles2, q.emit_at, st);
    hipLaunchKernelGGL(rw_pick_kernel, dim3(1), dim3(1), 0, st, counts, q.tiles2 + ntl);
    scan_u64(q.n_rep, n_tok, q.tiles2, q.rep_at, st);  // (reuses the tiles: after the pick)
    hipLaunchKernelGGL(rw_counts_kernel, dim3(1), dim3(1), 0, st, counts, q.tiles2 + ntl, q1.ctl_n,
                       q.live_over, n_tok ? t.kind + n_tok - 1 : nullptr,
                       n_tok ? t.pos + n_tok - 1 : nullptr);
    uint64_t h[6];
    hipError_t r = hipMemcpyAsync(h, counts, sizeof(h), hipMemcpyDeviceToHost, st);
    if (r == hipSuccess) r = hipStreamSynchronize(st);
    if (r == hipSuccess) {
      tot[0] = h[0];
      tot[1] = h[1];
      n_ctl = h[2];
      live_over = h[3];
      last_kind = static_cast<uint8_t>(h[4]);
      last_pos = h[5];
    }
    return r;
  };
  if ((e = count_pass()) != hipSuccess) return fail(e);
  if (live_over) {  // a control run longer than the walk's cap: the linear form, then recount
    const uint64_t ns = n_tok + 1;  // segments 0..n_tok at most
    const uint64_t tl = up256(8 * (ns / kScanTile + 2));
    void* lin = nullptr;
    if ((e = alloc(3 * up256(8 * (ns + 1)) + tl, &lin)) != hipSuccess) return fail(e);
    uint64_t* nt_f = static_cast<uint64_t*>(lin);
    uint64_t* cnt = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(lin) + up256(8 * (ns + 1)));
    uint64_t* pos = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(lin) + 2 * up256(8 * (ns + 1)));
    uint64_t* tiles = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(lin) + 3 * up256(8 * (ns + 1)));
    (void)hipMemsetAsync(nt_f, 0, 8 * ns, st);
    (void)hipMemsetAsync(nt_f, 1, 1, st);  // segment 0: nt = 1 (little endian)
    hipLaunchKernelGGL(rw_live_nt_kernel, tg, dim3(kLanes), 0, st, t, n_tok, q.head, q.seg,
                       q.seg_fl, nt_f);
    scan_u64(nt_f, ns, tiles, cnt, st);
    hipLaunchKernelGGL(rw_live_pos_kernel, grid_for(ns), dim3(kLanes), 0, st, ns, nt_f, cnt, pos);
    hipLaunchKernelGGL(rw_live_fix_kernel, tg, dim3(kLanes), 0, st, t, n_tok, q.head, q.seg,
                       q.seg_head, q.seg_fl, cnt, pos, q.live);
    if ((e = count_pass()) != hipSuccess) return fail(e);
  }
  // control records (types 9-11): read back, decided in reader order on the
  // host, their reports added before the report scan is taken again
  CtlHost ch;
  if (n_ctl) {
    uint64_t* list = q.ctl_list;
    if (n_ctl > kCtlCap) {  // more than the inline list holds: collect them again
      void* big = nullptr;
      if ((e = alloc(8 * n_ctl + 8, &big)) != hipSuccess) return fail(e);
      list = static_cast<uint64_t*>(big);
      if ((e = hipMemsetAsync(q1.ctl_n, 0, 8, st)) != hipSuccess) return fail(e);
      hipLaunchKernelGGL(rw_token_kernel, grid_for(nb + 1), dim3(kLanes), 0, st, a, q1.ibase,
                         q.it_off, q.it_old, q.ipack, q1.acc, q1.ev, q1.ev_pos, q1.rp_end,
                         q.tok_base, q1.first_stop, q1.recycled, t, list,
                         static_cast<uint64_t>(n_ctl), q1.ctl_n);
    }
    void* cs = nullptr;
    if ((e = alloc(up256(sizeof(CtlInfo) * n_ctl), &cs)) != hipSuccess) return fail(e);
    CtlInfo* dinfo = static_cast<CtlInfo*>(cs);
    hipLaunchKernelGGL(rw_ctl_info_kernel, grid_for(n_ctl), dim3(kLanes), 0, st, t, q.it_off,
                       q.ipack, list, static_cast<uint64_t>(n_ctl), q.emit_at, dinfo);
    std::vector<CtlInfo> info(n_ctl);
    if ((e = hipMemcpyAsync(info.data(), dinfo, sizeof(CtlInfo) * n_ctl, hipMemcpyDeviceToHost,
                            st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
      return fail(e);
    std::sort(info.begin(), info.end(),
              [](const CtlInfo& x, const CtlInfo& y) { return x.tok < y.tok; });
    std::vector<uint64_t> at(n_ctl);
    uint64_t tot_pl = 0;
    for (uint64_t j = 0; j < n_ctl; ++j) {
      at[j] = tot_pl;
      tot_pl += info[j].len;
    }
    std::vector<uint8_t> payload(tot_pl + 1);
    for (uint64_t j = 0; j < n_ctl; ++j)  // (few, short records)
      if (info[j].len &&
          (e = hipMemcpyAsync(payload.data() + at[j], log + info[j].payload, info[j].len,
                              hipMemcpyDeviceToHost, st)) != hipSuccess)
        return fail(e);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return fail(e);
    decide_controls(info, payload, at, &ch);
    if (ch.unsupported) {
      res->unsupported = 1;
      return fail(hipSuccess);
    }
    // tok | cnt | reason | bytes, uploaded once
    void* xs = nullptr;
    const size_t sz_tok = up256(8 * n_ctl), sz_cnt = up256(4 * n_ctl),
                 sz_rs = up256(4 * kCtlRep * n_ctl), sz_by = up256(8 * kCtlRep * n_ctl);
    if ((e = alloc(sz_tok + sz_cnt + sz_rs + sz_by, &xs)) != hipSuccess) return fail(e);
    uint8_t* xb = static_cast<uint8_t*>(xs);
    cr.tok = reinterpret_cast<uint64_t*>(xb);
    cr.cnt = reinterpret_cast<uint32_t*>(xb + sz_tok);
    cr.reason = reinterpret_cast<uint32_t*>(xb + sz_tok + sz_cnt);
    cr.bytes = reinterpret_cast<uint64_t*>(xb + sz_tok + sz_cnt + sz_rs);
    cr.n = n_ctl;
    if ((e = hipMemcpyAsync(const_cast<uint64_t*>(cr.tok), ch.tok.data(), 8 * n_ctl,
                            hipMemcpyHostToDevice, st)) != hipSuccess ||
        (e = hipMemcpyAsync(const_cast<uint32_t*>(cr.cnt), ch.cnt.data(), 4 * n_ctl,
                            hipMemcpyHostToDevice, st)) != hipSuccess ||
        (e = hipMemcpyAsync(const_cast<uint32_t*>(cr.reason), ch.reason.data(),
                            4 * kCtlRep * n_ctl, hipMemcpyHostToDevice, st)) != hipSuccess ||
        (e = hipMemcpyAsync(const_cast<uint64_t*>(cr.bytes), ch.bytes.data(),
                            8 * kCtlRep * n_ctl, hipMemcpyHostToDevice, st)) != hipSuccess)
      return fail(e);
    hipLaunchKernelGGL(rw_ctl_add_kernel, grid_for(n_ctl), dim3(kLanes), 0, st, cr.tok, cr.cnt,
                       static_cast<uint64_t>(n_ctl), q.n_rep);
    scan_u64(q.n_rep, n_tok, q.tiles2, q.rep_at, st);
    if ((e = hipMemcpyAsync(&tot[1], q.tiles2 + ntl, 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
      return fail(e);
  }
  const uint64_t n_rec = tot[0], n_rp = tot[1];
  res->n_records = n_rec;
  res->n_reports = n_rp;
  res->n_physical = ni;
  switch (last_kind) {
    case kTkStopEof:
    case kTkPEof: res->stop_reason = FORST_WAL_STOP_EOF; break;
    case kTkStopOld:
    case kTkPOld: res->stop_reason = FORST_WAL_STOP_OLD_RECORD; break;
    case kTkStopHeader:
    case kTkPHeader: res->stop_reason = FORST_WAL_STOP_TRUNCATED_HEADER; break;
    case kTkStopBadLenEof:
    case kTkPLenEof: res->stop_reason = FORST_WAL_STOP_TRUNCATED_BODY; break;
    default: res->stop_reason = FORST_WAL_STOP_RECYCLED_TAIL; break;
  }
  res->stop_offset = last_pos;
  res->truncated = (n_rec > rec_cap || n_rp > rep_cap) ? 1u : 0u;
  // records + reports at their positions, then the hashes
  const uint64_t nr = n_rec;
  // full record list in scratch first (the caller's capacity may be short)
  forst_wal_records full{};
  uint64_t* hash_begin = nullptr;
  uint64_t* last_tok = nullptr;
  void* s4 = nullptr;
  if ((e = alloc(up256(8 * nr) * 5 + up256(4 * nr), &s4)) != hipSuccess) return fail(e);
  {
    Arena A4{static_cast<uint8_t*>(s4), 0};
    full.offset = A4.take<uint64_t>(nr);
    full.length = A4.take<uint64_t>(nr);
    full.hash = A4.take<uint64_t>(nr);
    full.n_fragments = A4.take<uint32_t>(nr);
    // the caller's arrays hold every record: the kernels write them directly
    // (no copy-out; C5: four 80 MB device copies, 0.11 ms of a recovery)
    if (nr <= rec_cap) {
      if (recs.offset) full.offset = recs.offset;
      if (recs.length) full.length = recs.length;
      if (recs.hash) full.hash = recs.hash;
      if (recs.n_fragments) full.n_fragments = recs.n_fragments;
    }
    hash_begin = A4.take<uint64_t>(nr);
    last_tok = A4.take<uint64_t>(nr);
  }
  unsigned long long* hb_over = q.live_over;  // (reused: rw_live is done with it)
  (void)hipMemsetAsync(hb_over, 0, 8, st);
  hipLaunchKernelGGL(rw_emit_kernel<true>, tg, dim3(kLanes), 0, st, t, n_tok, f, mode, q.n_emit,
                     nullptr, q.emit_at, q.rep_at, cr, full, nr, reps, rep_cap, hash_begin,
                     last_tok, nullptr, nullptr, hb_over);
  if (nr) {
    // records that are exactly a candidate already have their hash (the
    // fused kernel); the rest are hashed here (sync: how many)
    void* s5 = nullptr;
    if ((e = alloc(up256(8 * nr) * 4 + up256(8 * (nr / kScanTile + 2)), &s5)) != hipSuccess)
      return fail(e);
    Arena A5{static_cast<uint8_t*>(s5), 0};
    uint64_t* need = A5.take<uint64_t>(nr);
    uint64_t* npos = A5.take<uint64_t>(nr);
    uint64_t* sub = A5.take<uint64_t>(nr);
    uint64_t* hsub = A5.take<uint64_t>(nr);
    uint64_t* tiles5 = A5.take<uint64_t>(nr / kScanTile + 2);
    Cand cm = q.c;
    if (!ni) cm.head = nullptr;
    uint64_t n_need = 0, over = 0;
    auto match = [&]() {
      hipLaunchKernelGGL(rw_match_kernel, grid_for(nr), dim3(kLanes), 0, st, t, f, hash_begin,
                         last_tok, nr, cm, q.cpos, n_long, q.cand_hash, full.hash, need);
      scan_u64(need, nr, tiles5, npos, st);
      hipError_t r = hipMemcpyAsync(&n_need, tiles5 + (nr + kScanTile - 1) / kScanTile, 8,
                                    hipMemcpyDeviceToHost, st);
      if (r == hipSuccess) r = hipMemcpyAsync(&over, hb_over, 8, hipMemcpyDeviceToHost, st);
      if (r == hipSuccess) r = hipStreamSynchronize(st);
      return r;
    };
    if ((e = match()) != hipSuccess) return fail(e);
    if (over) {  // a non-emitting run longer than the walk's cap: the linear form, again
      const uint64_t nt1 = n_tok + 1;
      void* hv = nullptr;
      if ((e = alloc(up256(8 * nt1) * 3 + up256(8 * (nt1 / kScanTile + 2)), &hv)) != hipSuccess)
        return fail(e);
      Arena AH{static_cast<uint8_t*>(hv), 0};
      uint64_t* fl = AH.take<uint64_t>(nt1);
      uint64_t* cnt = AH.take<uint64_t>(nt1);
      uint64_t* pos = AH.take<uint64_t>(nt1);
      uint64_t* tl = AH.take<uint64_t>(nt1 / kScanTile + 2);
      hipLaunchKernelGGL(rw_hb_flag_kernel, tg, dim3(kLanes), 0, st, t, f, n_tok, q.n_emit, fl);
      scan_u64(fl, n_tok, tl, cnt, st);
      hipLaunchKernelGGL(rw_hb_pos_kernel, tg, dim3(kLanes), 0, st, fl, cnt, n_tok, pos);
      hipLaunchKernelGGL(rw_emit_kernel<true>, tg, dim3(kLanes), 0, st, t, n_tok, f, mode,
                         q.n_emit, nullptr, q.emit_at, q.rep_at, cr, full, nr, reps, rep_cap,
                         hash_begin, last_tok, cnt, pos, hb_over);
      if ((e = match()) != hipSuccess) return fail(e);
    }
    if (n_need) {
      hipLaunchKernelGGL(rw_need_list_kernel, grid_for(nr), dim3(kLanes), 0, st, need, npos, nr,
                         sub);
      const RecFrags rf{hash_begin, last_tok, t.kind, t.item, q.it_off, q.ipack, q.seg, q.live,
                        q.seg_fl};
      const RecFragsSub rs{rf, sub};
      e = hash_logical_records(log, log_len, rs, n_need, hsub, st, name, false);
      if (e == hipSuccess)
        hipLaunchKernelGGL(rw_scatter_kernel, grid_for(n_need), dim3(kLanes), 0, st, sub, hsub,
                           n_need, full.hash);
    }
  }
  // copy the (capacity-limited) record list out
  const uint64_t nc = nr < rec_cap ? nr : rec_cap;
  if (e == hipSuccess && nc) {
    if (recs.offset && recs.offset != full.offset)
      e = hipMemcpyAsync(recs.offset, full.offset, 8 * nc, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && recs.length && recs.length != full.length)
      e = hipMemcpyAsync(recs.length, full.length, 8 * nc, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && recs.hash && recs.hash != full.hash)
      e = hipMemcpyAsync(recs.hash, full.hash, 8 * nc, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && recs.n_fragments && recs.n_fragments != full.n_fragments)
      e = hipMemcpyAsync(recs.n_fragments, full.n_fragments, 4 * nc, hipMemcpyDeviceToDevice, st);
  }
  if (e == hipSuccess) e = hipGetLastError();
  *name = "wal_recover";
  hipError_t fe = hipSuccess;
  for (auto it = held.rbegin(); it != held.rend(); ++it) {
    const hipError_t x = scratch_free(*it, st);
    if (fe == hipSuccess) fe = x;
  }
  return e != hipSuccess ? e : fe;
}

}  // namespace forst
