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
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "../../include/forst_checksum.h"
#include "device_common.h"
#include "engine.h"
#include "scan_common.h"
#include "wal_hash.h"

namespace forst {
namespace {

constexpr uint32_t kLogBlock = 32768;  // db/log_format.h:45
constexpr uint32_t kLogHdr = 7;        // :48
constexpr uint32_t kLogRHdr = 11;      // :52
constexpr uint32_t kLanes = 256;

// block terminal events (the reader's result when it leaves the block)
enum : uint32_t {
  kEvNone = 0,     // block consumed (trailer < header size skipped)
  kEvChecksum,     // kBadRecordChecksum: rest of block dropped
  kEvBadLen,       // kBadRecordLen, not at EOF: as a checksum error
  kEvZero,         // kZeroType, length 0 -> kBadRecord
  kEvOldStop,      // kOldRecord (not skip mode): reading ends
  kEvBadHeader,    // truncated header at EOF (kBadHeader): reading ends
  kEvBadLenEof,    // kBadRecordLen at EOF: reading ends
};

// token kinds
enum : uint8_t {
  kTkFull = 1, kTkFirst, kTkMiddle, kTkLast, kTkUnknown, kTkOldSkip, kTkZero, kTkChecksum,
  kTkBadLen, kTkStopHeader, kTkStopBadLenEof, kTkStopOld, kTkStopRecycled, kTkStopEof,
};

struct RecoverArgs {
  const uint8_t* log;
  uint64_t log_len;
  uint64_t n_blocks;
  uint32_t log_number;
  int mode;  // WALRecoveryMode
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

// ---- walk -------------------------------------------------------------------
// items: header offsets of the physical records the reader parses in block b
// (REC: CRC to check; OLD: skipped old record, kSkipAnyCorruptedRecords)
template <bool FILL>
__device__ uint32_t rw_walk_block(const RecoverArgs& a, uint64_t b, uint32_t* ev, uint32_t* ev_pos,
                                  uint64_t base, uint64_t* it_off, uint8_t* it_old,
                                  uint64_t* crc_off, uint32_t* crc_len, uint32_t* crc_stored,
                                  uint32_t* ipack) {
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  const bool eof_block = end - start < kLogBlock;  // ReadMore read short: eof_
  uint64_t pos = start;
  uint32_t n = 0, e = kEvNone;
  while (true) {
    const uint64_t rem = end - pos;
    if (rem < kLogHdr) {  // trailer skipped, or a truncated header at EOF
      if (rem > 0 && eof_block) e = kEvBadHeader;
      break;
    }
    const uint8_t* h = a.log + pos;
    const uint32_t length = static_cast<uint32_t>(h[4]) | (static_cast<uint32_t>(h[5]) << 8);
    const uint32_t type = h[6];
    const bool recyc = recyclable_type(type);
    const uint32_t hs = recyc ? kLogRHdr : kLogHdr;
    if (rem < hs) {
      if (eof_block) e = kEvBadHeader;
      break;
    }
    if (hs + length > rem) {
      e = eof_block ? kEvBadLenEof : kEvBadLen;
      break;
    }
    if (recyc && ld_le32(h + 7) != a.log_number) {
      if (a.mode != 3) {  // not kSkipAnyCorruptedRecords: reading ends here
        e = kEvOldStop;
        break;
      }
      if (FILL) {
        it_off[base + n] = pos;
        it_old[base + n] = 1;
        crc_off[base + n] = 0;
        crc_len[base + n] = 0;
        ipack[base + n] = length | (type << 16) | (recyc ? 1u << 24 : 0u);
      }
      ++n;
      pos += hs + length;
      continue;
    }
    if (type == 0 && length == 0) {
      e = kEvZero;
      break;
    }
    if (FILL) {
      it_off[base + n] = pos;
      it_old[base + n] = 0;
      crc_off[base + n] = pos + 6;
      crc_len[base + n] = hs + length - 6;
      crc_stored[base + n] = unmask(ld_le32(h));  // log_reader.cc:522-523
      ipack[base + n] = length | (type << 16) | (recyc ? 1u << 24 : 0u);
    }
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
  cnt[b] = rw_walk_block<false>(a, b, &ev, &ep, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr);
}

__global__ void __launch_bounds__(kLanes) rw_fill_kernel(RecoverArgs a, const uint64_t* base,
                                                         uint64_t* it_off, uint8_t* it_old,
                                                         uint64_t* crc_off, uint32_t* crc_len,
                                                         uint32_t* crc_stored, uint32_t* ipack,
                                                         uint32_t* ev, uint32_t* ev_pos) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (b >= a.n_blocks) return;
  rw_walk_block<true>(a, b, &ev[b], &ev_pos[b], base[b], it_off, it_old, crc_off, crc_len,
                      crc_stored, ipack);
}

// ---- per block: CRC truncation, reader position, stop -------------------------
// acc[b] = items consumed before the first CRC mismatch; the event becomes
// kEvChecksum at that record; rp_end[b] = reader position when leaving the
// block (end of the last consumed record, or the block end after a
// buffer-clearing event); ntok[b] = consumed items + the event token
__global__ void __launch_bounds__(kLanes) rw_block_kernel(RecoverArgs a, const uint64_t* cnt,
                                                          const uint64_t* base,
                                                          const uint64_t* it_off,
                                                          const uint8_t* it_old,
                                                          const uint64_t* crc_off,
                                                          const uint32_t* crc_len,
                                                          const uint32_t* crc_stored,
                                                          const uint32_t* computed, uint32_t* ev,
                                                          uint32_t* ev_pos, uint64_t* acc,
                                                          uint64_t* rp_end,
                                                          unsigned long long* first_stop,
                                                          uint32_t recycled) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (b >= a.n_blocks) return;
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  const uint64_t n = cnt[b], i0 = base[b];
  uint64_t k = 0, last_end = start;
  uint32_t e = ev[b], ep = ev_pos[b];
  // the fill's per-item arrays (stored CRC, record extent); the header is
  // re-read only for skipped old records (kSkipAnyCorruptedRecords)
  for (; k < n; ++k) {
    if (it_old[i0 + k]) {
      const uint8_t* h = a.log + it_off[i0 + k];
      const uint32_t length = static_cast<uint32_t>(h[4]) | (static_cast<uint32_t>(h[5]) << 8);
      last_end = it_off[i0 + k] + (recyclable_type(h[6]) ? kLogRHdr : kLogHdr) + length;
      continue;
    }
    if (crc_stored[i0 + k] != computed[i0 + k]) {
      e = kEvChecksum;
      ep = static_cast<uint32_t>(crc_off[i0 + k] - 6 - start);
      break;
    }
    last_end = crc_off[i0 + k] + crc_len[i0 + k];
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
  const bool stop = e == kEvOldStop || e == kEvBadHeader || e == kEvBadLenEof ||
                    ((e == kEvChecksum || e == kEvBadLen) && recycled && a.mode == 0);
  if (stop) atomicMin(first_stop, static_cast<unsigned long long>(b));
}

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
  ntok[b] = b > *first_stop ? 0 : acc[b] + (ev[b] != kEvNone ? 1 : 0);
}

// tokens: kind, item (physical record index; events: block), payload length
// (events: dropped bytes), reader position (physical_record_offset of the
// reference, end_of_buffer_offset_ - buffer_.size() before the read), type
struct Tokens {
  uint8_t* kind;
  uint64_t* item;
  uint32_t* len;
  uint64_t* pos;
  uint8_t* type;
};

__global__ void __launch_bounds__(kLanes) rw_token_kernel(RecoverArgs a, const uint64_t* base,
                                                          const uint64_t* it_off,
                                                          const uint8_t* it_old,
                                                          const uint32_t* ipack,
                                                          const uint64_t* acc, const uint32_t* ev,
                                                          const uint32_t* ev_pos,
                                                          const uint64_t* rp_end,
                                                          const uint64_t* tok_base,
                                                          const unsigned long long* first_stop,
                                                          uint32_t recycled, Tokens t,
                                                          uint32_t* unsupported) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLanes + threadIdx.x;
  if (b > a.n_blocks) return;
  uint64_t o = tok_base[b];
  if (b == a.n_blocks) {
    if (*first_stop == ~0ull) {  // kEof at the reader position after the last block
      t.kind[o] = kTkStopEof;
      t.item[o] = b;
      t.len[o] = 0;
      t.pos[o] = b == 0 ? 0 : rp_end[b - 1];
      t.type[o] = 0;
    }
    return;
  }
  if (b > *first_stop) return;
  const uint64_t start = b * kLogBlock;
  const uint64_t end = start + kLogBlock < a.log_len ? start + kLogBlock : a.log_len;
  uint64_t rp = b == 0 ? 0 : rp_end[b - 1];  // reader position entering the block
  const uint64_t n = acc[b], i0 = base[b];
  for (uint64_t k = 0; k < n; ++k, ++o) {
    const uint64_t off = it_off[i0 + k];
    const uint32_t pk = ipack[i0 + k];  // the fill's header fields (no header re-read)
    const uint32_t length = pk & 0xffffu;
    const uint32_t type = (pk >> 16) & 0xffu;
    const uint32_t nt = (type >= 5 && type <= 8) ? type - 4 : type;  // recyclable -> legacy
    uint8_t kind = nt == 1   ? kTkFull
                   : nt == 2 ? kTkFirst
                   : nt == 3 ? kTkMiddle
                   : nt == 4 ? kTkLast
                             : kTkUnknown;
    if (it_old[i0 + k]) kind = kTkOldSkip;
    // kSetCompressionType / (recyclable) kUserDefinedTimestampSizeType records
    // change how the reader decodes what follows: not handled on the device
    if (kind == kTkUnknown && (type == 9 || type == 10 || type == 11)) atomicOr(unsupported, 1u);
    t.kind[o] = kind;
    t.item[o] = i0 + k;
    t.len[o] = length;
    t.pos[o] = rp;
    t.type[o] = static_cast<uint8_t>(type);
    rp = off + ((pk >> 24) & 1u ? kLogRHdr : kLogHdr) + length;
  }
  const uint32_t e = ev[b];
  if (e == kEvNone) return;
  const bool recyc_stop = (e == kEvChecksum || e == kEvBadLen) && recycled && a.mode == 0;
  uint8_t kind = e == kEvChecksum   ? kTkChecksum
                 : e == kEvBadLen   ? kTkBadLen
                 : e == kEvZero     ? kTkZero
                 : e == kEvOldStop  ? kTkStopOld
                 : e == kEvBadHeader ? kTkStopHeader
                                     : kTkStopBadLenEof;
  if (recyc_stop) kind = kTkStopRecycled;
  t.kind[o] = kind;
  t.item[o] = b;
  t.len[o] = static_cast<uint32_t>(end - (start + ev_pos[b]));  // drop_size: rest of the buffer
  t.pos[o] = rp;
  t.type[o] = 0;
}

__device__ __forceinline__ bool is_head(uint8_t k) { return k != kTkMiddle && k != kTkLast; }
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

// reasons (forst_wal_report.reason)
enum : uint32_t {
  kRpPartial1 = 1, kRpPartial2, kRpMissing1, kRpMissing2, kRpMiddle, kRpChecksum, kRpBadLen,
  kRpTruncHeader, kRpTrailing, kRpTruncBody, kRpUnknown,
};

struct Fsm {
  const uint64_t* seg;
  const uint64_t* seg_head;
  const unsigned long long* seg_first_last;
  const uint64_t* pl;  // exclusive prefix of payload lengths
  const uint64_t* plen;
};

// the reader's fragment state entering head token i: the previous segment
// is an unfinished First segment (in_fragmented_record), scratch = its bytes
__device__ __forceinline__ void prev_state(const Tokens& t, const Fsm& f, uint64_t i, bool* in_frag,
                                           uint64_t* scratch) {
  const uint64_t s = f.seg[i];
  *in_frag = false;
  *scratch = 0;
  if (s < 2) return;
  const uint64_t h = f.seg_head[s - 1];
  if (t.kind[h] != kTkFirst || f.seg_first_last[s - 1] != ~0ull) return;
  *in_frag = true;
  *scratch = f.pl[i] - f.pl[h];  // B + M payloads up to this head
}

// per token: emitted logical records (0/1) and reports (0-2) -- or, with
// WRITE, the records and reports themselves at their scanned positions
template <bool WRITE>
__global__ void __launch_bounds__(kLanes) rw_emit_kernel(Tokens t, uint64_t n, Fsm f, int mode,
                                                         uint64_t* n_emit, uint64_t* n_rep,
                                                         const uint64_t* emit_at,
                                                         const uint64_t* rep_at,
                                                         forst_wal_records recs, uint64_t rec_cap,
                                                         forst_wal_reports reps, uint64_t rep_cap,
                                                         uint64_t* rec_head_tok) {
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
    const uint64_t h = s ? f.seg_head[s] : ~0ull;
    const bool b_seg = s && t.kind[h] == kTkFirst;
    const unsigned long long fl = s ? f.seg_first_last[s] : ~0ull;
    if (k == kTkMiddle) {
      if (!(b_seg && (fl == ~0ull || i < fl))) rep(kRpMissing1, t.len[i]);
    } else if (b_seg && fl == i) {
      emit = true;
      first = h;
    } else {
      rep(kRpMissing2, t.len[i]);
    }
  } else {
    bool in_frag;
    uint64_t scratch;
    prev_state(t, f, i, &in_frag, &scratch);
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
        if (in_frag) rep(kRpMiddle, scratch);
        break;
      case kTkChecksum:
      case kTkBadLen:
        rep(k == kTkChecksum ? kRpChecksum : kRpBadLen, t.len[i]);
        if (in_frag) rep(kRpMiddle, scratch);
        break;
      case kTkStopHeader:
        if (strict) rep(kRpTruncHeader, t.len[i]);
        if (strict && in_frag) rep(kRpTrailing, scratch);
        break;
      case kTkStopEof:
      case kTkStopOld:
        if (strict && in_frag) rep(kRpTrailing, scratch);
        break;
      case kTkStopBadLenEof:
        if (strict) rep(kRpTruncBody, t.len[i]);
        break;
      default:  // kTkStopRecycled: scratch cleared, no report
        break;
    }
  }
  if (!WRITE) {
    n_emit[i] = emit ? 1 : 0;
    n_rep[i] = static_cast<uint64_t>(nr);
    return;
  }
  if (emit) {
    const uint64_t j = emit_at[i];
    if (j < rec_cap) {
      recs.offset[j] = t.pos[first];  // Reader::LastRecordOffset
      recs.length[j] = f.pl[i] + f.plen[i] - f.pl[first];
      recs.n_fragments[j] = static_cast<uint32_t>(i - first + 1);
      rec_head_tok[j] = first;
    }
  }
  for (int r = 0; r < nr; ++r) {
    const uint64_t j = rep_at[i] + r;
    if (j < rep_cap) {
      if (reps.offset) reps.offset[j] = t.pos[i];
      if (reps.bytes) reps.bytes[j] = bytes[r];
      if (reps.reason) reps.reason[j] = reason[r];
      if (reps.type) reps.type[j] = t.type[i];
    }
  }
}

// ---- hashing (wal_hash.h): record j = tokens head_tok[j] .. + n_frag[j] - 1 --
struct RecFrags {
  const uint64_t* head_tok;
  const uint32_t* n_frag;
  const uint64_t* item;
  const uint64_t* it_off;
  const uint32_t* ipack;  // item: length | type << 16 | recyclable << 24 (rw_fill)
  __device__ uint64_t begin(uint64_t j) const { return head_tok[j]; }
  __device__ uint64_t end(uint64_t j) const { return head_tok[j] + n_frag[j]; }
  __device__ uint64_t header(uint64_t q) const { return it_off[item[q]]; }
  __device__ uint32_t hs(uint64_t q) const { return (ipack[item[q]] >> 24) & 1u ? kLogRHdr : kLogHdr; }
  __device__ uint32_t len(uint64_t q) const { return ipack[item[q]] & 0xffffu; }
  __device__ bool use(uint64_t) const { return true; }
};

__global__ void rw_recycled_kernel(RecoverArgs a, uint32_t* flag) {
  // Reader::recycled_: the first header of the file has a recyclable type
  // (log_reader.cc:480-483)
  *flag = a.log_len >= kLogHdr && recyclable_type(a.log[6]) ? 1u : 0u;
}

size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

dim3 grid_for(uint64_t n) { return dim3(static_cast<uint32_t>((n + kLanes - 1) / kLanes ? (n + kLanes - 1) / kLanes : 1)); }

// a bump allocator over one scratch allocation
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

}  // namespace

hipError_t launch_wal_recover(const uint8_t* log, uint64_t log_len, uint32_t log_number, int mode,
                              forst_wal_records recs, uint64_t rec_cap, forst_wal_reports reps,
                              uint64_t rep_cap, forst_wal_recover_result* res, hipStream_t st,
                              const char** name) {
  std::memset(res, 0, sizeof(*res));
  RecoverArgs a{log, log_len, (log_len + kLogBlock - 1) / kLogBlock, log_number, mode};
  const uint64_t nb = a.n_blocks;
  *name = "rw_walk";
  hipError_t e;
  // phase 1: per-block item counts -> item total (sync 1)
  const size_t p1 = 4 * up256(8 * (nb + 1)) + up256(8 * (nb / kScanTile + 2)) + 4 * up256(4 * (nb + 1)) +
                    up256(8) + 4096;
  void* s1 = nullptr;
  if ((e = scratch_alloc(&s1, p1, st)) != hipSuccess) return e;
  Arena A1{static_cast<uint8_t*>(s1), 0};
  uint64_t* cnt = A1.take<uint64_t>(nb + 1);
  uint64_t* ibase = A1.take<uint64_t>(nb + 1);
  uint64_t* acc = A1.take<uint64_t>(nb + 1);
  uint64_t* rp_end = A1.take<uint64_t>(nb + 1);
  uint64_t* tiles = A1.take<uint64_t>(nb / kScanTile + 2);
  uint32_t* ev = A1.take<uint32_t>(nb + 1);
  uint32_t* ev_pos = A1.take<uint32_t>(nb + 1);
  uint32_t* recycled_d = A1.take<uint32_t>(1);
  uint32_t* unsup_d = A1.take<uint32_t>(1);
  unsigned long long* first_stop = A1.take<unsigned long long>(1);
  uint64_t n_items = 0;
  uint32_t recycled = 0;
  if (nb) {
    hipLaunchKernelGGL(rw_count_kernel, grid_for(nb), dim3(kLanes), 0, st, a, cnt);
    scan_u64(cnt, nb, tiles, ibase, st);
  }
  hipLaunchKernelGGL(rw_recycled_kernel, dim3(1), dim3(1), 0, st, a, recycled_d);
  if ((e = hipMemsetAsync(first_stop, 0xff, 8, st)) != hipSuccess ||
      (e = hipMemsetAsync(unsup_d, 0, 4, st)) != hipSuccess ||
      (nb && (e = hipMemcpyAsync(&n_items, tiles + (nb + kScanTile - 1) / kScanTile, 8,
                                 hipMemcpyDeviceToHost, st)) != hipSuccess) ||
      (e = hipMemcpyAsync(&recycled, recycled_d, 4, hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (e = hipStreamSynchronize(st)) != hipSuccess) {
    (void)scratch_free(s1, st);
    return e;
  }
  // phase 2: items, CRCs, block truncation, tokens, state machine
  const uint64_t ni = n_items, nt_max = n_items + nb + 1;
  const size_t p2 = 3 * up256(8 * ni) + up256(ni) + 4 * up256(4 * ni) +  // items
                    up256(nt_max) * 2 + up256(8 * nt_max) * 2 + up256(4 * nt_max) +  // tokens
                    up256(8 * (nb + 2)) +                                          // token base
                    up256(8 * nt_max) * 8 + up256(8 * (nt_max + 1)) * 2 +          // fsm
                    up256(8 * (nt_max / kScanTile + 2)) + 8192;
  void* s2 = nullptr;
  if ((e = scratch_alloc(&s2, p2, st)) != hipSuccess) {
    (void)scratch_free(s1, st);
    return e;
  }
  Arena A{static_cast<uint8_t*>(s2), 0};
  uint64_t* it_off = A.take<uint64_t>(ni);
  uint8_t* it_old = A.take<uint8_t>(ni);
  uint64_t* crc_off = A.take<uint64_t>(ni);
  uint32_t* crc_len = A.take<uint32_t>(ni);
  uint32_t* crc_stored = A.take<uint32_t>(ni);
  uint32_t* ipack = A.take<uint32_t>(ni);
  uint32_t* computed = A.take<uint32_t>(ni);
  Tokens t{A.take<uint8_t>(nt_max), A.take<uint64_t>(nt_max), A.take<uint32_t>(nt_max),
           A.take<uint64_t>(nt_max), A.take<uint8_t>(nt_max)};
  uint64_t* ntok = A.take<uint64_t>(nb + 2);
  uint64_t* tok_base = A.take<uint64_t>(nb + 2);
  uint64_t* head = A.take<uint64_t>(nt_max);
  uint64_t* plen = A.take<uint64_t>(nt_max);
  uint64_t* pl = A.take<uint64_t>(nt_max);
  uint64_t* seg = A.take<uint64_t>(nt_max);
  uint64_t* seg_head = A.take<uint64_t>(nt_max + 1);
  unsigned long long* seg_fl = A.take<unsigned long long>(nt_max + 1);
  uint64_t* n_emit = A.take<uint64_t>(nt_max);
  uint64_t* n_rep = A.take<uint64_t>(nt_max);
  uint64_t* emit_at = A.take<uint64_t>(nt_max);
  uint64_t* rep_at = A.take<uint64_t>(nt_max);
  uint64_t* tiles2 = A.take<uint64_t>(nt_max / kScanTile + 2);
  if (nb) {
    hipLaunchKernelGGL(rw_fill_kernel, grid_for(nb), dim3(kLanes), 0, st, a, ibase, it_off, it_old,
                       crc_off, crc_len, crc_stored, ipack, ev, ev_pos);
    if (ni) {
      BlockArgs cb{};
      cb.base = log;
      cb.base_len = log_len;
      cb.offsets = crc_off;
      cb.sizes = crc_len;
      cb.out32 = computed;
      cb.n = ni;
      const char* crc_name = nullptr;
      if ((e = launch_crc32c_blocks(kModeRaw, cb, st, &crc_name)) != hipSuccess) {
        (void)scratch_free(s2, st);
        (void)scratch_free(s1, st);
        return e;
      }
    }
    hipLaunchKernelGGL(rw_block_kernel, grid_for(nb), dim3(kLanes), 0, st, a, cnt, ibase, it_off,
                       it_old, crc_off, crc_len, crc_stored, computed, ev, ev_pos, acc, rp_end,
                       first_stop, recycled);
  }
  hipLaunchKernelGGL(rw_ntok_kernel, grid_for(nb + 1), dim3(kLanes), 0, st, a, acc, ev, first_stop,
                     ntok);
  scan_u64(ntok, nb + 1, tiles, tok_base, st);
  uint64_t n_tok = 0;
  if ((e = hipMemcpyAsync(&n_tok, tiles + (nb + 1 + kScanTile - 1) / kScanTile, 8,
                          hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (e = hipStreamSynchronize(st)) != hipSuccess) {
    (void)scratch_free(s2, st);
    (void)scratch_free(s1, st);
    return e;
  }
  hipLaunchKernelGGL(rw_token_kernel, grid_for(nb + 1), dim3(kLanes), 0, st, a, ibase, it_off,
                     it_old, ipack, acc, ev, ev_pos, rp_end, tok_base, first_stop, recycled, t,
                     unsup_d);
  const dim3 tg = grid_for(n_tok);
  hipLaunchKernelGGL(rw_head_kernel, tg, dim3(kLanes), 0, st, t, n_tok, head, plen);
  scan_u64(head, n_tok, tiles2, seg, st);
  scan_u64(plen, n_tok, tiles2, pl, st);
  (void)hipMemsetAsync(seg_fl, 0xff, 8 * (n_tok + 1), st);
  hipLaunchKernelGGL(rw_seg_kernel, tg, dim3(kLanes), 0, st, t, n_tok, head, seg, seg_head, seg_fl);
  const Fsm f{seg, seg_head, seg_fl, pl, plen};
  forst_wal_records no_recs{};
  forst_wal_reports no_reps{};
  hipLaunchKernelGGL(rw_emit_kernel<false>, tg, dim3(kLanes), 0, st, t, n_tok, f, mode, n_emit,
                     n_rep, nullptr, nullptr, no_recs, 0, no_reps, 0, nullptr);
  uint64_t tot[2] = {0, 0};
  scan_u64(n_emit, n_tok, tiles2, emit_at, st);
  e = hipMemcpyAsync(&tot[0], tiles2 + (n_tok + kScanTile - 1) / kScanTile, 8,
                     hipMemcpyDeviceToHost, st);
  scan_u64(n_rep, n_tok, tiles2, rep_at, st);  // (after the copy above, stream order)
  if (e == hipSuccess)
    e = hipMemcpyAsync(&tot[1], tiles2 + (n_tok + kScanTile - 1) / kScanTile, 8,
                       hipMemcpyDeviceToHost, st);
  // stop reason / offset: the last token
  uint8_t last_kind = 0;
  uint64_t last_pos = 0;
  uint32_t unsupported = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&unsupported, unsup_d, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && n_tok)
    e = hipMemcpyAsync(&last_kind, t.kind + n_tok - 1, 1, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && n_tok)
    e = hipMemcpyAsync(&last_pos, t.pos + n_tok - 1, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    (void)scratch_free(s2, st);
    (void)scratch_free(s1, st);
    return e;
  }
  if (unsupported) {
    (void)scratch_free(s2, st);
    (void)scratch_free(s1, st);
    res->unsupported = 1;
    return hipSuccess;
  }
  const uint64_t n_rec = tot[0], n_rp = tot[1];
  res->n_records = n_rec;
  res->n_reports = n_rp;
  res->n_physical = ni;
  res->stop_reason = last_kind == kTkStopEof         ? FORST_WAL_STOP_EOF
                     : last_kind == kTkStopOld       ? FORST_WAL_STOP_OLD_RECORD
                     : last_kind == kTkStopHeader    ? FORST_WAL_STOP_TRUNCATED_HEADER
                     : last_kind == kTkStopBadLenEof ? FORST_WAL_STOP_TRUNCATED_BODY
                                                     : FORST_WAL_STOP_RECYCLED_TAIL;
  res->stop_offset = last_pos;
  res->truncated = (n_rec > rec_cap || n_rp > rep_cap) ? 1u : 0u;
  // records + reports at their positions, then the hashes
  const uint64_t nr = n_rec;
  // full record list in scratch first (the caller's capacity may be short)
  forst_wal_records full{};
  uint64_t* head_tok = nullptr;
  uint32_t* r_nf = nullptr;
  void* s4 = nullptr;
  if ((e = scratch_alloc(&s4, up256(8 * nr) * 4 + up256(4 * nr), st)) != hipSuccess) {
    (void)scratch_free(s2, st);
    (void)scratch_free(s1, st);
    return e;
  }
  {
    Arena A4{static_cast<uint8_t*>(s4), 0};
    full.offset = A4.take<uint64_t>(nr);
    full.length = A4.take<uint64_t>(nr);
    full.hash = A4.take<uint64_t>(nr);
    full.n_fragments = r_nf = A4.take<uint32_t>(nr);
    head_tok = A4.take<uint64_t>(nr);
  }
  hipLaunchKernelGGL(rw_emit_kernel<true>, tg, dim3(kLanes), 0, st, t, n_tok, f, mode, nullptr,
                     nullptr, emit_at, rep_at, full, nr, reps, rep_cap, head_tok);
  if (nr) {
    const RecFrags rf{head_tok, r_nf, t.item, it_off, ipack};
    e = hash_logical_records(log, log_len, rf, nr, full.hash, st, name);
  }
  // copy the (capacity-limited) record list out
  const uint64_t nc = nr < rec_cap ? nr : rec_cap;
  if (e == hipSuccess && nc) {
    if (recs.offset) e = hipMemcpyAsync(recs.offset, full.offset, 8 * nc, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && recs.length)
      e = hipMemcpyAsync(recs.length, full.length, 8 * nc, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && recs.hash)
      e = hipMemcpyAsync(recs.hash, full.hash, 8 * nc, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && recs.n_fragments)
      e = hipMemcpyAsync(recs.n_fragments, full.n_fragments, 4 * nc, hipMemcpyDeviceToDevice, st);
  }
  if (e == hipSuccess) e = hipGetLastError();
  *name = "wal_recover";
  const hipError_t f4 = scratch_free(s4, st), f2 = scratch_free(s2, st),
                   f1 = scratch_free(s1, st);
  if (e != hipSuccess) return e;
  for (hipError_t x : {f4, f2, f1})
    if (x != hipSuccess) return x;
  return hipSuccess;
}

}  // namespace forst
