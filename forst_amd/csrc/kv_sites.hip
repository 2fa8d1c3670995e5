// forst_amd/csrc/kv_sites.hip -- a15 at the WriteBatch call site: the
// protection info of every data record of a batch of WriteBatch reps
// (WriteBatchInternal::UpdateProtectionInfo, db/write_batch.cc:3164-3181, whose
// ProtectionInfoUpdater pushes ProtectKVO(key, value, op).ProtectC(cf) per
// record, :3016-3080), with the reps parsed on the device as
// ReadRecordFromWriteBatch / WriteBatchInternal::Iterate parse them
// (write_batch.cc:361-716).
//
//   1. wb_count_kernel: each rep's header count (rep bytes 8..11, or 0 for a
//      rep under the 12-byte header) -> one exclusive scan = every rep's first
//      protection slot; the total is read back (the one synchronisation);
//   2. wb_walk_kernel: one LANE per rep walks its records (tag, [cf varint],
//      length-prefixed key / value / xid / blob slices; 16-byte windows per
//      varint) and writes the data records' key / value / op / cf descriptors
//      into its slots -- only record headers are read;
//   3. kv_kernel<protect> (kv_protect.hip) over the descriptors: the record
//      bytes are read once, a 16-lane row per record.
// A rep's slots are its header count; records past it are parsed but get no
// slot (the rep then fails with "WriteBatch has wrong count" anyway).
#include "device_common.h"
#include "engine.h"
#include "scan_common.h"

namespace forst {
namespace {

constexpr uint32_t kWbThreads = 256;

__device__ __forceinline__ uint32_t wb_byte(const uint8_t* base, uint64_t p) {
  return ldu8(base + p);
}

// GetVarint32(&input, &v) with input = [p, end) (util/coding.h:109 +
// GetVarint32PtrFallback): the bytes consumed, 0 when it fails
__device__ __forceinline__ uint32_t wb_varint(const uint8_t* base, uint64_t p, uint64_t end,
                                              uint32_t& v) {
  uint32_t r = 0;
  for (uint32_t j = 0; j < 5; ++j) {
    if (p + j >= end) return 0;
    const uint32_t b = wb_byte(base, p + j);
    r |= (b & 127u) << (7 * j);
    if (!(b & 128u)) {
      v = r;
      return j + 1;
    }
  }
  return 0;
}

// GetLengthPrefixedSlice(&input, &slice) (util/coding.h): false when it fails;
// on success [off, off + len) is the slice and p moves past it
__device__ __forceinline__ bool wb_slice(const uint8_t* base, uint64_t& p, uint64_t end,
                                         uint64_t& off, uint32_t& len) {
  const uint32_t n = wb_varint(base, p, end, len);
  if (!n || end - (p + n) < len) return false;
  off = p + n;
  p = off + len;
  return true;
}

__global__ void __launch_bounds__(kWbThreads) wb_count_kernel(WbArgs a, uint64_t* cnt) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kWbThreads + threadIdx.x;
  if (b > a.n) return;
  uint64_t c = 0;
  if (b < a.n) {
    const uint64_t o = a.offsets[b], s = a.sizes[b];
    if (s >= 12 && o <= a.base_len && s <= a.base_len - o)  // WriteBatchInternal::Count
      c = ldu32(a.base + o + 8);
  }
  cnt[b] = c;
}

// ReadRecordFromWriteBatch tag handling (write_batch.cc:361-475) -> what the
// record holds, its error status, and ProtectionInfoUpdater's op type for the
// data records (write_batch.cc:3023-3052; 0xff = not a data record)
struct TagInfo {
  uint8_t cf, key, value, xid;  // parts, in this order (key+xid: commit ts)
  uint8_t err, op;
};
__device__ __forceinline__ TagInfo tag_info(uint32_t t) {
  switch (t) {
    case 0x05: return {1, 1, 1, 0, kWbBadPut, 0x01};
    case 0x01: return {0, 1, 1, 0, kWbBadPut, 0x01};
    case 0x04: return {1, 1, 0, 0, kWbBadDelete, 0x00};
    case 0x08: return {1, 1, 0, 0, kWbBadDelete, 0x07};
    case 0x00: return {0, 1, 0, 0, kWbBadDelete, 0x00};
    case 0x07: return {0, 1, 0, 0, kWbBadDelete, 0x07};
    case 0x0E: return {1, 1, 1, 0, kWbBadDeleteRange, 0x0F};
    case 0x0F: return {0, 1, 1, 0, kWbBadDeleteRange, 0x0F};
    case 0x06: return {1, 1, 1, 0, kWbBadMerge, 0x02};
    case 0x02: return {0, 1, 1, 0, kWbBadMerge, 0x02};
    case 0x10: return {1, 1, 1, 0, kWbBadBlobIndex, 0x11};
    case 0x11: return {0, 1, 1, 0, kWbBadBlobIndex, 0x11};
    case 0x17: return {1, 1, 1, 0, kWbBadPutEntity, 0x16};
    case 0x16: return {0, 1, 1, 0, kWbBadPutEntity, 0x16};
    case 0x03: return {0, 0, 0, 1, kWbBadBlob, 0xff};       // LogData blob
    case 0x0D: case 0x09: case 0x12: case 0x13:
      return {0, 0, 0, 0, kWbOk, 0xff};                      // Noop / BeginPrepare*
    case 0x0A: return {0, 0, 0, 1, kWbBadEndPrepareXid, 0xff};
    case 0x0B: return {0, 0, 0, 1, kWbBadCommitXid, 0xff};
    case 0x15: return {0, 1, 0, 1, kWbBadCommitTs, 0xff};    // ts, then the xid
    case 0x0C: return {0, 0, 0, 1, kWbBadRollbackXid, 0xff};
    default: return {0, 0, 0, 0, kWbUnknownTag, 0xff};
  }
}

__global__ void __launch_bounds__(kWbThreads) wb_walk_kernel(WbArgs a, const uint64_t* first,
                                                             uint64_t* ko, uint32_t* kl,
                                                             uint64_t* vo, uint32_t* vl,
                                                             uint8_t* ops, uint32_t* cfs) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kWbThreads + threadIdx.x;
  if (b >= a.n) return;
  const uint64_t o = a.offsets[b], s = a.sizes[b];
  const uint64_t e0 = first[b], slots = first[b + 1] - e0;
  uint32_t st = kWbOk;
  uint64_t found = 0;
  if (o > a.base_len || s > a.base_len - o) {
    st = kWbOutOfRange;
  } else if (s < 12) {
    st = kWbTooSmall;  // WriteBatch::Iterate (write_batch.cc:478-480)
  } else {
    uint64_t p = o + 12;
    const uint64_t end = o + s;
    while (p < end) {
      const TagInfo ti = tag_info(wb_byte(a.base, p));
      ++p;
      if (ti.err == kWbUnknownTag) {
        st = kWbUnknownTag;
        break;
      }
      uint32_t cf = 0, klen = 0, vlen = 0, xl = 0;
      uint64_t koff = 0, voff = 0, xo = 0;
      bool ok = true;
      if (ti.cf) {
        const uint32_t n = wb_varint(a.base, p, end, cf);
        ok = n != 0;
        p += n;
      }
      if (ok && ti.key) ok = wb_slice(a.base, p, end, koff, klen);
      if (ok && ti.value) ok = wb_slice(a.base, p, end, voff, vlen);
      if (!ok) {
        st = ti.err;
        break;
      }
      if (ti.xid && !wb_slice(a.base, p, end, xo, xl)) {
        // kTypeCommitXIDAndTimestamp: the ts parsed, the xid did not
        st = ti.key ? static_cast<uint32_t>(kWbBadCommitXid) : ti.err;
        break;
      }
      if (ti.op != 0xff) {
        if (found < slots) {
          const uint64_t j = e0 + found;
          ko[j] = koff;
          kl[j] = klen;
          vo[j] = ti.value ? voff : koff;  // Delete / SingleDelete: value "" (empty)
          vl[j] = ti.value ? vlen : 0;
          ops[j] = ti.op;
          cfs[j] = cf;
        }
        ++found;
      }
    }
    if (st == kWbOk && found != slots) st = kWbWrongCount;  // write_batch.cc:709-712
  }
  for (uint64_t k = found; k < slots; ++k) {  // slots no record filled: protection 0
    ko[e0 + k] = ~0ull;
    kl[e0 + k] = 0;
    vo[e0 + k] = ~0ull;
    vl[e0 + k] = 0;
    ops[e0 + k] = 0;
    cfs[e0 + k] = 0;
  }
  if (a.status) a.status[b] = static_cast<uint8_t>(st);
  if (a.n_protected) a.n_protected[b] = static_cast<uint32_t>(found < slots ? found : slots);
}

// ---- Block protection (table/block_based/block.cc:1113-1235) ---------------
// GetVarint64 over [p, end) (util/coding.h GetVarint64Ptr): bytes consumed, 0 on failure
__device__ __forceinline__ uint32_t blk_varint64(const uint8_t* base, uint64_t p, uint64_t end,
                                                 uint64_t& v) {
  uint64_t r = 0;
  for (uint32_t j = 0; j < 10; ++j) {
    if (p + j >= end) return 0;
    const uint64_t b = wb_byte(base, p + j);
    r |= (b & 127u) << (7 * j);
    if (!(b & 128u)) {
      v = r;
      return j + 1;
    }
  }
  return 0;
}

// The restart-array geometry of Block::Block (block.cc:1058-1111, NumRestarts
// :1016, IndexType :1038, DataBlockHashIndex::Initialize): false = the
// reference's size_ = 0 error marker (a block under 8 bytes with restarts
// wraps the offset here, as the iterators' "bad block contents")
__device__ __forceinline__ bool blk_geometry(const uint8_t* base, uint64_t o, uint32_t s,
                                             uint32_t& nr, uint32_t& ro) {
  if (s < 4) return false;
  const uint32_t footer = ldu32(base + o + s - 4);
  nr = footer;
  bool hash = false;
  if (s <= 65536) {  // kMaxBlockSizeSupportedByHashIndex
    hash = (footer >> 31) != 0;
    nr = footer & 0x7fffffffu;  // kNumRestartsMask
  }
  if (!hash) {
    ro = static_cast<uint32_t>(static_cast<uint64_t>(s) - (1 + static_cast<uint64_t>(nr)) * 4);
    return ro <= s - 4;
  }
  if (s < 6) return false;
  const uint32_t nb = ldu8(base + o + s - 6) | (ldu8(base + o + s - 5) << 8);
  const uint32_t map = static_cast<uint16_t>(s - 4 - 2 - nb);
  ro = static_cast<uint32_t>(static_cast<uint64_t>(map) - static_cast<uint64_t>(nr) * 4);
  return ro <= map;
}

// One walk over a block's entries [0, restart offset) as the block iterators
// parse them (BlockIter::ParseNextKey block.cc:637-686 with DecodeEntry /
// CheckAndDecodeEntry / DecodeEntryV4 :37-153, IndexBlockIter::
// DecodeCurrentValue :739-770 -> IndexValue::DecodeFrom format.cc:124-148):
// counts keys and the bytes of their materialised (4-byte padded) full keys,
// and with EMIT writes every key into mat (raw_key_: the previous key's first
// `shared` bytes + the delta, block.cc TrimAppend) and its descriptor.
// Returns a BlkStatus.
template <bool EMIT>
__device__ uint32_t blk_walk(const uint8_t* base, uint64_t o, uint32_t s, uint32_t kind,
                             uint64_t& nkeys, uint64_t& nmat, uint8_t* mat, uint64_t mat0,
                             uint64_t* ko, uint32_t* kl, uint64_t* vo, uint32_t* vl) {
  nkeys = nmat = 0;
  uint32_t nr = 0, ro = 0;
  if (!blk_geometry(base, o, s, nr, ro)) return kBlkBadContents;
  if (nr == 0) return kBlkOk;  // no restarts: no protection (block.cc:1116)
  const uint32_t k = kind & 3;
  const bool delta_v4 = k == kBlkIndex && !(kind & kBlkValueIsFull);
  const bool first_key = k == kBlkIndex && (kind & kBlkHasFirstKey);
  // (limit checks as the release build makes them: CheckAndDecodeEntry (meta)
  // and DecodeKeyV4 (delta index) check `limit - p < 3` and the meta slices;
  // DecodeEntry (data, full-value index) only asserts -- its slices may run
  // into the restart array.  Anything past the block's own bytes, which the
  // reference would read out of bounds, is reported as a bad entry.)
  const uint64_t end = o + ro, bend = o + s;
  const bool checked = k == kBlkMeta;
  uint64_t p = o;
  uint64_t prev = 0;  // previous key: mat offset (EMIT) and length
  uint32_t prev_len = 0;
  while (p < end) {
    uint32_t shared, non_shared, vlen = 0;
    if ((checked || delta_v4 ? end : bend) - p < 3) return kBlkBadEntry;
    shared = wb_byte(base, p);
    non_shared = wb_byte(base, p + 1);
    if (!delta_v4) vlen = wb_byte(base, p + 2);
    if ((shared | non_shared | vlen) < 128) {  // fast path: one byte each
      p += delta_v4 ? 2 : 3;
    } else {
      uint32_t n = wb_varint(base, p, end, shared);
      if (!n) return kBlkBadEntry;
      p += n;
      n = wb_varint(base, p, end, non_shared);
      if (!n) return kBlkBadEntry;
      p += n;
      if (!delta_v4) {
        n = wb_varint(base, p, end, vlen);
        if (!n) return kBlkBadEntry;
        p += n;
      }
    }
    if ((checked ? end : bend) - p < static_cast<uint64_t>(non_shared) + vlen) return kBlkBadEntry;
    if (prev_len < shared) return kBlkBadEntry;  // raw_key_.Size() < shared
    const uint64_t kd = p;
    const uint64_t v0 = p + non_shared;
    if (delta_v4 && v0 > end) return kBlkBadEntry;
    if (delta_v4) {  // IndexValue::DecodeFrom: the bytes it consumes are the raw value
      uint64_t q = v0, x;
      uint32_t n = blk_varint64(base, q, end, x);
      if (!n) return kBlkBadEntry;
      q += n;
      if (shared == 0) {  // full handle: offset, size
        n = blk_varint64(base, q, end, x);
        if (!n) return kBlkBadEntry;
        q += n;
      }
      if (first_key) {
        uint32_t fl;
        n = wb_varint(base, q, end, fl);
        if (!n || end - (q + n) < fl) return kBlkBadEntry;
        q += n + fl;
      }
      vlen = static_cast<uint32_t>(q - v0);
    }
    const uint32_t klen = shared + non_shared;
    if (EMIT) {
      uint8_t* dst = mat + mat0 + nmat;
      // shared prefix from the previous materialised key (4-byte aligned both)
      const uint32_t* ps = reinterpret_cast<const uint32_t*>(mat + prev);
      uint32_t* pd = reinterpret_cast<uint32_t*>(dst);
      for (uint32_t j = 0; j < (shared >> 2); ++j) pd[j] = ps[j];
      for (uint32_t j = shared & ~3u; j < shared; ++j) dst[j] = mat[prev + j];
      for (uint32_t j = 0; j < non_shared; ++j) dst[shared + j] = static_cast<uint8_t>(wb_byte(base, kd + j));
      ko[nkeys] = mat0 + nmat;
      kl[nkeys] = klen;
      vo[nkeys] = v0;
      vl[nkeys] = vlen;
      prev = mat0 + nmat;
    }
    prev_len = klen;
    nmat += (klen + 3) & ~3u;
    ++nkeys;
    p = v0 + vlen;
  }
  return kBlkOk;
}

__global__ void __launch_bounds__(kWbThreads) blk_count_kernel(BlkArgs a, uint64_t* cnt,
                                                               uint64_t* mat) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kWbThreads + threadIdx.x;
  if (b > a.n) return;
  uint64_t nk = 0, nm = 0;
  if (b < a.n) {
    const uint64_t o = a.offsets[b];
    const uint32_t s = a.sizes[b];
    uint32_t st = kBlkOutOfRange;
    if (o <= a.base_len && s <= a.base_len - o)
      st = blk_walk<false>(a.base, o, s, a.kinds[b], nk, nm, nullptr, 0, nullptr, nullptr,
                           nullptr, nullptr);
    if (st != kBlkOk) nk = nm = 0;  // the error marker: no kv_checksum_
    if (a.status) a.status[b] = static_cast<uint8_t>(st);
  }
  cnt[b] = nk;
  mat[b] = nm;
}

__global__ void __launch_bounds__(kWbThreads) blk_walk_kernel(BlkArgs a, const uint64_t* mat_pos,
                                                              uint8_t* mat, uint64_t* ko,
                                                              uint32_t* kl, uint64_t* vo,
                                                              uint32_t* vl) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kWbThreads + threadIdx.x;
  if (b >= a.n) return;
  const uint64_t e0 = a.first_key[b];
  if (a.first_key[b + 1] == e0) return;
  uint64_t nk, nm;
  (void)blk_walk<true>(a.base, a.offsets[b], a.sizes[b], a.kinds[b], nk, nm, mat, mat_pos[b],
                       ko + e0, kl + e0, vo + e0, vl + e0);
}

}  // namespace

hipError_t launch_block_kv_checksum(const BlkArgs& a, hipStream_t st, uint64_t* total,
                                    const char** name) {
  *total = 0;
  *name = "blk_walk_kernel";
  const uint64_t n1 = a.n + 1;
  const uint64_t nt = n1 / kScanTile + 2;
  void* s0 = nullptr;
  hipError_t e = scratch_alloc(&s0, 8 * (3 * n1 + nt) + 16, st);
  if (e != hipSuccess) return e;
  uint64_t* cnt = static_cast<uint64_t*>(s0);
  uint64_t* matn = cnt + n1;
  uint64_t* matp = matn + n1;
  uint64_t* tiles = matp + n1;
  const uint32_t g1 = static_cast<uint32_t>((n1 + kWbThreads - 1) / kWbThreads);
  hipLaunchKernelGGL(blk_count_kernel, dim3(g1), dim3(kWbThreads), 0, st, a, cnt, matn);
  scan_u64(cnt, n1, tiles, a.first_key, st);
  scan_u64(matn, n1, tiles, matp, st);
  uint64_t tot[2] = {0, 0};
  e = hipMemcpyAsync(&tot[0], a.first_key + a.n, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(&tot[1], matp + a.n, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  *total = tot[0];
  if (e != hipSuccess || tot[0] == 0 || tot[0] > a.capacity) {
    (void)scratch_free(s0, st);
    return e != hipSuccess ? e : tot[0] > a.capacity ? hipErrorInvalidValue : hipSuccess;
  }
  const uint64_t m = tot[0];
  void* s1 = nullptr;
  e = scratch_alloc(&s1, tot[1] + 24 * m + 256, st);
  if (e != hipSuccess) {
    (void)scratch_free(s0, st);
    return e;
  }
  uint64_t* ko = static_cast<uint64_t*>(s1);
  uint64_t* vo = ko + m;
  uint32_t* kl = reinterpret_cast<uint32_t*>(vo + m);
  uint32_t* vl = kl + m;
  uint8_t* mat = reinterpret_cast<uint8_t*>(vl + m);
  const uint32_t g = static_cast<uint32_t>((a.n + kWbThreads - 1) / kWbThreads);
  hipLaunchKernelGGL(blk_walk_kernel, dim3(g), dim3(kWbThreads), 0, st, a, matp, mat, ko, kl, vo,
                     vl);
  e = hipGetLastError();
  if (e == hipSuccess) {
    KvArgs k{};
    k.base = a.base;
    k.base_len = a.base_len;
    k.key_base = mat;
    k.key_base_len = tot[1];
    k.key_off = ko;
    k.key_len = kl;
    k.val_off = vo;
    k.val_len = vl;
    k.out = a.prot;
    k.enc_out = a.kv_checksums;
    k.prot_bytes = a.prot_bytes;
    k.n = m;
    e = launch_kv(kKvProtect, k, st, name);
  }
  const hipError_t f0 = scratch_free(s1, st), f1 = scratch_free(s0, st);
  if (e == hipSuccess) e = f0 != hipSuccess ? f0 : f1;
  return e;
}

hipError_t launch_write_batch_protect(const WbArgs& a, hipStream_t st, uint64_t* total,
                                      const char** name) {
  *total = 0;
  const uint64_t n1 = a.n + 1;
  const uint64_t nt = n1 / kScanTile + 2;
  void* s0 = nullptr;
  hipError_t e = scratch_alloc(&s0, 8 * (n1 + nt), st);
  if (e != hipSuccess) return e;
  uint64_t* cnt = static_cast<uint64_t*>(s0);
  uint64_t* tiles = cnt + n1;
  const uint32_t g1 = static_cast<uint32_t>((n1 + kWbThreads - 1) / kWbThreads);
  hipLaunchKernelGGL(wb_count_kernel, dim3(g1), dim3(kWbThreads), 0, st, a, cnt);
  scan_u64(cnt, n1, tiles, a.first_entry, st);
  e = hipMemcpyAsync(total, a.first_entry + a.n, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)scratch_free(s0, st);
  if (e != hipSuccess) return e;
  const uint64_t m = *total;
  if (m > a.capacity) return hipErrorInvalidValue;  // (the caller reports the needed size)
  void* s1 = nullptr;
  if (m) {
    e = scratch_alloc(&s1, (8 + 4 + 8 + 4 + 4 + 1) * m + 64, st);
    if (e != hipSuccess) return e;
  }
  uint8_t* q = static_cast<uint8_t*>(s1);
  uint64_t* ko = reinterpret_cast<uint64_t*>(q);
  uint64_t* vo = ko + m;
  uint32_t* kl = reinterpret_cast<uint32_t*>(vo + m);
  uint32_t* vl = kl + m;
  uint32_t* cfs = vl + m;
  uint8_t* ops = reinterpret_cast<uint8_t*>(cfs + m);
  const uint32_t g = static_cast<uint32_t>((a.n + kWbThreads - 1) / kWbThreads);
  hipLaunchKernelGGL(wb_walk_kernel, dim3(g), dim3(kWbThreads), 0, st, a, a.first_entry, ko, kl,
                     vo, vl, ops, cfs);
  e = hipGetLastError();
  if (e == hipSuccess && m) {
    KvArgs k{};
    k.base = a.base;
    k.base_len = a.base_len;
    k.key_off = ko;
    k.key_len = kl;
    k.val_off = vo;
    k.val_len = vl;
    k.ops = ops;
    k.cfs = cfs;
    k.out = a.prot;
    k.n = m;
    e = launch_kv(kKvProtect, k, st, name);
  } else {
    *name = "wb_walk_kernel";
  }
  if (s1) {
    const hipError_t f = scratch_free(s1, st);
    if (e == hipSuccess) e = f;
  }
  return e;
}

}  // namespace forst
