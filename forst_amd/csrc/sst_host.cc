// forst_amd/csrc/sst_host.cc -- whole-SST-file checksum verification
// (BlockBasedTable::VerifyChecksum, table/block_based/block_based_table_reader.cc:2457).
//
// The file structure is decoded on the host -- it is a handful of small,
// serially dependent blocks (footer -> metaindex -> properties / index ->
// index partitions) -- and every block checksum is verified on the GPU:
// the footer checksum (fv >= 6) and each structural block before it is
// trusted, then ALL meta blocks and data blocks of the file in one batch
// launch.  Decoders follow the reference block format:
//   footer           table/format.cc:170-463 (Footer::DecodeFrom)
//   block entries    table/block_based/block_builder.cc:187-237 (writer),
//                    block.cc:37-153 (DecodeEntry / DecodeKeyV4),
//                    data_block_footer.cc:41-57 (num_restarts packing)
//   index values     table/format.cc:105-148 (IndexValue), value delta
//                    encoding only for entries with shared key bytes
//   metaindex        table/meta_blocks.cc:38-54 (name -> BlockHandle)
//   properties       table/meta_blocks.cc:56-140, block_based_table_reader.cc:
//                    948-972 (index type, value delta flag, first-key flag)
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/forst/checksum_engine.h"
#include "../../include/forst_checksum.h"

namespace forst {
int uncompress_block(uint8_t type, uint32_t format_version, const uint8_t* in, size_t n,
                     std::vector<uint8_t>* out, std::string* err);  // block_codecs.cc
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t stream);  // capi.hip
hipError_t scratch_free(void* p, hipStream_t stream);
}  // namespace forst

namespace {

constexpr uint64_t kBlockBasedTableMagicNumber = 0x88e241b785f4cff7ull;        // builder.cc:201
constexpr uint64_t kLegacyBlockBasedTableMagicNumber = 0xdb4775248b80fb57ull;  // builder.cc:204
constexpr uint32_t kMaxVarint64Length = 10;
constexpr uint32_t kHandleMax = 2 * kMaxVarint64Length;                        // format.h:69
constexpr uint32_t kVersion0Len = 2 * kHandleMax + 8;                          // format.h:226
constexpr uint32_t kNewVersionsLen = 1 + 2 * kHandleMax + 4 + 8;               // format.h:234
constexpr uint32_t kLatestFormatVersion = 6;
constexpr uint32_t kBlockTrailer = 5;
constexpr uint64_t kMaxBlockSizeSupportedByHashIndex = 1u << 16;  // data_block_hash_index.h

thread_local std::string g_sst_err;

int corrupt(const std::string& m) {
  g_sst_err = m;
  return FORST_ECORRUPT;
}
int unsupported(const std::string& m) {
  g_sst_err = m;
  return FORST_EUNSUPPORTED;
}
// ReadFooterFromFile's own message ends in ": <file>" rather than the " in
// <file>" that CopyAppendMessage adds to DecodeFrom's errors (format.cc:491-495)
constexpr int kTooShort = -100;
int too_short(const std::string& m) {
  g_sst_err = m;
  return kTooShort;
}

uint32_t fixed32(const uint8_t* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
uint64_t fixed64(const uint8_t* p) { return uint64_t(fixed32(p)) | (uint64_t(fixed32(p + 4)) << 32); }

bool varint64(const uint8_t*& p, const uint8_t* lim, uint64_t* v) {  // util/coding.cc
  uint64_t r = 0;
  for (uint32_t shift = 0; shift <= 63 && p < lim; shift += 7) {
    const uint64_t b = *p++;
    r |= (b & 127) << shift;
    if (!(b & 128)) {
      *v = r;
      return true;
    }
  }
  return false;
}
bool varint32(const uint8_t*& p, const uint8_t* lim, uint32_t* v) {
  uint32_t r = 0;
  for (uint32_t shift = 0; shift <= 28 && p < lim; shift += 7) {
    const uint32_t b = *p++;
    r |= (b & 127) << shift;
    if (!(b & 128)) {
      *v = r;
      return true;
    }
  }
  return false;
}

struct Handle {
  uint64_t off = 0, size = 0;
};

bool decode_handle(const uint8_t*& p, const uint8_t* lim, Handle* h) {  // format.cc BlockHandle
  return varint64(p, lim, &h->off) && varint64(p, lim, &h->size);
}

std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789ABCDEF";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}

constexpr uint64_t kBad = ~0ull;

// Walks the entries of one block (block.cc ParseNextKey).  For value-delta
// encoded index blocks the value length is not stored: `fn` decodes the
// value and returns the bytes it consumed (kBad = corrupt).
template <typename F>
int for_each_entry(const uint8_t* blk, uint64_t size, bool value_delta, F&& fn) {
  if (size < 4) return corrupt("bad block contents");
  uint32_t nr = fixed32(blk + size - 4);
  if (size <= kMaxBlockSizeSupportedByHashIndex) nr &= 0x7fffffffu;  // block.cc:1020-1035
  if ((uint64_t(nr) + 1) * 4 > size) return corrupt("bad block contents");
  const uint8_t* p = blk;
  const uint8_t* lim = blk + size - (uint64_t(nr) + 1) * 4;
  std::string key;
  while (p < lim) {
    uint32_t shared = 0, non_shared = 0, vlen = 0;
    if (!varint32(p, lim, &shared) || !varint32(p, lim, &non_shared) ||
        (!value_delta && !varint32(p, lim, &vlen)))
      return corrupt("bad entry in block");
    if (shared > key.size() || uint64_t(lim - p) < uint64_t(non_shared) + vlen)
      return corrupt("bad entry in block");
    key.resize(shared);
    key.append(reinterpret_cast<const char*>(p), non_shared);
    p += non_shared;
    const uint8_t* vlim = value_delta ? lim : p + vlen;
    const uint64_t used = fn(key, shared != 0, p, vlim);  // kBad = corrupt value
    if (used == kBad || (value_delta && (used == 0 || used > uint64_t(vlim - p))))
      return corrupt("bad entry in block");
    p += value_delta ? used : vlen;
  }
  return FORST_OK;
}

// index block -> block handles (IndexValue, format.cc:123-148)
int index_handles(const uint8_t* blk, uint64_t size, bool value_delta, bool first_key,
                  std::vector<Handle>* out) {
  Handle prev;
  bool have_prev = false;
  return for_each_entry(blk, size, value_delta,
                        [&](const std::string&, bool shared, const uint8_t* v,
                            const uint8_t* vlim) -> uint64_t {
                          const uint8_t* q = v;
                          Handle h;
                          if (value_delta && shared) {
                            uint64_t z;
                            if (!have_prev || !varint64(q, vlim, &z)) return kBad;
                            const int64_t delta = int64_t(z >> 1) ^ -int64_t(z & 1);  // zigzag
                            h.off = prev.off + prev.size + kBlockTrailer;
                            h.size = prev.size + uint64_t(delta);
                          } else if (!decode_handle(q, vlim, &h)) {
                            return kBad;
                          }
                          if (first_key) {
                            uint32_t kl;
                            if (!varint32(q, vlim, &kl) || uint64_t(vlim - q) < kl) return kBad;
                            q += kl;
                          }
                          out->push_back(h);
                          prev = h;
                          have_prev = true;
                          return static_cast<uint64_t>(q - v);
                        });
}

struct MetaEntry {
  std::string name;
  Handle h;
};

int metaindex_entries(const uint8_t* blk, uint64_t size, std::vector<MetaEntry>* out) {
  return for_each_entry(blk, size, false,
                        [&](const std::string& k, bool, const uint8_t* v,
                            const uint8_t* vlim) -> uint64_t {
                          const uint8_t* q = v;
                          MetaEntry e;
                          e.name = k;
                          if (!decode_handle(q, vlim, &e.h)) return kBad;
                          out->push_back(e);
                          return static_cast<uint64_t>(vlim - v);  // value length is stored
                        });
}

int properties(const uint8_t* blk, uint64_t size, forst_sst_properties* pr) {
  std::memset(pr, 0, sizeof(*pr));
  return for_each_entry(
      blk, size, false,
      [&](const std::string& k, bool, const uint8_t* v, const uint8_t* vlim) -> uint64_t {
        const uint8_t* q = v;
        uint64_t x = 0;
        if (k == "rocksdb.block.based.table.index.type") {  // block_based_table_builder.cc:237
          if (vlim - v >= 4) pr->index_type = fixed32(v);
        } else if (k == "rocksdb.index.value.is.delta.encoded") {  // table_properties.cc:264
          if (varint64(q, vlim, &x)) pr->index_value_is_delta_encoded = x;
        } else if (k == "rocksdb.index.key.is.user.key") {
          if (varint64(q, vlim, &x)) pr->index_key_is_user_key = x;
        } else if (k == "rocksdb.num.data.blocks") {
          if (varint64(q, vlim, &x)) pr->num_data_blocks = x;
        } else if (k == "rocksdb.index.partitions") {
          if (varint64(q, vlim, &x)) pr->index_partitions = x;
        } else if (k == "rocksdb.format.version") {
          if (varint64(q, vlim, &x)) pr->format_version = x;
        } else if (k == "rocksdb.data.size") {
          if (varint64(q, vlim, &x)) pr->data_size = x;
        } else if (k == "rocksdb.external_sst_file.global_seqno") {  // sst_file_writer_collectors.h
          pr->global_seqno_value_offset = static_cast<uint64_t>(v - blk);
        }
        return static_cast<uint64_t>(vlim - v);
      });
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) const char* forst_sst_last_error(void) {
  return g_sst_err.c_str();
}

static int footer_decode(const uint8_t* tail, uint64_t tail_len, uint64_t file_size,
                         forst_sst_footer* f);

// Footer::DecodeFrom (format.cc:355-463) on the last <= 53 bytes of a file.
__attribute__((visibility("default"))) int forst_sst_footer_decode(const uint8_t* tail,
                                                                  uint64_t tail_len,
                                                                  uint64_t file_size,
                                                                  forst_sst_footer* f) {
  const int rc = footer_decode(tail, tail_len, file_size, f);
  return rc == kTooShort ? FORST_ECORRUPT : rc;
}

static int footer_decode(const uint8_t* tail, uint64_t tail_len, uint64_t file_size,
                         forst_sst_footer* f) {
  if (!tail || !f) return FORST_EINVAL;
  std::memset(f, 0, sizeof(*f));
  if (file_size < kVersion0Len || tail_len < kVersion0Len)  // format.cc:490-496 (+ ": <file>")
    return too_short("file is too short (" + std::to_string(file_size) +
                     " bytes) to be an sstable: ");
  if (tail_len > file_size) return FORST_EINVAL;
  const uint64_t input_offset = file_size - tail_len;
  const uint8_t* magic_ptr = tail + tail_len - 8;
  uint64_t magic = fixed64(magic_ptr);
  const bool legacy = magic == kLegacyBlockBasedTableMagicNumber;
  if (legacy) magic = kBlockBasedTableMagicNumber;
  if (magic != kBlockBasedTableMagicNumber)
    return unsupported("not a block-based table (magic " + std::to_string(magic) +
                       "): no block checksums to verify");
  f->table_magic_number = magic;
  f->block_trailer_size = kBlockTrailer;
  const uint8_t* in;
  uint64_t in_len;
  if (legacy) {
    in = tail + tail_len - kVersion0Len;
    in_len = kVersion0Len;
    f->format_version = 0;
    f->checksum_type = 1;  // kCRC32c
    f->footer_offset = file_size - kVersion0Len;
    f->footer_len = kVersion0Len;
  } else {
    f->format_version = fixed32(magic_ptr - 4);
    if (f->format_version > kLatestFormatVersion)
      return corrupt("Corrupt or unsupported format_version: " +
                     std::to_string(f->format_version));
    if (tail_len < kNewVersionsLen) return corrupt("Input is too short to be an SST file");
    in = tail + tail_len - kNewVersionsLen;
    in_len = kNewVersionsLen;
    f->footer_offset = input_offset + (tail_len - kNewVersionsLen);
    f->footer_len = kNewVersionsLen;
    const uint8_t t = in[0];
    if (t > 4)  // options_helper.h:34-39
      return corrupt("Corrupt or unsupported checksum type: " + std::to_string(t));
    f->checksum_type = t;
    std::memcpy(f->footer_zeroed, in, kNewVersionsLen);
    std::memset(f->footer_zeroed + 5, 0, 4);  // format.cc:405
    ++in;
    --in_len;
  }
  (void)in_len;
  if (f->format_version >= 6) {
    static const uint8_t kExtMagic[4] = {0x3e, 0x00, 0x7a, 0x00};
    if (std::memcmp(in, kExtMagic, 4) != 0)
      return corrupt("Bad extended magic number: 0x" + hex(in, 4));
    f->stored_footer_checksum = fixed32(in + 4);
    f->base_context_checksum = fixed32(in + 8);
    if (forst_gpu::ChecksumModifierForContext(f->base_context_checksum, 0) == 0)
      return corrupt("Invalid base context checksum");
    const uint32_t metaindex_size = fixed32(in + 12);
    const uint64_t metaindex_end = f->footer_offset - kBlockTrailer;
    f->metaindex_offset = metaindex_end - metaindex_size;
    f->metaindex_size = metaindex_size;
    f->index_offset = f->index_size = 0;  // in the metaindex ("rocksdb.index")
    // format.cc:440-448: checked after the footer checksum (by the caller)
    f->future_feature = fixed64(in + 32) != 0 ? 1u : 0u;
    f->footer_checksum_modifier =
        forst_gpu::ChecksumModifierForContext(f->base_context_checksum, f->footer_offset);
  } else {
    const uint8_t* p = in;
    const uint8_t* lim = in + 2 * kHandleMax;
    Handle mi, ix;
    if (!decode_handle(p, lim, &mi) || !decode_handle(p, lim, &ix))
      return corrupt("bad block handle");
    f->metaindex_offset = mi.off;
    f->metaindex_size = mi.size;
    f->index_offset = ix.off;
    f->index_size = ix.size;
  }
  return FORST_OK;
}

__attribute__((visibility("default"))) int forst_sst_index_handles(
    const uint8_t* block, uint64_t block_size, int value_delta_encoded, int has_first_key,
    uint64_t* offsets, uint64_t* sizes, uint64_t capacity, uint64_t* n) {
  if (!block || !n) return FORST_EINVAL;
  std::vector<Handle> hs;
  const int rc = index_handles(block, block_size, value_delta_encoded != 0, has_first_key != 0, &hs);
  if (rc) return rc;
  *n = hs.size();
  for (uint64_t i = 0; i < hs.size() && i < capacity; ++i) {
    if (offsets) offsets[i] = hs[i].off;
    if (sizes) sizes[i] = hs[i].size;
  }
  return hs.size() > capacity && (offsets || sizes) ? FORST_EINVAL : FORST_OK;
}

__attribute__((visibility("default"))) int forst_sst_properties_decode(const uint8_t* block,
                                                                      uint64_t block_size,
                                                                      forst_sst_properties* out) {
  if (!block || !out) return FORST_EINVAL;
  return properties(block, block_size, out);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// BlockBasedTable::VerifyChecksum over a file staged in device memory
// ---------------------------------------------------------------------------
namespace forst_gpu {
namespace {

// Footer errors carry Status::CopyAppendMessage(s, " in ", file) of
// ReadFooterFromFile (format.cc:548-551); errors of the block iterators that
// parse the metaindex, properties and index blocks do not (block.h:559
// CorruptionError, "bad entry in block"; block.cc:1242 "bad block contents")
Status from_sst_rc(int rc, const std::string& file, bool in_file = true) {
  const std::string sfx = in_file ? " in " + file : std::string();
  if (rc == kTooShort) return Status::Corruption(g_sst_err + file);
  if (rc == FORST_ECORRUPT) return Status::Corruption(g_sst_err + sfx);
  if (rc == FORST_EUNSUPPORTED) return Status::NotSupported(g_sst_err + sfx);
  return Status::InvalidArgument("forst_sst: " + std::to_string(rc));
}

Status hip_status(hipError_t e, const char* what) {
  return e == hipSuccess ? Status::OK()
                         : Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// The whole VerifyChecksum walk of one file.  With `bulk` null the final
// batch (every meta block, then every data block) is verified here; with
// `bulk` set its handles are returned instead, already past every structural
// check, so a multi-file caller can verify the blocks of many files in one
// launch (VerifySstFilesChecksums below).
static Status WalkSstFile(BlockChecksumEngine& eng, const uint8_t* host_file, uint64_t file_size,
                          const uint8_t* dev_file, const std::string& file_name,
                          SstVerifyReport& rep, uint32_t* bcc_out, std::vector<Handle>* bulk) {
  rep = SstVerifyReport();
  hipStream_t st = static_cast<hipStream_t>(eng.stream());
  // 1. footer (ReadFooterFromFile, format.cc:486-553)
  forst_sst_footer f;
  const uint64_t tail = file_size < kNewVersionsLen ? file_size : kNewVersionsLen;
  int rc = footer_decode(host_file + file_size - tail, tail, file_size, &f);
  if (rc) return from_sst_rc(rc, file_name);
  rep.format_version = f.format_version;
  rep.checksum_type = f.checksum_type;
  const ChecksumType type = static_cast<ChecksumType>(f.checksum_type);
  const uint32_t bcc = f.base_context_checksum;
  if (bcc_out) *bcc_out = bcc;
  // footer checksum (fv >= 6): ComputeBuiltinChecksum over the 53 footer bytes
  // with the field zeroed, + ChecksumModifierForContext(base, footer_offset),
  // on the GPU (compute mode: 52 bytes + the last one from memory)
  if (f.format_version >= 6) {  // (kNoChecksum: computed = 0 + modifier)
    void* d = nullptr;
    Status s = hip_status(forst::scratch_alloc(&d, 256, st), "scratch_alloc");
    if (!s.ok()) return s;
    uint8_t* dz = static_cast<uint8_t*>(d);
    uint64_t* doff = reinterpret_cast<uint64_t*>(dz + 64);
    uint32_t* dsz = reinterpret_cast<uint32_t*>(dz + 72);
    uint32_t* dmod = reinterpret_cast<uint32_t*>(dz + 76);
    uint32_t* dout = reinterpret_cast<uint32_t*>(dz + 80);
    const uint64_t zero = 0;
    const uint32_t n52 = kNewVersionsLen - 1, mod = f.footer_checksum_modifier;
    uint32_t got = 0;
    s = hip_status(hipMemcpyAsync(dz, f.footer_zeroed, kNewVersionsLen, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s.ok()) s = hip_status(hipMemcpyAsync(doff, &zero, 8, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s.ok()) s = hip_status(hipMemcpyAsync(dsz, &n52, 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s.ok()) s = hip_status(hipMemcpyAsync(dmod, &mod, 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s.ok()) {
      rc = forst_block_checksum_batch(type, dz, kNewVersionsLen, doff, dsz, nullptr, dmod, dout, 1,
                                      eng.stream());
      if (rc) s = Status::IOError(std::string("footer checksum launch: ") + forst_last_error());
    }
    if (s.ok()) s = hip_status(hipMemcpyAsync(&got, dout, 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    if (s.ok()) s = hip_status(hipStreamSynchronize(st), "hipStreamSynchronize");
    (void)forst::scratch_free(d, st);
    if (!s.ok()) return s;
    if (got != f.stored_footer_checksum)  // format.cc:425-428
      return Status::Corruption("Footer at " + std::to_string(f.footer_offset) +
                                " checksum mismatch in " + file_name);
  }
  if (f.future_feature)  // format.cc:440-448, after the checksum compare
    return Status::NotSupported("File uses a future feature not supported in this version in " +
                                file_name);
  // device descriptors for block batches
  auto verify = [&](const std::vector<Handle>& hs, std::vector<uint64_t>* failed) -> Status {
    if (hs.empty()) return Status::OK();
    for (const Handle& h : hs)
      if (h.off > file_size || h.size > file_size - h.off || file_size - h.off - h.size < kBlockTrailer)
        return Status::Corruption("block handle past end of file in " + file_name);
    std::vector<uint64_t> offs(hs.size());
    std::vector<uint32_t> sz(hs.size());
    for (size_t i = 0; i < hs.size(); ++i) {
      offs[i] = hs[i].off;
      if (hs[i].size > 0xffffffffull) return Status::NotSupported("block larger than 4 GiB");
      sz[i] = static_cast<uint32_t>(hs[i].size);
    }
    void* d = nullptr;
    Status s = hip_status(forst::scratch_alloc(&d, hs.size() * 12 + 256, st), "scratch_alloc");
    if (!s.ok()) return s;
    uint64_t* doffs = static_cast<uint64_t*>(d);
    uint32_t* dsz = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d) + hs.size() * 8);
    s = hip_status(hipMemcpyAsync(doffs, offs.data(), hs.size() * 8, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s.ok()) s = hip_status(hipMemcpyAsync(dsz, sz.data(), hs.size() * 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s.ok()) {
      DeviceBlockBatch b;
      b.base = dev_file;
      b.base_len = file_size;
      b.offsets = doffs;
      b.sizes = dsz;
      b.n = hs.size();
      s = eng.VerifyBlocks(type, bcc, b, file_name, offs, failed);
      rep.blocks_verified += hs.size();
    }
    (void)hipStreamSynchronize(st);
    (void)forst::scratch_free(d, st);
    return s;
  };
  // VerifyBlockChecksum over a host copy of block h (+ trailer) whose 8 bytes
  // at `zero_at` are zeroed (meta_blocks.cc:407-414), checksummed on the GPU
  auto verify_patched = [&](const Handle& h, uint64_t zero_at) -> Status {
    const uint64_t len = h.size + kBlockTrailer;
    std::vector<uint8_t> tmp(host_file + h.off, host_file + h.off + len);
    std::memset(tmp.data() + zero_at, 0, 8);
    void* d = nullptr;
    Status s2 = hip_status(forst::scratch_alloc(&d, len + 256, st), "scratch_alloc");
    if (!s2.ok()) return s2;
    uint8_t* dblk = static_cast<uint8_t*>(d);
    uint64_t* doff = reinterpret_cast<uint64_t*>(dblk + ((len + 15) & ~uint64_t(15)));
    uint32_t* dsz = reinterpret_cast<uint32_t*>(doff + 1);
    const uint64_t zero = 0;
    const uint32_t sz = static_cast<uint32_t>(h.size);
    s2 = hip_status(hipMemcpyAsync(dblk, tmp.data(), len, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s2.ok()) s2 = hip_status(hipMemcpyAsync(doff, &zero, 8, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s2.ok()) s2 = hip_status(hipMemcpyAsync(dsz, &sz, 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
    if (s2.ok()) {
      DeviceBlockBatch b;
      b.base = dblk;
      b.base_len = len;
      b.offsets = doff;
      b.sizes = dsz;
      b.n = 1;
      s2 = eng.VerifyBlocks(type, bcc, b, file_name, {h.off}, nullptr);
    }
    (void)hipStreamSynchronize(st);
    (void)forst::scratch_free(d, st);
    return s2;
  };
  // the contents BlockFetcher hands the reader after the checksum check:
  // decompressed when the trailer's type byte says so (block_fetcher.cc:
  // 333-345, UncompressSerializedBlock) -- metaindex, index and index
  // partitions; the properties block is read raw (meta_blocks.cc:258-262,
  // decompress = false)
  std::vector<std::vector<uint8_t>> keep;  // decompressed contents in use
  auto host_block = [&](const Handle& h, const char* what, bool decompress, const uint8_t** data,
                        uint64_t* size) -> Status {
    if (h.off > file_size || h.size > file_size - h.off || file_size - h.off - h.size < kBlockTrailer)
      return Status::Corruption(std::string(what) + " block handle past end of file in " + file_name);
    *data = host_file + h.off;
    *size = h.size;
    const uint8_t t = host_file[h.off + h.size];
    if (!decompress || t == 0) return Status::OK();
    keep.emplace_back();
    std::string err;
    const int rc2 = forst::uncompress_block(t, f.format_version, host_file + h.off, h.size,
                                            &keep.back(), &err);
    if (rc2 == FORST_EUNSUPPORTED) return Status::NotSupported(err);
    if (rc2 != FORST_OK) return Status::Corruption(err);
    *data = keep.back().data();
    *size = keep.back().size();
    return Status::OK();
  };
  // 2. metaindex (+ index when the footer holds it) read with checksum verify
  const Handle mi{f.metaindex_offset, f.metaindex_size};
  std::vector<Handle> first = {mi};
  Handle ix{f.index_offset, f.index_size};
  const bool index_in_footer = f.format_version < 6;
  if (index_in_footer) first.push_back(ix);
  Status s = verify(first, nullptr);
  if (!s.ok()) return s;
  const uint8_t* blk = nullptr;
  uint64_t blk_size = 0;
  s = host_block(mi, "metaindex", true, &blk, &blk_size);
  if (!s.ok()) return s;
  std::vector<MetaEntry> meta;
  rc = metaindex_entries(blk, blk_size, &meta);
  if (rc) return from_sst_rc(rc, file_name, false);
  // 3. properties (ReadTablePropertiesHelper) and the index handle (fv >= 6)
  forst_sst_properties props;
  std::memset(&props, 0, sizeof(props));
  bool have_index = index_in_footer;
  std::vector<Handle> meta_blocks;  // VerifyChecksumInMetaBlocks order
  for (const MetaEntry& e : meta) {
    if (e.name == "rocksdb.properties" || e.name == "rocksdb.stats") {
      // ReadTablePropertiesHelper (meta_blocks.cc:250-417): decode, then the
      // checksum -- retried with an ingested file's global seqno zeroed
      s = host_block(e.h, "properties", false, &blk, &blk_size);
      if (!s.ok()) return s;
      rc = properties(blk, blk_size, &props);
      if (rc) return from_sst_rc(rc, file_name, false);
      s = verify({e.h}, nullptr);
      if (s.IsCorruption() && props.global_seqno_value_offset != 0 &&
          props.global_seqno_value_offset + 8 <= e.h.size) {
        s = verify_patched(e.h, props.global_seqno_value_offset);
      }
      if (!s.ok()) return s;
    } else if (e.name == "rocksdb.index") {
      ix = e.h;
      have_index = true;
      meta_blocks.push_back(e.h);  // verified with the other meta blocks
    } else {
      meta_blocks.push_back(e.h);
    }
  }
  // FindMetaBlock (meta_blocks.cc:478-486)
  if (!have_index) return Status::Corruption("Cannot find the meta block: rocksdb.index");
  rep.index_type = props.index_type;
  // 4. index (and partitions) -> data block handles
  if (!index_in_footer) {
    s = verify({ix}, nullptr);
    if (!s.ok()) return s;
  }
  s = host_block(ix, "index", true, &blk, &blk_size);
  if (!s.ok()) return s;
  const bool delta = props.index_value_is_delta_encoded != 0;
  const bool first_key = props.index_type == 3;  // kBinarySearchWithFirstKey
  std::vector<Handle> top, data;
  rc = index_handles(blk, blk_size, delta, first_key, &top);
  if (rc) return from_sst_rc(rc, file_name, false);
  if (props.index_type == 2) {  // kTwoLevelIndexSearch: top level -> partitions
    rep.index_partitions = top.size();
    s = verify(top, nullptr);
    if (!s.ok()) return s;
    for (const Handle& p : top) {
      s = host_block(p, "index partition", true, &blk, &blk_size);
      if (!s.ok()) return s;
      rc = index_handles(blk, blk_size, delta, first_key, &data);
      if (rc) return from_sst_rc(rc, file_name, false);
    }
  } else {
    data.swap(top);
  }
  rep.data_blocks = data.size();
  rep.meta_blocks = meta_blocks.size();
  // 5. every meta block, then every data block, in one launch
  std::vector<Handle> all(meta_blocks);
  all.insert(all.end(), data.begin(), data.end());
  if (bulk) {
    for (const Handle& h : all)
      if (h.off > file_size || h.size > file_size - h.off || file_size - h.off - h.size < kBlockTrailer)
        return Status::Corruption("block handle past end of file in " + file_name);
    for (const Handle& h : all)
      if (h.size > 0xffffffffull) return Status::NotSupported("block larger than 4 GiB");
    bulk->swap(all);
    return Status::OK();
  }
  return verify(all, &rep.failed);
}

Status VerifySstFileChecksums(BlockChecksumEngine& eng, const uint8_t* host_file,
                              uint64_t file_size, const uint8_t* dev_file,
                              const std::string& file_name, SstVerifyReport* report) {
  SstVerifyReport local;
  return WalkSstFile(eng, host_file, file_size, dev_file, file_name, report ? *report : local,
                     nullptr, nullptr);
}

// DB::VerifyChecksum over many files (db_impl.cc:6254 walks every live SST
// file, convenience.cc:57 per file).  Structural blocks are checked per file
// (they gate the decoding of what follows); the meta + data blocks of ALL
// files then go to the GPU as one batch per checksum type over the arena,
// with per-block context modifiers (fv >= 6 files carry their own base).
std::vector<Status> VerifySstFilesChecksums(BlockChecksumEngine& eng,
                                            const std::vector<SstFileRef>& files,
                                            const uint8_t* dev_arena, uint64_t arena_len,
                                            std::vector<SstVerifyReport>* reports) {
  const size_t nf = files.size();
  std::vector<Status> out(nf);
  std::vector<SstVerifyReport> local;
  std::vector<SstVerifyReport>& reps = reports ? *reports : local;
  reps.assign(nf, SstVerifyReport());
  hipStream_t st = static_cast<hipStream_t>(eng.stream());
  struct Blk {
    uint32_t file, idx;
    uint64_t off;  // in the file
    uint32_t size;
  };
  std::vector<Blk> by_type[5];
  std::vector<uint32_t> bcc(nf, 0);
  for (size_t f = 0; f < nf; ++f) {
    const SstFileRef& r = files[f];
    if (r.dev_offset > arena_len || r.file_size > arena_len - r.dev_offset) {
      out[f] = Status::InvalidArgument("file " + r.file_name + " outside the device arena");
      continue;
    }
    if ((reinterpret_cast<uintptr_t>(dev_arena) + r.dev_offset) & 3) {
      out[f] = Status::InvalidArgument("file " + r.file_name +
                                       ": device offset must be 4-byte aligned");
      continue;
    }
    std::vector<Handle> bulk;
    out[f] = WalkSstFile(eng, r.host_file, r.file_size, dev_arena + r.dev_offset, r.file_name,
                         reps[f], &bcc[f], &bulk);
    if (!out[f].ok()) continue;
    const int t = reps[f].checksum_type;
    if (t < 0 || t > 4) {
      out[f] = Status::Corruption("Corrupt or unsupported checksum type: " + std::to_string(t));
      continue;
    }
    for (size_t i = 0; i < bulk.size(); ++i)
      by_type[t].push_back({uint32_t(f), uint32_t(i), bulk[i].off, uint32_t(bulk[i].size)});
  }
  for (int t = 0; t < 5; ++t) {
    const std::vector<Blk>& v = by_type[t];
    if (v.empty()) continue;
    const uint64_t n = v.size();
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> sz(n), mods(n);
    for (uint64_t i = 0; i < n; ++i) {
      offs[i] = files[v[i].file].dev_offset + v[i].off;
      sz[i] = v[i].size;
      mods[i] = ChecksumModifierForContext(bcc[v[i].file], v[i].off);
    }
    // device layout: offsets | sizes | modifiers | computed | stored | ok | bad
    const uint64_t need = n * (8 + 4 + 4 + 4 + 4 + 1) + 64;
    void* d = nullptr;
    Status s = hip_status(hipMallocAsync(&d, need, st), "hipMallocAsync");
    std::vector<uint8_t> ok(n);
    std::vector<uint32_t> computed(n), stored(n);
    if (s.ok()) {
      uint8_t* p = static_cast<uint8_t*>(d);
      uint64_t* doffs = reinterpret_cast<uint64_t*>(p);
      uint32_t* dsz = reinterpret_cast<uint32_t*>(p + n * 8);
      uint32_t* dmod = dsz + n;
      uint32_t* dcomp = dmod + n;
      uint32_t* dstor = dcomp + n;
      uint8_t* dok = reinterpret_cast<uint8_t*>(dstor + n);
      unsigned long long* dbad =
          reinterpret_cast<unsigned long long*>(p + ((n * 24 + n + 7) & ~uint64_t(7)));
      unsigned long long bad = 0;
      s = hip_status(hipMemcpyAsync(doffs, offs.data(), n * 8, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
      if (s.ok()) s = hip_status(hipMemcpyAsync(dsz, sz.data(), n * 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
      if (s.ok()) s = hip_status(hipMemcpyAsync(dmod, mods.data(), n * 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
      if (s.ok()) s = hip_status(hipMemsetAsync(dbad, 0, 8, st), "hipMemsetAsync");
      if (s.ok()) {
        int rc = forst_block_verify_batch(t, dev_arena, arena_len, doffs, dsz, dmod, dcomp, dstor,
                                          dok, dbad, n, eng.stream());
        if (rc) s = Status::IOError(std::string("verify launch: ") + forst_last_error());
      }
      if (s.ok()) s = hip_status(hipMemcpyAsync(&bad, dbad, 8, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
      if (s.ok()) s = hip_status(hipStreamSynchronize(st), "hipStreamSynchronize");
      if (s.ok() && bad) {
        s = hip_status(hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
        if (s.ok()) s = hip_status(hipMemcpyAsync(computed.data(), dcomp, n * 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
        if (s.ok()) s = hip_status(hipMemcpyAsync(stored.data(), dstor, n * 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
        if (s.ok()) s = hip_status(hipStreamSynchronize(st), "hipStreamSynchronize");
      } else {
        std::fill(ok.begin(), ok.end(), 1);
      }
      (void)hipFreeAsync(d, st);
    }
    const ChecksumType type = static_cast<ChecksumType>(t);
    for (uint64_t i = 0; i < n; ++i) {
      const Blk& b = v[i];
      if (!s.ok()) {
        if (out[b.file].ok()) out[b.file] = s;
        continue;
      }
      reps[b.file].blocks_verified += 1;
      if (ok[i]) continue;
      reps[b.file].failed.push_back(b.idx);
      if (out[b.file].ok()) {  // blocks of a file are in walk order: first failure wins
        uint32_t st_v = stored[i], co_v = computed[i];
        if (type == kCRC32c) {  // reader_common.cc:50-54
          st_v = crc32c::Unmask(st_v);
          co_v = crc32c::Unmask(co_v);
        }
        out[b.file] = Status::Corruption(BlockChecksumMismatchMessage(
            type, st_v, co_v, mods[i] != 0, files[b.file].file_name, b.off, b.size));
      }
    }
  }
  return out;
}

}  // namespace forst_gpu

namespace {
void fill_result(forst_sst_verify_result* out, const forst_gpu::Status& s,
                 const forst_gpu::SstVerifyReport& rep) {
  std::memset(out, 0, sizeof(*out));
  out->status = s.code();
  out->blocks_verified = rep.blocks_verified;
  out->data_blocks = rep.data_blocks;
  out->meta_blocks = rep.meta_blocks;
  out->index_partitions = rep.index_partitions;
  out->n_failed = rep.failed.size();
  out->format_version = rep.format_version;
  out->checksum_type = rep.checksum_type;
  out->index_type = rep.index_type;
  std::strncpy(out->message, s.ok() ? "OK" : s.ToString().c_str(), sizeof(out->message) - 1);
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int forst_sst_verify_files(
    const uint8_t* const* host_files, const uint64_t* file_sizes, const uint64_t* dev_offsets,
    const uint8_t* dev_arena, uint64_t arena_len, const char* const* file_names, uint64_t n_files,
    forst_sst_verify_result* out, void* stream) {
  if (n_files == 0) return FORST_OK;
  if (!host_files || !file_sizes || !dev_offsets || !dev_arena || !out) return FORST_EINVAL;
  std::vector<forst_gpu::SstFileRef> files(n_files);
  for (uint64_t i = 0; i < n_files; ++i) {
    if (!host_files[i]) return FORST_EINVAL;
    files[i].host_file = host_files[i];
    files[i].file_size = file_sizes[i];
    files[i].dev_offset = dev_offsets[i];
    files[i].file_name = (file_names && file_names[i]) ? file_names[i] : "";
  }
  forst_gpu::BlockChecksumEngine eng(stream);
  std::vector<forst_gpu::SstVerifyReport> reps;
  std::vector<forst_gpu::Status> st =
      forst_gpu::VerifySstFilesChecksums(eng, files, dev_arena, arena_len, &reps);
  for (uint64_t i = 0; i < n_files; ++i) fill_result(&out[i], st[i], reps[i]);
  return FORST_OK;
}

extern "C" __attribute__((visibility("default"))) int forst_sst_verify_file(
    const uint8_t* host_file, uint64_t file_size, const uint8_t* dev_file, const char* file_name,
    forst_sst_verify_result* out, void* stream) {
  if (!host_file || !dev_file || !out) return FORST_EINVAL;
  forst_gpu::BlockChecksumEngine eng(stream);
  forst_gpu::SstVerifyReport rep;
  forst_gpu::Status s = forst_gpu::VerifySstFileChecksums(eng, host_file, file_size, dev_file,
                                                      file_name ? file_name : "", &rep);
  fill_result(out, s, rep);
  return FORST_OK;
}
