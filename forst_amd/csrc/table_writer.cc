// forst_amd/csrc/table_writer.cc -- write-side batching for flush and
// compaction: BlockBasedTableBuilder::
// WriteMaybeCompressedBlock (table/block_based/block_based_table_builder.cc:
// 1311-1360) with the trailer deferred to a GPU batch.
//
// The reference appends every block and immediately its 5-byte trailer
// [compression type][LE32 ComputeBuiltinChecksumWithLastByte(block, type) +
// ChecksumModifierForContext(base_context_checksum, offset)].  Here a block is
// placed at its final file offset at once -- the handle is known, the builder
// can index it -- with the type byte written and the 4 checksum bytes left
// open; blocks accumulate in a pinned host window and a full window goes to
// the GPU in ONE forst_block_checksum_batch (the type byte is read from the
// window, the fv6 modifier is the block's), the checksums come back and fill
// the open bytes, and the window is handed to the file (the sink:
// WritableFileWriter::Append).  Two windows alternate so the builder keeps
// filling one while the other is on the GPU -- the role of the parallel-
// compression writer queue (:1416-1481), which is where ForSt would defer.
// block_align padding (:1385-1395) and the footer (FooterBuilder::Build,
// table/format.cc:231-330, fv6 footer checksum on the GPU) follow the
// reference.  The bytes emitted are those of the reference builder.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/forst/checksum_engine.h"
#include "../../include/forst_checksum.h"

namespace forst {  // the engine's stream-ordered scratch pool (capi.hip)
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t stream);
hipError_t scratch_free(void* p, hipStream_t stream);
}  // namespace forst

namespace forst_gpu {

namespace {
constexpr uint32_t kTrailer = 5;                                     // block_based_table_reader.h:75
constexpr uint64_t kBlockBasedTableMagicNumber = 0x88e241b785f4cff7ull;        // builder.cc:201
constexpr uint64_t kLegacyBlockBasedTableMagicNumber = 0xdb4775248b80fb57ull;  // builder.cc:204
constexpr uint32_t kFooterLen = 53;  // Footer::kNewVersionsEncodedLength (format.h:234)
constexpr uint32_t kVersion0Len = 48;

Status HipS(hipError_t e, const char* what) {
  return e == hipSuccess ? Status::OK()
                         : Status::IOError(std::string(what) + ": " + hipGetErrorString(e));
}

void PutFixed32(uint8_t* p, uint32_t v) {
  for (int i = 0; i < 4; ++i) p[i] = static_cast<uint8_t>(v >> (8 * i));
}
void PutFixed64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = static_cast<uint8_t>(v >> (8 * i));
}
uint8_t* PutVarint64(uint8_t* p, uint64_t v) {  // util/coding.h
  while (v >= 128) {
    *p++ = static_cast<uint8_t>(v | 128);
    v >>= 7;
  }
  *p++ = static_cast<uint8_t>(v);
  return p;
}
}  // namespace

struct GpuTrailerWriter::Window {
  uint64_t cap = 0;        // bytes
  uint64_t len = 0;        // bytes used
  uint64_t file_offset = 0;
  uint8_t* h = nullptr;    // pinned host window
  uint8_t* d = nullptr;    // device copy
  std::vector<uint64_t> offs;  // block offsets in the window
  std::vector<uint32_t> sizes, mods;
  uint64_t dcap_blocks = 0;
  uint64_t* d_offs = nullptr;
  uint32_t *d_sizes = nullptr, *d_mods = nullptr, *d_out = nullptr;
  uint32_t* h_out = nullptr;
  hipEvent_t done = nullptr;
  bool in_flight = false;
};

GpuTrailerWriter::GpuTrailerWriter(const Options& opt, Sink sink, void* stream)
    : opt_(opt), sink_(std::move(sink)), stream_(stream), offset_(opt.start_offset) {
  win_[0] = new Window();
  win_[1] = new Window();
}

GpuTrailerWriter::~GpuTrailerWriter() {
  for (Window* w : win_) {
    if (w->done) {
      (void)hipEventSynchronize(w->done);
      (void)hipEventDestroy(w->done);
    }
    (void)hipHostFree(w->h);
    (void)hipFree(w->d);
    (void)hipFree(w->d_offs);
    (void)hipHostFree(w->h_out);
    delete w;
  }
}

Status GpuTrailerWriter::Reserve(Window& w, uint64_t bytes, uint64_t blocks) {
  if (!w.done) {
    Status s = HipS(hipEventCreateWithFlags(&w.done, hipEventDisableTiming), "hipEventCreate");
    if (!s.ok()) return s;
  }
  if (bytes > w.cap) {  // only called on an empty window
    const uint64_t cap = std::max<uint64_t>(bytes, opt_.window_bytes);
    (void)hipHostFree(w.h);
    (void)hipFree(w.d);
    w.h = nullptr;
    w.d = nullptr;
    w.cap = 0;
    Status s = HipS(hipHostMalloc(&w.h, cap), "hipHostMalloc");
    if (s.ok()) s = HipS(hipMalloc(&w.d, (cap + 255) & ~uint64_t(255)), "hipMalloc");
    if (!s.ok()) return s;
    w.cap = cap;
  }
  if (blocks > w.dcap_blocks) {
    const uint64_t nb = std::max<uint64_t>(blocks, 2 * w.dcap_blocks + 1024);
    (void)hipFree(w.d_offs);
    (void)hipHostFree(w.h_out);
    w.d_offs = nullptr;
    w.h_out = nullptr;
    w.dcap_blocks = 0;
    void* p = nullptr;
    Status s = HipS(hipMalloc(&p, nb * 20), "hipMalloc");
    if (!s.ok()) return s;
    w.d_offs = static_cast<uint64_t*>(p);
    w.d_sizes = reinterpret_cast<uint32_t*>(w.d_offs + nb);
    w.d_mods = w.d_sizes + nb;
    w.d_out = w.d_mods + nb;
    s = HipS(hipHostMalloc(&p, nb * 4), "hipHostMalloc");
    if (!s.ok()) return s;
    w.h_out = static_cast<uint32_t*>(p);
    w.dcap_blocks = nb;
  }
  return Status::OK();
}

// the window's blocks in one GPU batch (asynchronous)
Status GpuTrailerWriter::Launch(Window& w) {
  const uint64_t n = w.offs.size();
  if (n == 0) return Status::OK();
  hipStream_t st = static_cast<hipStream_t>(stream_);
  Status s = HipS(hipMemcpyAsync(w.d, w.h, w.len, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok()) s = HipS(hipMemcpyAsync(w.d_offs, w.offs.data(), n * 8, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (s.ok()) s = HipS(hipMemcpyAsync(w.d_sizes, w.sizes.data(), n * 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  const bool ctx = opt_.base_context_checksum != 0;
  if (s.ok() && ctx) s = HipS(hipMemcpyAsync(w.d_mods, w.mods.data(), n * 4, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  if (!s.ok()) return s;
  // ComputeBuiltinChecksumWithLastByte(type, block, n, comp_type) +
  // ChecksumModifierForContext(base, offset): the type byte is in the window
  const int rc = forst_block_checksum_batch(opt_.checksum, w.d, w.len, w.d_offs, w.d_sizes, nullptr,
                                            ctx ? w.d_mods : nullptr, w.d_out, n, stream_);
  if (rc != FORST_OK) return Status::IOError(std::string("trailer batch: ") + forst_last_error());
  s = HipS(hipMemcpyAsync(w.h_out, w.d_out, n * 4, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
  if (s.ok()) s = HipS(hipEventRecord(w.done, st), "hipEventRecord");
  if (s.ok()) {
    w.in_flight = true;
    stats_.block_checksum_compute_count += n;
  }
  return s;
}

// wait for the window's checksums, fill the trailers, hand the bytes on
Status GpuTrailerWriter::Retire(Window& w) {
  if (w.in_flight) {
    Status s = HipS(hipEventSynchronize(w.done), "hipEventSynchronize");
    if (!s.ok()) return s;
    for (size_t i = 0; i < w.offs.size(); ++i) PutFixed32(w.h + w.offs[i] + w.sizes[i] + 1, w.h_out[i]);
    w.in_flight = false;
  }
  if (w.len) {
    Status s = sink_(reinterpret_cast<const char*>(w.h), w.len);
    if (!s.ok()) return s;
  }
  w.len = 0;
  w.offs.clear();
  w.sizes.clear();
  w.mods.clear();
  return Status::OK();
}

Status GpuTrailerWriter::AddBlock(const char* data, size_t n, uint8_t compression_type,
                                  bool is_data_block, uint64_t* handle_offset,
                                  uint64_t* handle_size) {
  if (!status_.ok()) return status_;
  if (n > 0xffffffffull) return status_ = Status::NotSupported("block larger than 4 GiB");
  uint64_t pad = 0;  // block_based_table_builder.cc:1385-1395
  if (opt_.block_align && is_data_block) {
    const uint64_t a = opt_.alignment;
    pad = (a - ((n + kTrailer) & (a - 1))) & (a - 1);
  }
  const uint64_t need = n + kTrailer + pad;
  Window* w = win_[cur_];
  if (w->len && w->len + need > w->cap) {
    // this window is full: on to the GPU, continue in the other one
    Status s = Launch(*w);
    cur_ ^= 1;
    w = win_[cur_];
    if (s.ok()) s = Retire(*w);  // the other window's earlier blocks go first
    if (!s.ok()) return status_ = s;
  }
  if (w->len == 0) {
    Status s = Reserve(*w, need, 0);
    if (!s.ok()) return status_ = s;
    w->file_offset = offset_;
  }
  Status s = Reserve(*w, 0, w->offs.size() + 1);
  if (!s.ok()) return status_ = s;
  // WriteMaybeCompressedBlock: handle = (offset, n), block, trailer
  *handle_offset = offset_;
  *handle_size = n;
  uint8_t* p = w->h + w->len;
  std::memcpy(p, data, n);
  p[n] = compression_type;  // trailer[0]; the LE32 checksum comes from the GPU
  std::memset(p + n + 1, 0, 4);
  if (pad) std::memset(p + n + kTrailer, 0, pad);  // WritableFileWriter::Pad
  w->offs.push_back(w->len);
  w->sizes.push_back(static_cast<uint32_t>(n));
  w->mods.push_back(ChecksumModifierForContext(opt_.base_context_checksum, offset_));
  w->len += need;
  offset_ += need;
  return Status::OK();
}

Status GpuTrailerWriter::Flush() {
  if (!status_.ok()) return status_;
  // file order: the other window's (earlier) blocks, then this one's
  Window* w = win_[cur_];
  Status s = Launch(*w);
  if (s.ok()) s = Retire(*win_[cur_ ^ 1]);
  if (s.ok()) s = Retire(*w);
  if (!s.ok()) status_ = s;
  return s;
}

Status GpuTrailerWriter::WriteFooter(uint32_t format_version, uint64_t metaindex_offset,
                                     uint64_t metaindex_size, uint64_t index_offset,
                                     uint64_t index_size) {
  Status s = Flush();
  if (!s.ok()) return s;
  uint8_t f[kFooterLen];
  uint32_t len = 0;
  const int rc = forst_sst_footer_build(format_version, opt_.checksum, offset_,
                                        opt_.base_context_checksum, metaindex_offset,
                                        metaindex_size, index_offset, index_size, f, &len,
                                        stream_);
  if (rc != FORST_OK) return status_ = Status::InvalidArgument(forst_sst_last_error());
  s = sink_(reinterpret_cast<const char*>(f), len);
  if (s.ok()) offset_ += len;
  return s;
}

}  // namespace forst_gpu

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
#define FORST_API extern "C" __attribute__((visibility("default")))

namespace {
thread_local std::string g_tw_err;
int tw_fail(const forst_gpu::Status& s) {
  g_tw_err = s.ToString();
  return s.IsCorruption() ? FORST_ECORRUPT
         : s.code() == forst_gpu::Status::kInvalidArgument ? FORST_EINVAL
         : s.code() == forst_gpu::Status::kNotSupported    ? FORST_EUNSUPPORTED
                                                         : FORST_EHIP;
}
}  // namespace

struct forst_trailer_writer {
  forst_gpu::GpuTrailerWriter* w;
};

FORST_API const char* forst_trailer_writer_last_error(void) { return g_tw_err.c_str(); }

FORST_API int forst_trailer_writer_open(int checksum_type, uint32_t base_context_checksum,
                                        uint64_t start_offset, uint32_t block_align,
                                        uint64_t window_bytes, forst_sink_fn sink, void* sink_arg,
                                        void* stream, forst_trailer_writer** out) {
  if (!out || !sink) return tw_fail(forst_gpu::Status::InvalidArgument("null sink / out"));
  if (checksum_type < FORST_kNoChecksum || checksum_type > FORST_kXXH3)
    return tw_fail(forst_gpu::Status::InvalidArgument("unknown ChecksumType " +
                                                    std::to_string(checksum_type)));
  if (block_align && (block_align & (block_align - 1)))
    return tw_fail(forst_gpu::Status::InvalidArgument("alignment must be a power of 2"));
  forst_gpu::GpuTrailerWriter::Options o;
  o.checksum = static_cast<forst_gpu::ChecksumType>(checksum_type);
  o.base_context_checksum = base_context_checksum;
  o.start_offset = start_offset;
  o.block_align = block_align != 0;
  o.alignment = block_align ? block_align : 4096;
  if (window_bytes) o.window_bytes = window_bytes;
  auto fn = [sink, sink_arg](const char* d, size_t n) {
    return sink(sink_arg, reinterpret_cast<const uint8_t*>(d), n) == 0
               ? forst_gpu::Status::OK()
               : forst_gpu::Status::IOError("sink failed");
  };
  *out = new forst_trailer_writer{new forst_gpu::GpuTrailerWriter(o, fn, stream)};
  return FORST_OK;
}

FORST_API int forst_trailer_writer_add(forst_trailer_writer* w, const uint8_t* block,
                                       uint64_t size, uint8_t compression_type,
                                       int is_data_block, uint64_t* handle_offset,
                                       uint64_t* handle_size) {
  if (!w || (!block && size) || !handle_offset || !handle_size)
    return tw_fail(forst_gpu::Status::InvalidArgument("null argument"));
  forst_gpu::Status s = w->w->AddBlock(reinterpret_cast<const char*>(block), size, compression_type,
                                     is_data_block != 0, handle_offset, handle_size);
  return s.ok() ? FORST_OK : tw_fail(s);
}

FORST_API int forst_trailer_writer_flush(forst_trailer_writer* w) {
  if (!w) return tw_fail(forst_gpu::Status::InvalidArgument("null writer"));
  forst_gpu::Status s = w->w->Flush();
  return s.ok() ? FORST_OK : tw_fail(s);
}

FORST_API int forst_trailer_writer_footer(forst_trailer_writer* w, uint32_t format_version,
                                          uint64_t metaindex_offset, uint64_t metaindex_size,
                                          uint64_t index_offset, uint64_t index_size) {
  if (!w) return tw_fail(forst_gpu::Status::InvalidArgument("null writer"));
  forst_gpu::Status s = w->w->WriteFooter(format_version, metaindex_offset, metaindex_size,
                                        index_offset, index_size);
  return s.ok() ? FORST_OK : tw_fail(s);
}

FORST_API uint64_t forst_trailer_writer_offset(const forst_trailer_writer* w) {
  return w ? w->w->offset() : 0;
}

FORST_API int forst_trailer_writer_close(forst_trailer_writer* w) {
  if (!w) return FORST_OK;
  forst_gpu::Status s = w->w->Flush();
  delete w->w;
  delete w;
  return s.ok() ? FORST_OK : tw_fail(s);
}

// FooterBuilder::Build (table/format.cc:231-330) for the block-based table.
// fv >= 6: the footer checksum = ComputeBuiltinChecksum(type, footer with the
// field zeroed, 53) + ChecksumModifierForContext(base, footer_offset), on the
// GPU (compute mode: 52 bytes + the last from memory).
FORST_API int forst_sst_footer_build(uint32_t format_version, int checksum_type,
                                     uint64_t footer_offset, uint32_t base_context_checksum,
                                     uint64_t metaindex_offset, uint64_t metaindex_size,
                                     uint64_t index_offset, uint64_t index_size, uint8_t* out,
                                     uint32_t* out_len, void* stream) {
  using forst_gpu::PutFixed32;
  using forst_gpu::PutFixed64;
  if (!out || !out_len) return FORST_EINVAL;
  if (format_version > 6 || checksum_type < 0 || checksum_type > 4) return FORST_EINVAL;
  uint8_t f[forst_gpu::kFooterLen];
  std::memset(f, 0, sizeof(f));
  if (format_version == 0) {  // legacy: part2 + legacy magic, kCRC32c implied
    if (checksum_type != FORST_kCRC32c && checksum_type != FORST_kNoChecksum) return FORST_EINVAL;
    uint8_t* cur = forst_gpu::PutVarint64(f, metaindex_offset);
    cur = forst_gpu::PutVarint64(cur, metaindex_size);
    cur = forst_gpu::PutVarint64(cur, index_offset);
    forst_gpu::PutVarint64(cur, index_size);
    PutFixed64(f + 40, forst_gpu::kLegacyBlockBasedTableMagicNumber);
    std::memcpy(out, f, forst_gpu::kVersion0Len);
    *out_len = forst_gpu::kVersion0Len;
    return FORST_OK;
  }
  f[0] = static_cast<uint8_t>(checksum_type);
  PutFixed32(f + 41, format_version);
  PutFixed64(f + 45, forst_gpu::kBlockBasedTableMagicNumber);
  if (format_version < 6) {
    uint8_t* cur = forst_gpu::PutVarint64(f + 1, metaindex_offset);
    cur = forst_gpu::PutVarint64(cur, metaindex_size);
    cur = forst_gpu::PutVarint64(cur, index_offset);
    forst_gpu::PutVarint64(cur, index_size);
    std::memcpy(out, f, forst_gpu::kFooterLen);
    *out_len = forst_gpu::kFooterLen;
    return FORST_OK;
  }
  if (forst_gpu::ChecksumModifierForContext(base_context_checksum, 0) == 0) return FORST_EINVAL;
  if (metaindex_size > 0xffffffffull) return FORST_EUNSUPPORTED;  // "Metaindex block size > 4GB"
  static const uint8_t kExt[4] = {0x3e, 0x00, 0x7a, 0x00};
  std::memcpy(f + 1, kExt, 4);
  PutFixed32(f + 9, base_context_checksum);
  PutFixed32(f + 13, static_cast<uint32_t>(metaindex_size));
  // checksum field (f + 5) zero; compute on the GPU, in scratch from the
  // engine's stream-ordered pool (no driver allocation per footer)
  hipStream_t st = static_cast<hipStream_t>(stream);
  void* d = nullptr;
  if (forst::scratch_alloc(&d, 256, st) != hipSuccess) return FORST_EHIP;
  uint8_t* dz = static_cast<uint8_t*>(d);
  uint64_t* doff = reinterpret_cast<uint64_t*>(dz + 64);
  uint32_t* dsz = reinterpret_cast<uint32_t*>(dz + 72);
  uint32_t* dmod = reinterpret_cast<uint32_t*>(dz + 76);
  uint32_t* dout = reinterpret_cast<uint32_t*>(dz + 80);
  const uint64_t zero = 0;
  const uint32_t n52 = forst_gpu::kFooterLen - 1;
  const uint32_t mod = forst_gpu::ChecksumModifierForContext(base_context_checksum, footer_offset);
  uint32_t c = 0;
  bool ok = hipMemcpyAsync(dz, f, forst_gpu::kFooterLen, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(doff, &zero, 8, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dsz, &n52, 4, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dmod, &mod, 4, hipMemcpyHostToDevice, st) == hipSuccess;
  int rc = ok ? forst_block_checksum_batch(checksum_type, dz, forst_gpu::kFooterLen, doff, dsz,
                                           nullptr, dmod, dout, 1, stream)
              : FORST_EHIP;
  if (rc == FORST_OK)
    rc = hipMemcpyAsync(&c, dout, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipStreamSynchronize(st) == hipSuccess
             ? FORST_OK
             : FORST_EHIP;
  (void)forst::scratch_free(d, st);
  if (rc != FORST_OK) return rc;
  PutFixed32(f + 5, c);
  std::memcpy(out, f, forst_gpu::kFooterLen);
  *out_len = forst_gpu::kFooterLen;
  return FORST_OK;
}
