// forst_amd/csrc/wal_host.cc -- host-side WAL framing for the writer path.
//
// log::Writer::AddRecord (db/log_writer.cc:65-160, no compression) splits each
// logical record into physical records that never straddle a 32 KiB log block
// (db/log_format.h:45), zero-pads a block tail shorter than a header
// (:86-102) and types the fragments Full / First / Middle / Last
// (:133-146; the recyclable types when recycling, log_format.h:20-41).  The
// layout is a serial walk over the records (each fragment's position depends
// on all earlier ones), cheap on the host; the bytes themselves are written on
// the GPU and the CRCs filled in place by forst_wal_record_crc_batch.
#include <cstdint>

#include "../../include/forst_checksum.h"

namespace {
constexpr uint32_t kBlockSize = 32768;   // db/log_format.h:45
constexpr uint32_t kHeaderSize = 7;      // db/log_format.h:48
constexpr uint32_t kRecyclableHeaderSize = 11;  // db/log_format.h:52
enum : uint8_t {  // db/log_format.h:20-41
  kFullType = 1, kFirstType = 2, kMiddleType = 3, kLastType = 4,
  kRecyclableFullType = 5, kRecyclableFirstType = 6, kRecyclableMiddleType = 7,
  kRecyclableLastType = 8,
};
}  // namespace

extern "C" __attribute__((visibility("default"))) int forst_wal_layout_at(
    const uint32_t* lengths, uint64_t n_records, int recyclable, uint32_t block_offset,
    uint64_t* rec_offsets, uint32_t* rec_lengths, uint8_t* rec_types, uint64_t capacity,
    uint64_t* pad_offsets, uint32_t* pad_lengths, uint64_t pad_capacity, uint64_t* n_phys,
    uint64_t* n_pads, uint64_t* total_bytes, uint32_t* end_block_offset) {
  if (n_records && !lengths) return FORST_EINVAL;
  if (block_offset > kBlockSize) return FORST_EINVAL;
  const uint32_t hs = recyclable ? kRecyclableHeaderSize : kHeaderSize;
  uint64_t off = 0, np = 0, npad = 0;
  uint32_t bo = block_offset;  // Writer::block_offset_ (offsets below: from the append position)
  for (uint64_t r = 0; r < n_records; ++r) {
    uint64_t left = lengths[r];
    bool begin = true;
    do {  // log_writer.cc:86-151
      const uint32_t leftover = kBlockSize - bo;
      if (leftover < hs) {
        if (leftover > 0) {
          if (pad_offsets && npad < pad_capacity) {
            pad_offsets[npad] = off;
            if (pad_lengths) pad_lengths[npad] = leftover;
          }
          ++npad;
        }
        off += leftover;
        bo = 0;
      }
      const uint32_t avail = kBlockSize - bo - hs;
      const uint64_t frag = left < avail ? left : avail;
      const bool end = left == frag;
      uint8_t type;
      if (begin && end)
        type = recyclable ? kRecyclableFullType : kFullType;
      else if (begin)
        type = recyclable ? kRecyclableFirstType : kFirstType;
      else if (end)
        type = recyclable ? kRecyclableLastType : kLastType;
      else
        type = recyclable ? kRecyclableMiddleType : kMiddleType;
      if (np < capacity) {
        if (rec_offsets) rec_offsets[np] = off;
        if (rec_lengths) rec_lengths[np] = static_cast<uint32_t>(frag);
        if (rec_types) rec_types[np] = type;
      }
      ++np;
      off += hs + frag;
      bo += hs + static_cast<uint32_t>(frag);
      left -= frag;
      begin = false;
    } while (left > 0);
  }
  if (n_phys) *n_phys = np;
  if (n_pads) *n_pads = npad;
  if (total_bytes) *total_bytes = off;
  if (end_block_offset) *end_block_offset = bo;
  return (np > capacity || npad > pad_capacity) && (rec_offsets || pad_offsets) ? FORST_EINVAL
                                                                                : FORST_OK;
}

// a fresh log (Writer::block_offset_ = 0, log_writer.cc:25)
extern "C" __attribute__((visibility("default"))) int forst_wal_layout(
    const uint32_t* lengths, uint64_t n_records, int recyclable, uint64_t* rec_offsets,
    uint32_t* rec_lengths, uint8_t* rec_types, uint64_t capacity, uint64_t* pad_offsets,
    uint32_t* pad_lengths, uint64_t pad_capacity, uint64_t* n_phys, uint64_t* n_pads,
    uint64_t* total_bytes) {
  return forst_wal_layout_at(lengths, n_records, recyclable, 0, rec_offsets, rec_lengths,
                             rec_types, capacity, pad_offsets, pad_lengths, pad_capacity, n_phys,
                             n_pads, total_bytes, nullptr);
}
