// tests/golden/ref_sst_shim.cc -- TEST INFRASTRUCTURE ONLY (fixture generation).
//
// extern "C" veneer over the reference's OWN block-based-table writer pieces,
// compiled by tests/golden/gen_sst_golden.py from the sources where they lie
// under /root/reference into a temporary directory outside the repository
// (hidden visibility + --gc-sections: only what these functions reach is
// linked).  Every function forwards to the reference symbol named in its
// comment; nothing here restates an encoding.  The library never enters the
// repository or travels to the GPU box; the product never links or loads it.

#include <cstdint>
#include <cstring>
#include <string>

#include "rocksdb/table.h"
#include "table/block_based/block_builder.h"
#include "table/format.h"
#include "table/meta_blocks.h"

using namespace ROCKSDB_NAMESPACE;

#define SHIM_API extern "C" __attribute__((visibility("default")))

static int put_out(const Slice& r, char* out, uint64_t cap, uint64_t* out_len) {
  if (r.size() > cap) return -1;
  std::memcpy(out, r.data(), r.size());
  *out_len = r.size();
  return 0;
}

// table/format.cc:231 FooterBuilder::Build (legacy magic for format_version 0
// chosen by the builder itself)
SHIM_API int ref_footer_build(uint64_t magic, uint32_t format_version, uint64_t footer_offset,
                              int checksum_type, uint64_t mi_off, uint64_t mi_size,
                              uint64_t ix_off, uint64_t ix_size, uint32_t base_context_checksum,
                              char* out, uint64_t cap, uint64_t* out_len) {
  FooterBuilder fb;
  Status s = fb.Build(magic, format_version, footer_offset, static_cast<ChecksumType>(checksum_type),
                      BlockHandle(mi_off, mi_size), BlockHandle(ix_off, ix_size),
                      base_context_checksum);
  if (!s.ok()) return -2;
  return put_out(fb.GetSlice(), out, cap, out_len);
}

// table/block_based/block_builder.cc BlockBuilder(restart_interval,
// use_delta_encoding, use_value_delta_encoding) + Add(key, value,
// delta_value) + Finish.  Entries: [u32 klen][u32 vlen][u32 dlen or
// 0xffffffff][key][value][delta]
SHIM_API int ref_block_build(int restart_interval, int delta_keys, int value_delta,
                             const char* entries, uint32_t n, char* out, uint64_t cap,
                             uint64_t* out_len) {
  BlockBuilder b(restart_interval, delta_keys != 0, value_delta != 0);
  const char* p = entries;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t kl, vl, dl;
    std::memcpy(&kl, p, 4);
    std::memcpy(&vl, p + 4, 4);
    std::memcpy(&dl, p + 8, 4);
    p += 12;
    const Slice key(p, kl), value(p + kl, vl);
    p += kl + vl;
    if (dl != 0xffffffffu) {
      const Slice delta(p, dl);
      p += dl;
      b.Add(key, value, &delta);
    } else {
      b.Add(key, value);
    }
  }
  return put_out(b.Finish(), out, cap, out_len);
}

// table/format.cc:60 BlockHandle::EncodeTo
SHIM_API int ref_handle_encode(uint64_t off, uint64_t size, char* out, uint64_t cap,
                               uint64_t* out_len) {
  std::string s;
  BlockHandle(off, size).EncodeTo(&s);
  return put_out(s, out, cap, out_len);
}

// table/format.cc:85 IndexValue::EncodeTo (full, or delta against the
// previous handle)
SHIM_API int ref_index_value_encode(uint64_t off, uint64_t size, const char* first_key,
                                    uint32_t first_key_len, int have_first_key, int delta,
                                    uint64_t prev_off, uint64_t prev_size, char* out,
                                    uint64_t cap, uint64_t* out_len) {
  IndexValue v(BlockHandle(off, size), Slice(first_key, first_key_len));
  const BlockHandle prev(prev_off, prev_size);
  std::string s;
  v.EncodeTo(&s, have_first_key != 0, delta ? &prev : nullptr);
  return put_out(s, out, cap, out_len);
}

// table/meta_blocks.cc PropertyBlockBuilder::Add(key, uint64_t) /
// Add(key, string) + Finish.  Entries: [u32 klen][u8 kind 0 = u64, 1 =
// string][u32 vlen][key][8-byte LE value or vlen bytes]
SHIM_API int ref_properties_build(const char* entries, uint32_t n, char* out, uint64_t cap,
                                  uint64_t* out_len) {
  PropertyBlockBuilder b;
  const char* p = entries;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t kl, vl;
    std::memcpy(&kl, p, 4);
    const uint8_t kind = static_cast<uint8_t>(p[4]);
    std::memcpy(&vl, p + 5, 4);
    p += 9;
    const std::string key(p, kl);
    p += kl;
    if (kind == 0) {
      uint64_t v;
      std::memcpy(&v, p, 8);
      b.Add(key, v);
    } else {
      b.Add(key, std::string(p, vl));
    }
    p += vl;
  }
  return put_out(b.Finish(), out, cap, out_len);
}

// table/meta_blocks.cc MetaIndexBuilder::Add(name, BlockHandle) + Finish.
// Entries: [u32 klen][u64 offset][u64 size][key]
SHIM_API int ref_metaindex_build(const char* entries, uint32_t n, char* out, uint64_t cap,
                                 uint64_t* out_len) {
  MetaIndexBuilder b;
  const char* p = entries;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t kl;
    uint64_t off, size;
    std::memcpy(&kl, p, 4);
    std::memcpy(&off, p + 4, 8);
    std::memcpy(&size, p + 12, 8);
    p += 20;
    b.Add(std::string(p, kl), BlockHandle(off, size));
    p += kl;
  }
  return put_out(b.Finish(), out, cap, out_len);
}
