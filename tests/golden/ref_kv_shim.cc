// tests/golden/ref_kv_shim.cc -- TEST INFRASTRUCTURE ONLY (fixture veneer).
//
// C entry points over the REFERENCE's own per-KV protection call sites, compiled
// by tests/golden/gen_kv_golden.py against the reference archive
// (tests/golden/refbuild.py) in a temporary directory and never shipped:
//   * MemTable::Add with memtable_protection_bytes_per_key (db/memtable.cc:696-732)
//     -- the entries are read back through the memtable's own iterator, so their
//     layout and checksum bytes are the reference's -- and the static
//     MemTable::VerifyEntryChecksum (memtable.cc:273-307) on intact and
//     corrupted copies;
//   * WriteBatch reps built with WriteBatch / WriteBatchInternal, parsed by the
//     reference's WriteBatch::Iterate (db/write_batch.cc:477-716) with a handler
//     that does what ProtectionInfoUpdater does (write_batch.cc:3016-3080:
//     ProtectKVO(key, value, op).ProtectC(cf) per data record);
//   * Block::InitializeData/Index/MetaIndexBlockProtectionInfo
//     (table/block_based/block.cc:1113-1235) on blocks cut from the committed
//     reference-written SST fixtures, their kv_checksum_ read with
//     Block::TEST_GetKVChecksum (block.h:274).
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "db/dbformat.h"
#include "db/kv_checksum.h"
#include "db/memtable.h"
#include "db/write_batch_internal.h"
#include "memory/arena.h"
#include "options/cf_options.h"
#include "rocksdb/comparator.h"
#include "rocksdb/options.h"
#include "rocksdb/write_batch.h"
#include "rocksdb/write_buffer_manager.h"
#include "table/block_based/block.h"
#include "table/format.h"
#include "util/coding.h"

using namespace ROCKSDB_NAMESPACE;

#define API extern "C" __attribute__((visibility("default")))

namespace {

uint64_t mix(uint64_t& s) {  // splitmix64
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

std::string rnd_bytes(uint64_t& s, size_t n) {
  std::string r(n, '\0');
  for (size_t i = 0; i < n; ++i) r[i] = static_cast<char>(mix(s) & 0xff);
  return r;
}

// lengths with every XXPH3 length class (0-16, 17-128, 129-240, long, > 1 KiB)
size_t rnd_len(uint64_t& s, size_t cap) {
  static const size_t kEdge[] = {0,   1,   3,   4,   8,   9,   16,   17,   32,  33,
                                 64,  65,  96,  97,  128, 129, 239,  240,  241, 255,
                                 256, 512, 1023, 1024, 1025, 2047, 2048, 3000};
  const uint64_t r = mix(s);
  size_t n = (r & 3) == 0 ? kEdge[(r >> 8) % (sizeof(kEdge) / sizeof(kEdge[0]))] : (r >> 16) % cap;
  return n < cap ? n : cap;
}

void put_msg(char* msg, size_t cap, const Status& st) {
  if (msg && cap) std::snprintf(msg, cap, "%s", st.ToString().c_str());
}

}  // namespace

// ---- MemTable ---------------------------------------------------------------
// Adds n entries (types Put / Delete / SingleDelete / Merge / BlobIndex) to a
// MemTable with protection_bytes_per_key = prot_bytes, then copies every entry
// (varint32 klen .. checksum) in iterator order into out, gap bytes between
// them; offsets[i] = entry i's start.  Returns the entry count, -1 on error.
API int ref_memtable_build(int prot_bytes, int n, unsigned long long seed, char* out, size_t cap,
                           unsigned long long* offsets, size_t* n_bytes) {
  Options opts;
  opts.memtable_protection_bytes_per_key = static_cast<uint32_t>(prot_bytes);
  ImmutableOptions ioptions(opts);
  MutableCFOptions mopts(opts);
  InternalKeyComparator cmp(BytewiseComparator());
  WriteBufferManager wbm(opts.db_write_buffer_size);
  MemTable* mem = new MemTable(cmp, ioptions, mopts, &wbm, kMaxSequenceNumber, 0);
  mem->Ref();
  uint64_t s = seed;
  static const ValueType kTypes[] = {kTypeValue, kTypeDeletion, kTypeSingleDeletion, kTypeMerge,
                                     kTypeBlobIndex};
  for (int i = 0; i < n; ++i) {
    const ValueType t = kTypes[mix(s) % 5];
    std::string key = rnd_bytes(s, rnd_len(s, 300));
    key += std::to_string(i);  // distinct user keys
    const std::string value =
        (t == kTypeDeletion || t == kTypeSingleDeletion) ? std::string() : rnd_bytes(s, rnd_len(s, 4000));
    const SequenceNumber seq = (mix(s) >> 9) + 1;
    Status st = mem->Add(seq, t, key, value, nullptr);
    if (!st.ok()) return -1;
  }
  Arena arena;
  ReadOptions ro;
  InternalIterator* it = mem->NewIterator(ro, &arena);
  size_t pos = 0;
  int k = 0;
  for (it->SeekToFirst(); it->Valid(); it->Next()) {
    const Slice ik = it->key(), v = it->value();
    const char* entry = ik.data() - VarintLength(ik.size());
    const size_t len = static_cast<size_t>(v.data() + v.size() - entry) + prot_bytes;
    pos += mix(s) % 8;  // unaligned starts
    if (pos + len > cap) return -1;
    std::memcpy(out + pos, entry, len);
    offsets[k++] = pos;
    pos += len;
  }
  it->~InternalIterator();
  *n_bytes = pos;
  delete mem->Unref();
  return k;
}

// MemTable::VerifyEntryChecksum(entry, prot_bytes, allow_data_in_errors):
// 1 OK, 0 Corruption (message in msg)
API int ref_memtable_verify(const char* entry, int prot_bytes, int allow_data, char* msg,
                            size_t cap) {
  Status st = MemTable::VerifyEntryChecksum(entry, static_cast<uint32_t>(prot_bytes), allow_data != 0);
  put_msg(msg, cap, st);
  return st.ok() ? 1 : 0;
}

// ---- WriteBatch -------------------------------------------------------------
namespace {
// the records ProtectionInfoUpdater protects (write_batch.cc:3023-3052), with
// the op types it uses
class ProtCollector : public WriteBatch::Handler {
 public:
  std::vector<uint64_t> v;
  Status PutCF(uint32_t cf, const Slice& k, const Slice& x) override { return add(cf, k, x, kTypeValue); }
  Status PutEntityCF(uint32_t cf, const Slice& k, const Slice& e) override {
    return add(cf, k, e, kTypeWideColumnEntity);
  }
  Status DeleteCF(uint32_t cf, const Slice& k) override { return add(cf, k, "", kTypeDeletion); }
  Status SingleDeleteCF(uint32_t cf, const Slice& k) override {
    return add(cf, k, "", kTypeSingleDeletion);
  }
  Status DeleteRangeCF(uint32_t cf, const Slice& b, const Slice& e) override {
    return add(cf, b, e, kTypeRangeDeletion);
  }
  Status MergeCF(uint32_t cf, const Slice& k, const Slice& x) override { return add(cf, k, x, kTypeMerge); }
  Status PutBlobIndexCF(uint32_t cf, const Slice& k, const Slice& x) override {
    return add(cf, k, x, kTypeBlobIndex);
  }
  Status MarkBeginPrepare(bool) override { return Status::OK(); }
  Status MarkEndPrepare(const Slice&) override { return Status::OK(); }
  Status MarkCommit(const Slice&) override { return Status::OK(); }
  Status MarkCommitWithTimestamp(const Slice&, const Slice&) override { return Status::OK(); }
  Status MarkRollback(const Slice&) override { return Status::OK(); }
  Status MarkNoop(bool) override { return Status::OK(); }
  void LogData(const Slice&) override {}

 private:
  Status add(uint32_t cf, const Slice& k, const Slice& x, ValueType op) {
    char b[8];  // Encode(8) = the full value, LE (kv_checksum.h:97-115)
    ProtectionInfo64().ProtectKVO(k, x, op).ProtectC(cf).Encode(8, b);
    v.push_back(DecodeFixed64(b));
    return Status::OK();
  }
};
}  // namespace

// A random WriteBatch of n records (every record kind ReadRecordFromWriteBatch
// parses, default and non-default column families) -> its rep.
API int ref_write_batch_build(int n, unsigned long long seed, char* out, size_t cap, size_t* n_bytes) {
  WriteBatch wb;
  uint64_t s = seed;
  for (int i = 0; i < n; ++i) {
    const uint32_t cf = (mix(s) & 1) ? 0 : static_cast<uint32_t>(mix(s) % 1000);
    const std::string k = rnd_bytes(s, rnd_len(s, 300));
    const std::string v = rnd_bytes(s, rnd_len(s, 3000));
    Status st;
    switch (mix(s) % 12) {
      case 0: case 1: case 2: st = WriteBatchInternal::Put(&wb, cf, k, v); break;
      case 3: st = WriteBatchInternal::Delete(&wb, cf, k); break;
      case 4: st = WriteBatchInternal::SingleDelete(&wb, cf, k); break;
      case 5: st = WriteBatchInternal::DeleteRange(&wb, cf, k, v); break;
      case 6: st = WriteBatchInternal::Merge(&wb, cf, k, v); break;
      case 7: st = WriteBatchInternal::PutBlobIndex(&wb, cf, k, v); break;
      case 8: {
        WideColumns cols{{"a", Slice(v.data(), v.size() / 2)}, {"b", "x"}};
        st = WriteBatchInternal::PutEntity(&wb, cf, k, cols);
        break;
      }
      case 9: st = wb.PutLogData(v); break;
      case 10: st = WriteBatchInternal::InsertNoop(&wb); break;
      default: st = WriteBatchInternal::Put(&wb, cf, Slice(), Slice()); break;
    }
    if (!st.ok()) return -1;
  }
  const std::string& rep = wb.Data();
  if (rep.size() > cap) return -1;
  std::memcpy(out, rep.data(), rep.size());
  *n_bytes = rep.size();
  return static_cast<int>(WriteBatchInternal::Count(&wb));
}

// WriteBatch(rep).Iterate with the collector: the protection values of its
// data records; returns 1 OK / 0 Corruption (msg) and *n_out = values made.
API int ref_write_batch_protect(const char* rep, size_t n, unsigned long long* out, size_t cap,
                                size_t* n_out, char* msg, size_t msg_cap) {
  WriteBatch wb(std::string(rep, n));
  ProtCollector h;
  Status st = wb.Iterate(&h);
  put_msg(msg, msg_cap, st);
  size_t k = 0;
  for (; k < h.v.size() && k < cap; ++k) out[k] = h.v[k];
  *n_out = h.v.size();
  return st.ok() ? 1 : 0;
}

// ---- Block protection -------------------------------------------------------
// kind 0 data, 1 index (value_is_full / has_first_key flags), 2 metaindex:
// the block's kv_checksum_ (num_keys * prot_bytes bytes) into out; returns the
// key count, -1 when the block failed to initialise (size_ error marker).
API long ref_block_kv_checksum(const char* data, size_t n, int kind, int prot_bytes,
                               int value_is_full, int has_first_key, char* out, size_t cap) {
  BlockContents contents(Slice(data, n));
  Block b(std::move(contents));
  if (b.size() == 0) return -1;
  if (kind == 0) {
    b.InitializeDataBlockProtectionInfo(static_cast<uint8_t>(prot_bytes), BytewiseComparator());
  } else if (kind == 1) {
    b.InitializeIndexBlockProtectionInfo(static_cast<uint8_t>(prot_bytes), BytewiseComparator(),
                                         value_is_full != 0, has_first_key != 0);
  } else {
    b.InitializeMetaIndexBlockProtectionInfo(static_cast<uint8_t>(prot_bytes));
  }
  if (b.size() == 0) return -1;
  const char* c = b.TEST_GetKVChecksum();
  size_t keys = 0;
  if (c) {
    // num_keys * prot_bytes bytes: count with the reference's own iterator
    std::unique_ptr<DataBlockIter> dit;
    if (kind == 0) {
      dit.reset(b.NewDataIterator(BytewiseComparator(), kDisableGlobalSequenceNumber));
      for (dit->SeekToFirst(); dit->Valid(); dit->Next()) ++keys;
    } else if (kind == 1) {
      std::unique_ptr<IndexBlockIter> iit(b.NewIndexIterator(
          BytewiseComparator(), kDisableGlobalSequenceNumber, nullptr, nullptr, true,
          has_first_key != 0, false, value_is_full != 0));
      for (iit->SeekToFirst(); iit->Valid(); iit->Next()) ++keys;
    } else {
      std::unique_ptr<MetaBlockIter> mit(b.NewMetaIterator());
      for (mit->SeekToFirst(); mit->Valid(); mit->Next()) ++keys;
    }
    if (keys * prot_bytes > cap) return -1;
    std::memcpy(out, c, keys * prot_bytes);
  }
  return static_cast<long>(keys);
}
