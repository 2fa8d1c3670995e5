// tests/golden/ref_sstwriter_shim.cc -- TEST INFRASTRUCTURE ONLY (fixture veneer).
//
// C entry points over the REFERENCE's own SstFileWriter / BlockBasedTableBuilder
// (table/sst_file_writer.cc, table/block_based/block_based_table_builder.cc) and
// SstFileReader::VerifyChecksum (table/sst_file_reader.cc ->
// BlockBasedTable::VerifyChecksum, block_based_table_reader.cc:2457), compiled by
// tests/golden/gen_sst_golden.py against the reference archive
// (tests/golden/refbuild.py) in a temporary directory and never shipped.
// The files they write -- block order, filter / index partitions, compressed
// data and index blocks, range deletions, compression dictionary, properties,
// metaindex and footer all decided by the reference builder -- are committed as
// fixtures, with the Status the reference's own VerifyChecksum returns for
// corrupted copies.
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "rocksdb/env.h"
#include "rocksdb/filter_policy.h"
#include "rocksdb/options.h"
#include "rocksdb/sst_file_reader.h"
#include "rocksdb/sst_file_writer.h"
#include "rocksdb/table.h"

using namespace ROCKSDB_NAMESPACE;

namespace {

uint64_t mix(uint64_t& s) {  // splitmix64
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

void put_err(char* err, size_t cap, const Status& s) {
  std::snprintf(err, cap, "%s", s.ToString().c_str());
}

}  // namespace

// filter: 0 none, 1 full bloom, 2 partitioned bloom (needs index_type 2)
extern "C" __attribute__((visibility("default"))) int ref_sst_write(
    const char* path, int format_version, int checksum, int index_type, int filter,
    int compression, int index_compression, int block_size, int restart_interval, int n_keys,
    int value_len, unsigned long long seed, int range_dels, int dict_bytes, char* err,
    size_t err_cap) {
  Options options;
  options.compression = static_cast<CompressionType>(compression);
  options.db_host_id = "";  // no host name in the fixture's properties
  if (dict_bytes) {
    options.compression_opts.max_dict_bytes = dict_bytes;
    options.compression_opts.zstd_max_train_bytes = 0;
  }
  BlockBasedTableOptions t;
  t.checksum = static_cast<ChecksumType>(checksum);
  t.format_version = static_cast<uint32_t>(format_version);
  t.index_type = static_cast<BlockBasedTableOptions::IndexType>(index_type);
  t.enable_index_compression = index_compression != 0;
  t.block_size = static_cast<size_t>(block_size);
  t.block_restart_interval = restart_interval;
  t.metadata_block_size = 512;  // several index / filter partitions in a small file
  if (filter) {
    t.filter_policy.reset(NewBloomFilterPolicy(10));
    t.partition_filters = filter == 2;
  }
  options.table_factory.reset(NewBlockBasedTableFactory(t));
  SstFileWriter w(EnvOptions(), options);
  Status s = w.Open(path);
  uint64_t st = seed;
  // compressible values: words from a small vocabulary
  static const char* kWords[] = {"state", "flink", "window", "checkpoint", "operator",
                                 "keyed", "timer", "value", "list", "map"};
  char key[64];
  for (int i = 0; s.ok() && i < n_keys; ++i) {
    std::snprintf(key, sizeof(key), "key%010d", i * 3);
    std::string v;
    while (static_cast<int>(v.size()) < value_len) {
      v += kWords[mix(st) % 10];
      v.push_back(static_cast<char>('0' + mix(st) % 10));
    }
    v.resize(value_len);
    s = w.Put(key, v);
  }
  for (int r = 0; s.ok() && r < range_dels; ++r) {
    char b[32], e[32];
    std::snprintf(b, sizeof(b), "key%010d", r * 7);
    std::snprintf(e, sizeof(e), "key%010d", r * 7 + 5);
    s = w.DeleteRange(b, e);
  }
  if (s.ok()) s = w.Finish();
  if (!s.ok()) {
    put_err(err, err_cap, s);
    return 1;
  }
  return 0;
}

// SstFileReader::Open + VerifyChecksum: the reference's Status text
extern "C" __attribute__((visibility("default"))) int ref_sst_verify(const char* path, char* msg,
                                                                    size_t cap) {
  Options options;
  SstFileReader r(options);
  Status s = r.Open(path);
  if (s.ok()) s = r.VerifyChecksum();
  std::snprintf(msg, cap, "%s", s.ToString().c_str());
  return s.ok() ? 0 : 1;
}
