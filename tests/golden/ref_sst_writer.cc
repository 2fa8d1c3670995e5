// tests/golden/ref_sst_writer.cc -- TEST INFRASTRUCTURE ONLY (fixture maker).
//
// Writes one SST file with the REFERENCE's own writer (SstFileWriter ->
// BlockBasedTableBuilder, table/block_based/block_based_table_builder.cc), so
// the committed fixtures carry reference-produced bytes: every block trailer
// (WriteMaybeCompressedBlock :1311-1360), the index / metaindex / properties
// blocks and the footer (FooterBuilder::Build, table/format.cc:231-330).
// Built transiently by tests/golden/gen_sst_fixtures.py against reference
// objects compiled in a temporary directory; nothing of it is committed
// except the SST files it writes.
//
// usage: ref_sst_writer <out.sst> <format_version> <checksum> <index_type>
//                       <n_keys> <value_len> <block_size> <seed> [align]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "rocksdb/env.h"
#include "rocksdb/options.h"
#include "rocksdb/sst_file_writer.h"
#include "rocksdb/table.h"

using namespace ROCKSDB_NAMESPACE;

static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  if (argc < 9) {
    std::fprintf(stderr, "usage: %s out fv checksum index_type n value_len block_size seed [align]\n",
                 argv[0]);
    return 2;
  }
  const std::string out = argv[1];
  BlockBasedTableOptions t;
  t.format_version = static_cast<uint32_t>(std::atoi(argv[2]));
  t.checksum = static_cast<ChecksumType>(std::atoi(argv[3]));
  t.index_type = static_cast<BlockBasedTableOptions::IndexType>(std::atoi(argv[4]));
  const long n = std::atol(argv[5]);
  const long vlen = std::atol(argv[6]);
  t.block_size = static_cast<size_t>(std::atol(argv[7]));
  uint64_t seed = std::strtoull(argv[8], nullptr, 0);
  if (argc > 9 && std::atoi(argv[9])) t.block_align = true;
  if (t.index_type == BlockBasedTableOptions::kTwoLevelIndexSearch) t.metadata_block_size = 1024;
  Options opt;
  opt.compression = kNoCompression;
  opt.table_factory.reset(NewBlockBasedTableFactory(t));
  SstFileWriter w(EnvOptions(), opt);
  Status s = w.Open(out);
  char key[32];
  std::string val;
  for (long i = 0; s.ok() && i < n; ++i) {
    std::snprintf(key, sizeof(key), "key%012ld", i);
    const long len = vlen > 0 ? (vlen / 2 + static_cast<long>(splitmix(seed) % vlen)) : 0;
    val.resize(static_cast<size_t>(len));
    for (long k = 0; k < len; k += 8) {
      const uint64_t r = splitmix(seed);
      for (long j = 0; j < 8 && k + j < len; ++j) val[k + j] = static_cast<char>(r >> (8 * j));
    }
    s = w.Put(key, val);
  }
  if (s.ok()) s = w.Finish();
  if (!s.ok()) {
    std::fprintf(stderr, "%s\n", s.ToString().c_str());
    return 1;
  }
  return 0;
}
