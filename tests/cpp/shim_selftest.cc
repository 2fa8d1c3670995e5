// tests/cpp/shim_selftest.cc -- exercises the C++ host shim
// (include/forst/checksum_engine.h) the way a ForSt call site would.
//   shim_selftest pure   host-only helpers (no GPU)
//   shim_selftest gpu    BlockChecksumEngine write/verify on a real MI355X
// Prints PASS or FAIL lines; exit code 0 iff all passed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "forst/checksum_engine.h"

using namespace forstdb;

static int g_fail = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

// test-only bytewise CRC32C (for expected values)
static uint32_t crc32c_ref(const uint8_t* p, size_t n) {
  uint32_t c = ~0u;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
  }
  return ~c;
}

static void pure() {
  // util/crc32c_test.cc:121-127
  uint32_t crc = crc32c_ref(reinterpret_cast<const uint8_t*>("foo"), 3);
  CHECK(crc != crc32c::Mask(crc));
  CHECK(crc == crc32c::Unmask(crc32c::Mask(crc)));
  CHECK(crc == crc32c::Unmask(crc32c::Unmask(crc32c::Mask(crc32c::Mask(crc)))));
  // util/crc32c_test.cc:128-142
  const uint32_t c1 = crc32c_ref(reinterpret_cast<const uint8_t*>("hello "), 6);
  const uint32_t c2 = crc32c_ref(reinterpret_cast<const uint8_t*>("world"), 5);
  const uint32_t c3 = crc32c_ref(reinterpret_cast<const uint8_t*>("hello world"), 11);
  CHECK(crc32c::Crc32cCombine(c1, c2, 5) == c3);
  CHECK(crc32c::Crc32cCombine(c2, c1, 6) != c3);
  // table/format.h:119
  CHECK(ChecksumModifierForContext(0, 12345) == 0);
  CHECK(ChecksumModifierForContext(7, 0x100000001ull) == (7u ^ 2u));
  CHECK(IsSupportedChecksumType(kXXH3));
  CHECK(!IsSupportedChecksumType(static_cast<ChecksumType>(5)));
  CHECK(GpuSupportsChecksumType(kCRC32c) && GpuSupportsChecksumType(kxxHash) &&
        GpuSupportsChecksumType(kxxHash64) &&
        !GpuSupportsChecksumType(static_cast<ChecksumType>(5)));
  // reader_common.cc:55-60 exact format
  Status s = Status::Corruption(
      BlockChecksumMismatchMessage(kCRC32c, 1, 2, false, "f.sst", 7, 4096));
  CHECK(s.ToString() ==
        "Corruption: block checksum mismatch: stored = 1, computed = 2, type = 1  in f.sst "
        "offset 7 size 4096");
  Status s2 = Status::Corruption(
      BlockChecksumMismatchMessage(kXXH3, 3, 4, true, "x", 0, 0));
  CHECK(s2.ToString() ==
        "Corruption: block checksum mismatch: stored(context removed) = 3, computed = 4, "
        "type = 4  in x offset 0 size 0");
}

static void gpu() {
  const int n = 1000;
  std::vector<uint64_t> offs(n);
  std::vector<uint32_t> sizes(n);
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    sizes[i] = (i * 2654435761u) % 9000;
    offs[i] = total;
    total += sizes[i] + 5;
  }
  uint8_t* d_base;
  uint64_t* d_offs;
  uint32_t* d_sizes;
  uint8_t* d_types;
  CHECK(hipMalloc(&d_base, total + 256) == hipSuccess);
  CHECK(hipMalloc(&d_offs, n * 8) == hipSuccess);
  CHECK(hipMalloc(&d_sizes, n * 4) == hipSuccess);
  CHECK(hipMalloc(&d_types, n) == hipSuccess);
  CHECK(hipMemcpy(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(hipMemcpy(d_sizes, sizes.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(hipMemset(d_types, 0, n) == hipSuccess);
  CHECK(forst_fill_stream(d_base, 0, total, 42, nullptr) == FORST_OK);
  for (ChecksumType t : {kCRC32c, kXXH3}) {
    BlockChecksumEngine eng;
    DeviceBlockBatch b{d_base, total, d_offs, d_sizes, static_cast<uint64_t>(n)};
    CHECK(eng.WriteTrailers(t, b, d_types, nullptr, nullptr).ok());
    std::vector<uint64_t> file_offsets(offs.begin(), offs.end());
    std::vector<uint64_t> failed;
    Status s = eng.VerifyBlocks(t, 0, b, "000042.sst", file_offsets, &failed);
    CHECK(s.ok());
    CHECK(failed.empty());
    // corrupt one payload byte of block 500
    const int v = 500;
    uint8_t byte;
    CHECK(hipMemcpy(&byte, d_base + offs[v], 1, hipMemcpyDeviceToHost) == hipSuccess);
    byte ^= 0x20;
    CHECK(hipMemcpy(d_base + offs[v], &byte, 1, hipMemcpyHostToDevice) == hipSuccess);
    s = eng.VerifyBlocks(t, 0, b, "000042.sst", file_offsets, &failed);
    CHECK(s.IsCorruption());
    CHECK(failed.size() == 1 && failed[0] == static_cast<uint64_t>(v));
    if (t == kCRC32c) {
      std::vector<uint8_t> blk(sizes[v] + 5);
      CHECK(hipMemcpy(blk.data(), d_base + offs[v], blk.size(), hipMemcpyDeviceToHost) ==
            hipSuccess);
      uint32_t stored;
      std::memcpy(&stored, blk.data() + sizes[v] + 1, 4);
      const uint32_t computed = crc32c_ref(blk.data(), sizes[v] + 1);
      const std::string want =
          "Corruption: block checksum mismatch: stored = " +
          std::to_string(crc32c::Unmask(stored)) + ", computed = " + std::to_string(computed) +
          ", type = 1  in 000042.sst offset " + std::to_string(offs[v]) + " size " +
          std::to_string(sizes[v]);
      CHECK(s.ToString() == want);
      if (s.ToString() != want) std::printf("got  %s\nwant %s\n", s.ToString().c_str(), want.c_str());
    }
    CHECK(eng.stats().block_checksum_mismatch_count == 1);
    byte ^= 0x20;
    CHECK(hipMemcpy(d_base + offs[v], &byte, 1, hipMemcpyHostToDevice) == hipSuccess);
  }
  // unsupported / unknown types behave like the reference selector
  BlockChecksumEngine eng;
  DeviceBlockBatch b{d_base, total, d_offs, d_sizes, static_cast<uint64_t>(n)};
  std::vector<uint64_t> fo(offs.begin(), offs.end());
  Status bad = eng.VerifyBlocks(static_cast<ChecksumType>(123), 0, b, "in test", fo);
  CHECK(bad.ToString() == "Corruption: Corrupt or unsupported checksum type: 123");
  (void)hipFree(d_base);
  (void)hipFree(d_offs);
  (void)hipFree(d_sizes);
  (void)hipFree(d_types);
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "pure";
  pure();
  if (mode == "gpu") gpu();
  std::printf(g_fail ? "FAIL (%d)\n" : "PASS\n", g_fail);
  return g_fail ? 1 : 0;
}
