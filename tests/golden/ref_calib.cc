// tests/golden/ref_calib.cc -- TEST INFRASTRUCTURE ONLY (CPU-baseline calibration).
//
// A batch loop over the reference's own table/format.cc:594
// ComputeBuiltinChecksumWithLastByte, one std::thread per contiguous range of
// blocks, shaped like oracle_block_checksum_batch so tools/calibrate_cpu.py can
// time the port (oracle/oracle.c) against the compiled reference on the same
// blocks.  Built with ref_shim.cc into a temporary directory outside the
// repository; never committed as a binary, never shipped to the GPU box.

#include <cstdint>
#include <thread>
#include <vector>

#include "rocksdb/table.h"
#include "table/format.h"

using namespace ROCKSDB_NAMESPACE;

extern "C" __attribute__((visibility("default"))) void ref_block_checksum_batch(
    int type, const char* base, const uint64_t* offsets, const uint32_t* sizes,
    const uint8_t* last_bytes, uint64_t n, int nthreads, uint32_t* out) {
  auto run = [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i)
      out[i] = ComputeBuiltinChecksumWithLastByte(static_cast<ChecksumType>(type),
                                                  base + offsets[i], sizes[i],
                                                  static_cast<char>(last_bytes[i]));
  };
  if (nthreads <= 1) {
    run(0, n);
    return;
  }
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back(run, n * t / nthreads, n * (t + 1) / nthreads);
  for (auto& t : ts) t.join();
}
