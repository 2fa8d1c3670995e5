// tests/cpp/shim_selftest.cc -- exercises the C++ host shim
// (include/forst/checksum_engine.h) the way a ForSt call site would.
//   shim_selftest pure   host-only helpers (no GPU)
//   shim_selftest gpu    BlockChecksumEngine write/verify on a real MI355X
//   shim_selftest wal    WalWriteGroup framing + WalRecovery round trip
//   shim_selftest threads  4 host threads, one HIP stream each, interleaving
//                        write-side, verify, WAL and raw-hash calls against
//                        the engine's shared per-device scratch pool
// Prints PASS or FAIL lines; exit code 0 iff all passed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "forst/checksum_engine.h"

using namespace forst_gpu;

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

// One thread's private inputs: an SST-packed batch and a WAL image.
struct Work {
  int n = 0;
  uint64_t total = 0;
  std::vector<uint64_t> offs;
  std::vector<uint32_t> sizes;
  uint8_t *d_base = nullptr, *d_types = nullptr, *d_log = nullptr;
  uint64_t *d_offs = nullptr, *d_hoffs = nullptr, *d_h64 = nullptr;
  uint32_t *d_sizes = nullptr, *d_out = nullptr, *d_comp = nullptr, *d_crc = nullptr;
  uint8_t *d_ok = nullptr, *d_st = nullptr;
  uint32_t *d_nrec = nullptr, *d_fail = nullptr;
  unsigned long long* d_bad = nullptr;
  uint64_t log_len = 0, n_phys = 0, n_lblocks = 0;
  // expected results (single-threaded pass)
  std::vector<uint32_t> want_out, want_crc;
  std::vector<uint64_t> want_h64;
};

static bool setup_work(Work& w, int seed) {
  bool ok = true;
  w.n = 3000;
  w.offs.resize(w.n);
  w.sizes.resize(w.n);
  for (int i = 0; i < w.n; ++i) {
    w.sizes[i] = ((i + seed) * 2654435761u) % 20000;
    w.offs[i] = w.total;
    w.total += w.sizes[i] + 5;
  }
  ok &= hipMalloc(&w.d_base, w.total + 256) == hipSuccess;
  ok &= hipMalloc(&w.d_offs, w.n * 8) == hipSuccess;
  ok &= hipMalloc(&w.d_sizes, w.n * 4) == hipSuccess;
  ok &= hipMalloc(&w.d_types, w.n) == hipSuccess;
  ok &= hipMalloc(&w.d_out, w.n * 4) == hipSuccess;
  ok &= hipMalloc(&w.d_comp, w.n * 4) == hipSuccess;
  ok &= hipMalloc(&w.d_ok, w.n) == hipSuccess;
  ok &= hipMalloc(&w.d_h64, w.n * 8) == hipSuccess;
  ok &= hipMemcpy(w.d_offs, w.offs.data(), w.n * 8, hipMemcpyHostToDevice) == hipSuccess;
  ok &= hipMemcpy(w.d_sizes, w.sizes.data(), w.n * 4, hipMemcpyHostToDevice) == hipSuccess;
  ok &= hipMemset(w.d_types, 1, w.n) == hipSuccess;
  ok &= forst_fill_stream(w.d_base, 0, w.total, 1000 + seed, nullptr) == FORST_OK;
  // WAL image (db/log_writer.cc layout from forst_wal_layout, payload from
  // the splitmix stream, zero-filled block tails, CRCs by the writer kernel)
  std::vector<uint32_t> lens(2000);
  for (size_t i = 0; i < lens.size(); ++i) lens[i] = ((i + seed) * 40503u) % 40000;
  uint64_t np = 0, npad = 0, tot = 0;
  ok &= forst_wal_layout(lens.data(), lens.size(), 0, nullptr, nullptr, nullptr, 0, nullptr,
                         nullptr, 0, &np, &npad, &tot) == FORST_OK;
  std::vector<uint64_t> ho(np), po(npad + 1);
  std::vector<uint32_t> hl(np), pl(npad + 1);
  std::vector<uint8_t> ht(np);
  ok &= forst_wal_layout(lens.data(), lens.size(), 0, ho.data(), hl.data(), ht.data(), np,
                         po.data(), pl.data(), npad, &np, &npad, &tot) == FORST_OK;
  w.log_len = tot;
  w.n_phys = np;
  w.n_lblocks = (tot + 32767) / 32768;
  ok &= hipMalloc(&w.d_log, tot + 256) == hipSuccess;
  ok &= forst_fill_stream(w.d_log, 0, tot, 2000 + seed, nullptr) == FORST_OK;
  std::vector<uint8_t> img(tot);
  ok &= hipMemcpy(img.data(), w.d_log, tot, hipMemcpyDeviceToHost) == hipSuccess;
  for (uint64_t i = 0; i < np; ++i) {
    img[ho[i] + 4] = static_cast<uint8_t>(hl[i]);
    img[ho[i] + 5] = static_cast<uint8_t>(hl[i] >> 8);
    img[ho[i] + 6] = ht[i];
  }
  for (uint64_t i = 0; i < npad; ++i) std::memset(img.data() + po[i], 0, pl[i]);
  ok &= hipMemcpy(w.d_log, img.data(), tot, hipMemcpyHostToDevice) == hipSuccess;
  ok &= hipMalloc(&w.d_hoffs, np * 8) == hipSuccess;
  ok &= hipMemcpy(w.d_hoffs, ho.data(), np * 8, hipMemcpyHostToDevice) == hipSuccess;
  ok &= hipMalloc(&w.d_crc, np * 4) == hipSuccess;
  ok &= hipMalloc(&w.d_st, w.n_lblocks) == hipSuccess;
  ok &= hipMalloc(&w.d_nrec, w.n_lblocks * 4) == hipSuccess;
  ok &= hipMalloc(&w.d_fail, w.n_lblocks * 4) == hipSuccess;
  ok &= hipMalloc(&w.d_bad, 8) == hipSuccess;
  return ok;
}

// one round of every kind of call on `stream`; results compared with the
// expected ones when `check`, recorded as expected otherwise
static bool round_of_calls(Work& w, void* stream, bool check) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  bool ok = true;
  ok &= forst_block_trailer_batch(kCRC32c, w.d_base, w.total, w.d_offs, w.d_sizes, w.d_types,
                                  nullptr, w.d_out, w.n, stream) == FORST_OK;
  ok &= hipMemsetAsync(w.d_bad, 0, 8, st) == hipSuccess;
  ok &= forst_block_verify_batch(kCRC32c, w.d_base, w.total, w.d_offs, w.d_sizes, nullptr,
                                 w.d_comp, nullptr, w.d_ok, w.d_bad, w.n, stream) == FORST_OK;
  ok &= forst_wal_record_crc_batch(w.d_log, w.log_len, w.d_hoffs, w.n_phys, 1, w.d_crc,
                                   stream) == FORST_OK;
  unsigned long long bad_blocks = 0;
  ok &= hipMemsetAsync(w.d_bad, 0, 8, st) == hipSuccess;
  ok &= forst_xxh3_64_batch(w.d_base, w.total, w.d_offs, w.d_sizes, w.d_h64, w.n, stream) ==
        FORST_OK;
  // (synchronises its stream once: the record total sizes the descriptors)
  ok &= forst_wal_verify_batch(w.d_log, w.log_len, 0, w.n_lblocks, 0, w.d_st, w.d_nrec,
                               w.d_fail, w.d_bad, stream) == FORST_OK;
  std::vector<uint32_t> out(w.n), comp(w.n), crc(w.n_phys), nrec(w.n_lblocks);
  std::vector<uint64_t> h64(w.n);
  std::vector<uint8_t> okv(w.n);
  ok &= hipMemcpyAsync(out.data(), w.d_out, w.n * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok &= hipMemcpyAsync(comp.data(), w.d_comp, w.n * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok &= hipMemcpyAsync(okv.data(), w.d_ok, w.n, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok &= hipMemcpyAsync(crc.data(), w.d_crc, w.n_phys * 4, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok &= hipMemcpyAsync(h64.data(), w.d_h64, w.n * 8, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok &= hipMemcpyAsync(nrec.data(), w.d_nrec, w.n_lblocks * 4, hipMemcpyDeviceToHost, st) ==
        hipSuccess;
  ok &= hipMemcpyAsync(&bad_blocks, w.d_bad, 8, hipMemcpyDeviceToHost, st) == hipSuccess;
  ok &= hipStreamSynchronize(st) == hipSuccess;
  if (!ok) return false;
  for (int i = 0; i < w.n; ++i) ok &= okv[i] == 1 && comp[i] == out[i];
  uint64_t recs = 0;
  for (uint32_t r : nrec) recs += r;
  ok &= recs == w.n_phys && bad_blocks == 0;
  if (!check) {
    w.want_out = out;
    w.want_crc = crc;
    w.want_h64 = h64;
    return ok;
  }
  return ok && out == w.want_out && crc == w.want_crc && h64 == w.want_h64;
}

static void threads() {
  constexpr int kThreads = 4, kRounds = 12;
  std::vector<Work> work(kThreads);
  for (int t = 0; t < kThreads; ++t) CHECK(setup_work(work[t], t));
  for (int t = 0; t < kThreads; ++t) CHECK(round_of_calls(work[t], nullptr, false));
  std::atomic<int> failures{0};
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      hipStream_t s;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        ++failures;
        return;
      }
      for (int r = 0; r < kRounds; ++r)
        if (!round_of_calls(work[t], s, true)) ++failures;
      (void)hipStreamDestroy(s);
    });
  }
  for (auto& x : th) x.join();
  CHECK(failures.load() == 0);
  std::printf("threads: %d x %d rounds, failures %d\n", kThreads, kRounds, failures.load());
}

// WalWriteGroup (log::Writer::AddRecord for a write group) and WalRecovery
// (RecoverLogFiles' ReadRecord loop) round trip: groups framed one after the
// other from the writer's block offset make the log the serial writer would
// (every CRC restated here bytewise); recovery hands back every record's
// bytes in order with no reports; a flipped payload byte gives the reader's
// "checksum mismatch" report right before the next record it returns.
static void wal(bool recyclable) {
  const uint32_t log_number = 0x51u;
  std::vector<std::string> recs;
  for (int i = 0; i < 700; ++i) {
    size_t n = (static_cast<size_t>(i) * 2654435761u) % (i % 50 == 0 ? 90000 : 9000);
    if (i % 97 == 3) n = 0;
    std::string r(n, '\0');
    for (size_t k = 0; k < n; ++k) r[k] = static_cast<char>((k * 131 + i * 7) & 0xff);
    recs.push_back(r);
  }
  std::string log;
  uint32_t bo = 0;
  size_t i0 = 0;
  uint64_t n_phys = 0;
  const uint32_t hs = recyclable ? 11 : 7;
  WalWriteGroup g(recyclable, log_number);
  while (i0 < recs.size()) {  // write groups of 1..37 records
    const size_t i1 = std::min(recs.size(), i0 + 1 + (i0 * 7) % 37);
    std::vector<ByteRange> grp;
    for (size_t i = i0; i < i1; ++i) grp.push_back({recs[i].data(), recs[i].size()});
    CHECK(g.Frame(grp, bo).ok());
    log.append(g.data(), g.size());
    bo = g.end_block_offset();
    n_phys += g.physical_records();
    i0 = i1;
  }
  CHECK(bo == (log.size() % 32768 ? log.size() % 32768 : (log.empty() ? 0 : 32768)) ||
        (log.size() % 32768 == 0 && bo == 0));
  // every physical record: header CRC = Mask(crc32c(header[6..hs) || payload))
  uint64_t p = 0, seen = 0;
  bool crc_ok = true;
  while (p + hs <= log.size()) {
    if (32768 - p % 32768 < hs) {
      p += 32768 - p % 32768;
      continue;
    }
    const uint8_t* h = reinterpret_cast<const uint8_t*>(log.data() + p);
    const uint32_t n = h[4] | (h[5] << 8);
    uint32_t stored;
    std::memcpy(&stored, h, 4);
    crc_ok &= crc32c::Mask(crc32c_ref(h + 6, hs - 6 + n)) == stored;
    if (recyclable) {
      uint32_t ln;
      std::memcpy(&ln, h + 7, 4);
      crc_ok &= ln == log_number;
    }
    p += hs + n;
    ++seen;
  }
  CHECK(crc_ok);
  CHECK(seen == n_phys && p == log.size());
  uint8_t* d_log = nullptr;
  CHECK(hipMalloc(&d_log, log.size() + 256) == hipSuccess);
  CHECK(hipMemcpy(d_log, log.data(), log.size(), hipMemcpyHostToDevice) == hipSuccess);
  const uint8_t* host = reinterpret_cast<const uint8_t*>(log.data());
  WalRecovery rec;
  CHECK(rec.Recover(d_log, host, log.size(), log_number, 2 /*kPointInTimeRecovery*/).ok());
  WalRecord r;
  size_t k = 0;
  bool same = true;
  while (rec.Next(&r)) {
    same &= k < recs.size() && r.size == recs[k].size() &&
            std::memcmp(r.data, recs[k].data(), r.size) == 0 && r.reports_before.empty();
    ++k;
  }
  CHECK(rec.status().ok());
  CHECK(same && k == recs.size());
  CHECK(rec.trailing_reports().empty());
  // a flipped payload byte in record 300 (the reader drops the rest of its block)
  uint64_t off300 = 0;
  {
    WalRecovery r2;
    CHECK(r2.Recover(d_log, host, log.size(), log_number, 2).ok());
    for (int j = 0; j <= 300 && r2.Next(&r); ++j) off300 = r.offset;
  }
  std::string bad = log;
  const uint64_t flip = off300 + (32768 - off300 % 32768 < hs ? 32768 - off300 % 32768 : 0) + hs;
  bad[flip] ^= 0x04;
  CHECK(hipMemcpy(d_log, bad.data(), bad.size(), hipMemcpyHostToDevice) == hipSuccess);
  const uint8_t* bhost = reinterpret_cast<const uint8_t*>(bad.data());
  CHECK(rec.Recover(d_log, bhost, bad.size(), log_number, 2).ok());
  k = 0;
  same = true;
  bool reported = false;
  while (rec.Next(&r)) {
    if (r.offset < off300) {
      same &= r.size == recs[k].size() && std::memcmp(r.data, recs[k].data(), r.size) == 0;
      ++k;
    } else if (!r.reports_before.empty() && !reported) {
      reported = r.reports_before[0].Text() == "checksum mismatch" &&
                 r.reports_before[0].offset <= flip;
    }
  }
  CHECK(same && k == 300);
  CHECK(reported);
  CHECK(rec.result().n_reports >= 1);
  std::printf("wal%s: %zu records, %llu physical, %zu log bytes\n", recyclable ? " (recyclable)" : "",
              recs.size(), static_cast<unsigned long long>(n_phys), log.size());
  (void)hipFree(d_log);
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "pure";
  pure();
  if (mode == "gpu") gpu();
  if (mode == "threads") threads();
  if (mode == "wal") {
    wal(false);
    wal(true);
  }
  std::printf(g_fail ? "FAIL (%d)\n" : "PASS\n", g_fail);
  return g_fail ? 1 : 0;
}
