/* oracle/oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ForSt's block-checksum hot path.  It is the parity oracle
 * for the HIP engine in forst_amd/ and, compiled at x86-64-v3 with the same
 * instruction classes the reference picks at compile time, the "port" CPU
 * baseline timed by bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it.  The product never does.
 *
 * Parity: pinned by the reference's own known-answer tests
 * (table/table_test.cc:2312-2398, util/crc32c_test.cc:26-110) and by golden
 * vectors under tests/golden/ -- see tests/test_oracle_golden.py.
 *
 * Reference = ForSt (RocksDB 8.10.0 fork); file:line cited per function.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <nmmintrin.h>
#include <wmmintrin.h>
#define OR_HAVE_X86 1
#endif

/* ======================================================================== */
/* CRC32C                                                                    */
/* ======================================================================== */

/* Castagnoli polynomial, reflected (util/crc32c.cc:1198 uses 0x82f63b78). */
#define CRC32C_POLY 0x82F63B78u

static uint32_t g_crc_tab[8][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* reflected multiply-by-x modulo P */
static inline uint32_t gf_mulx(uint32_t v) {
  return (v >> 1) ^ ((v & 1u) ? CRC32C_POLY : 0u);
}
/* reflected GF(2)[x]/P product; bit 31 is the x^0 coefficient
 * (same algebra as gf_multiply_sw, util/crc32c.cc:1143) */
static uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 0; i < 32; i++) {
    if (a & (0x80000000u >> i)) r ^= b;
    b = gf_mulx(b);
  }
  return r;
}
/* x^e mod P, reflected, square-and-multiply (util/crc32c.cc:1200-1230) */
static uint32_t gf_xpow(uint64_t e) {
  uint32_t result = 0x80000000u; /* 1 */
  uint32_t sq = 0x40000000u;     /* x */
  while (e) {
    if (e & 1) result = gf_mul(result, sq);
    sq = gf_mul(sq, sq);
    e >>= 1;
  }
  return result;
}

#ifdef OR_HAVE_X86
/* clmul shift constants for the 3-way fast path: shift(c, L) =
 * crc32_u64(0, clmul(c, x^(8L-33))) -- the algebra of CombineCRC,
 * util/crc32c.cc:545-562. */
#define OR_BLK_LARGE 1024
#define OR_BLK_SMALL 128
static uint64_t g_k_large1, g_k_large2, g_k_small1, g_k_small2;
#endif

static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ CRC32C_POLY : c >> 1;
    g_crc_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++)
    for (int t = 1; t < 8; t++)
      g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^
                        g_crc_tab[0][g_crc_tab[t - 1][i] & 0xff];
#ifdef OR_HAVE_X86
  g_k_large1 = gf_xpow(8ull * OR_BLK_LARGE - 33);
  g_k_large2 = gf_xpow(16ull * OR_BLK_LARGE - 33);
  g_k_small1 = gf_xpow(8ull * OR_BLK_SMALL - 33);
  g_k_small2 = gf_xpow(16ull * OR_BLK_SMALL - 33);
#endif
}
static inline void crc_once(void) { pthread_once(&g_once, crc_init); }

static inline uint64_t ld64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static inline uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

/* Raw (no pre/post inversion) slicing-by-8 update: the portable
 * ExtendImpl<DefaultCRC32> family, util/crc32c.cc:252-315. */
static uint32_t crc_raw_update(uint32_t c, const uint8_t* p, size_t n) {
  while (n && ((uintptr_t)p & 7)) {
    c = g_crc_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    n--;
  }
  while (n >= 8) {
    uint64_t w = ld64(p);
    uint32_t lo = c ^ (uint32_t)w, hi = (uint32_t)(w >> 32);
    c = g_crc_tab[7][lo & 0xff] ^ g_crc_tab[6][(lo >> 8) & 0xff] ^
        g_crc_tab[5][(lo >> 16) & 0xff] ^ g_crc_tab[4][lo >> 24] ^
        g_crc_tab[3][hi & 0xff] ^ g_crc_tab[2][(hi >> 8) & 0xff] ^
        g_crc_tab[1][(hi >> 16) & 0xff] ^ g_crc_tab[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_crc_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c;
}

/* util/crc32c.cc:1133 crc32c::Extend -- portable restatement */
uint32_t oracle_crc32c_extend(uint32_t crc, const void* p, size_t n) {
  crc_once();
  return ~crc_raw_update(~crc, (const uint8_t*)p, n);
}

#ifdef OR_HAVE_X86
static inline uint32_t clmul_shift(uint32_t c, uint64_t k) {
  __m128i a = _mm_cvtsi32_si128((int)c);
  __m128i b = _mm_cvtsi64_si128((long long)k);
  uint64_t prod = (uint64_t)_mm_cvtsi128_si64(_mm_clmulepi64_si128(a, b, 0));
  return (uint32_t)_mm_crc32_u64(0, prod);
}
/* three interleaved SSE4.2 crc32q streams + clmul recombination: the same
 * instruction classes as crc32c_3way, util/crc32c.cc:572-1103. */
static uint32_t crc_raw_update_fast(uint32_t c, const uint8_t* p, size_t n) {
  while (n && ((uintptr_t)p & 7)) {
    c = _mm_crc32_u8(c, *p++);
    n--;
  }
  while (n >= 3 * OR_BLK_LARGE) {
    uint64_t c0 = c, c1 = 0, c2 = 0;
    const uint8_t* q1 = p + OR_BLK_LARGE;
    const uint8_t* q2 = p + 2 * OR_BLK_LARGE;
    for (int i = 0; i < OR_BLK_LARGE; i += 8) {
      c0 = _mm_crc32_u64(c0, ld64(p + i));
      c1 = _mm_crc32_u64(c1, ld64(q1 + i));
      c2 = _mm_crc32_u64(c2, ld64(q2 + i));
    }
    c = clmul_shift((uint32_t)c0, g_k_large2) ^
        clmul_shift((uint32_t)c1, g_k_large1) ^ (uint32_t)c2;
    p += 3 * OR_BLK_LARGE;
    n -= 3 * OR_BLK_LARGE;
  }
  while (n >= 3 * OR_BLK_SMALL) {
    uint64_t c0 = c, c1 = 0, c2 = 0;
    const uint8_t* q1 = p + OR_BLK_SMALL;
    const uint8_t* q2 = p + 2 * OR_BLK_SMALL;
    for (int i = 0; i < OR_BLK_SMALL; i += 8) {
      c0 = _mm_crc32_u64(c0, ld64(p + i));
      c1 = _mm_crc32_u64(c1, ld64(q1 + i));
      c2 = _mm_crc32_u64(c2, ld64(q2 + i));
    }
    c = clmul_shift((uint32_t)c0, g_k_small2) ^
        clmul_shift((uint32_t)c1, g_k_small1) ^ (uint32_t)c2;
    p += 3 * OR_BLK_SMALL;
    n -= 3 * OR_BLK_SMALL;
  }
  uint64_t c64 = c;
  while (n >= 8) {
    c64 = _mm_crc32_u64(c64, ld64(p));
    p += 8;
    n -= 8;
  }
  c = (uint32_t)c64;
  while (n--) c = _mm_crc32_u8(c, *p++);
  return c;
}
#endif

uint32_t oracle_crc32c_extend_fast(uint32_t crc, const void* p, size_t n) {
  crc_once();
#ifdef OR_HAVE_X86
  return ~crc_raw_update_fast(~crc, (const uint8_t*)p, n);
#else
  return ~crc_raw_update(~crc, (const uint8_t*)p, n);
#endif
}

/* util/crc32c.h:35 */
uint32_t oracle_crc32c_value(const void* p, size_t n) {
  return oracle_crc32c_extend(0, p, n);
}

/* raw state shifted by nbytes zero bytes: x^(8 nbytes) = (x^8)^nbytes, exact
 * for every 64-bit count (the reference walks the bits of len/4 over 62
 * powers, util/crc32c.cc:1200-1224, also exact; 8 * nbytes would wrap) */
uint32_t oracle_crc32c_shift(uint32_t state, uint64_t nbytes) {
  uint32_t m = 0x80000000u; /* 1 */
  uint32_t sq = 0x00800000u; /* x^8 */
  for (; nbytes; nbytes >>= 1) {
    if (nbytes & 1) m = gf_mul(m, sq);
    sq = gf_mul(sq, sq);
  }
  return gf_mul(state, m);
}

/* util/crc32c.cc:1279 Crc32cCombine: crc(A||B) from crc(A), crc(B), |B|.
 * With finalized CRCs F(M) = ~raw_{~0}(M):
 *   F(A||B) = shift(F(A), |B|) ^ F(B)   (the ~0 terms cancel). */
uint32_t oracle_crc32c_combine(uint32_t crc1, uint32_t crc2, size_t len2) {
  return oracle_crc32c_shift(crc1, len2) ^ crc2;
}

/* util/crc32c.h:44-53 */
static const uint32_t kMaskDelta = 0xa282ead8u;
uint32_t oracle_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + kMaskDelta;
}
uint32_t oracle_crc32c_unmask(uint32_t masked) {
  uint32_t rot = masked - kMaskDelta;
  return (rot >> 17) | (rot << 15);
}

/* ======================================================================== */
/* xxHash 0.8.1 (util/xxhash.h)                                              */
/* ======================================================================== */

#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P32_4 0x27D4EB2Fu
#define P32_5 0x165667B1u
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull

/* util/xxhash.h:3644 XXH3_kSecret (FARSH-derived, public constant) */
static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c,
    0xf7, 0x21, 0xad, 0x1c, 0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb,
    0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f, 0xcb, 0x79, 0xe6, 0x4e,
    0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6,
    0x81, 0x3a, 0x26, 0x4c, 0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb,
    0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3, 0x71, 0x64, 0x48, 0x97,
    0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7,
    0xc7, 0x0b, 0x4f, 0x1d, 0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31,
    0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, 0xea, 0xc5, 0xac, 0x83,
    0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26,
    0x29, 0xd4, 0x68, 0x9e, 0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc,
    0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce, 0x45, 0xcb, 0x3a, 0x8f,
    0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

static inline uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
static inline uint32_t rotl32(uint32_t x, int r) {
  return (x << r) | (x >> (32 - r));
}
static inline uint64_t swap64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint32_t swap32(uint32_t x) { return __builtin_bswap32(x); }

/* util/xxhash.h:3846 XXH3_mul128_fold64 */
static inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  __uint128_t p = (__uint128_t)a * b;
  return (uint64_t)p ^ (uint64_t)(p >> 64);
}
/* util/xxhash.h:2774 XXH64_avalanche */
static inline uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}
/* util/xxhash.h:3866 XXH3_avalanche */
static inline uint64_t xxh3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= 0x165667919E3779F9ull;
  h ^= h >> 32;
  return h;
}
/* util/xxhash.h:3878 XXH3_rrmxmx */
static inline uint64_t xxh3_rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= 0x9FB21C651E98DF25ull;
  h ^= (h >> 35) + len;
  h *= 0x9FB21C651E98DF25ull;
  return h ^ (h >> 28);
}

/* util/xxhash.h:3918-4001 XXH3_len_{1to3,4to8,9to16}_64b, seed 0 */
static uint64_t xxh3_len_0to16(const uint8_t* in, size_t len) {
  const uint8_t* s = kSecret;
  if (len > 8) {
    uint64_t bitflip1 = ld64(s + 24) ^ ld64(s + 32);
    uint64_t bitflip2 = ld64(s + 40) ^ ld64(s + 48);
    uint64_t lo = ld64(in) ^ bitflip1;
    uint64_t hi = ld64(in + len - 8) ^ bitflip2;
    uint64_t acc = len + swap64(lo) + hi + mul128_fold64(lo, hi);
    return xxh3_avalanche(acc);
  }
  if (len >= 4) {
    uint32_t in1 = ld32(in), in2 = ld32(in + len - 4);
    uint64_t bitflip = ld64(s + 8) ^ ld64(s + 16);
    uint64_t in64 = in2 + ((uint64_t)in1 << 32);
    return xxh3_rrmxmx(in64 ^ bitflip, len);
  }
  if (len) {
    uint8_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
    uint32_t combined = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) |
                        ((uint32_t)c3 << 0) | ((uint32_t)len << 8);
    uint64_t bitflip = (uint64_t)(ld32(s) ^ ld32(s + 4));
    return xxh64_avalanche((uint64_t)combined ^ bitflip);
  }
  return xxh64_avalanche(ld64(s + 56) ^ ld64(s + 64));
}

/* util/xxhash.h:4010 XXH3_mix16B, seed 0 */
static inline uint64_t mix16B(const uint8_t* in, const uint8_t* s) {
  return mul128_fold64(ld64(in) ^ ld64(s), ld64(in + 8) ^ ld64(s + 8));
}

/* util/xxhash.h:4043 XXH3_len_17to128_64b */
static uint64_t xxh3_len_17to128(const uint8_t* in, size_t len) {
  const uint8_t* s = kSecret;
  uint64_t acc = len * P64_1, acc_end;
  acc += mix16B(in + 0, s + 0);
  acc_end = mix16B(in + len - 16, s + 16);
  if (len > 32) {
    acc += mix16B(in + 16, s + 32);
    acc_end += mix16B(in + len - 32, s + 48);
    if (len > 64) {
      acc += mix16B(in + 32, s + 64);
      acc_end += mix16B(in + len - 48, s + 80);
      if (len > 96) {
        acc += mix16B(in + 48, s + 96);
        acc_end += mix16B(in + len - 64, s + 112);
      }
    }
  }
  return xxh3_avalanche(acc + acc_end);
}

/* util/xxhash.h:4083 XXH3_len_129to240_64b */
static uint64_t xxh3_len_129to240(const uint8_t* in, size_t len) {
  const uint8_t* s = kSecret;
  uint64_t acc = len * P64_1, acc_end;
  unsigned nbRounds = (unsigned)len / 16;
  for (unsigned i = 0; i < 8; i++) acc += mix16B(in + 16 * i, s + 16 * i);
  acc_end = mix16B(in + len - 16, s + 136 - 17);
  acc = xxh3_avalanche(acc);
  for (unsigned i = 8; i < nbRounds; i++)
    acc_end += mix16B(in + 16 * i, s + 16 * (i - 8) + 3);
  return xxh3_avalanche(acc + acc_end);
}

/* util/xxhash.h:4924-4927 XXH3_scalarRound / accumulate_512 */
static inline void acc512_scalar(uint64_t* acc, const uint8_t* in,
                                 const uint8_t* s) {
  for (int i = 0; i < 8; i++) {
    uint64_t d = ld64(in + 8 * i);
    uint64_t dk = d ^ ld64(s + 8 * i);
    acc[i ^ 1] += d;
    acc[i] += (uint64_t)(uint32_t)dk * (dk >> 32);
  }
}
/* util/xxhash.h:4962-4977 XXH3_scalarScrambleRound */
static inline void scramble_scalar(uint64_t* acc, const uint8_t* s) {
  for (int i = 0; i < 8; i++) {
    uint64_t a = acc[i];
    a ^= a >> 47;
    a ^= ld64(s + 8 * i);
    a *= P32_1;
    acc[i] = a;
  }
}

#ifdef OR_HAVE_X86
/* AVX2 form of the same two steps (util/xxhash.h XXH3_accumulate_512_avx2 /
 * XXH3_scrambleAcc_avx2 are the reference's selection at -march=native). */
__attribute__((target("avx2"))) static inline void acc512_avx2(
    __m256i* acc, const uint8_t* in, const uint8_t* s) {
  for (int i = 0; i < 2; i++) {
    __m256i d = _mm256_loadu_si256((const __m256i*)(in + 32 * i));
    __m256i k = _mm256_loadu_si256((const __m256i*)(s + 32 * i));
    __m256i dk = _mm256_xor_si256(d, k);
    __m256i dk_hi = _mm256_srli_epi64(dk, 32);
    __m256i prod = _mm256_mul_epu32(dk, dk_hi);
    __m256i dsw = _mm256_shuffle_epi32(d, _MM_SHUFFLE(1, 0, 3, 2));
    acc[i] = _mm256_add_epi64(acc[i], _mm256_add_epi64(prod, dsw));
  }
}
__attribute__((target("avx2"))) static inline void scramble_avx2(
    __m256i* acc, const uint8_t* s) {
  const __m256i prime = _mm256_set1_epi32((int)P32_1);
  for (int i = 0; i < 2; i++) {
    __m256i a = acc[i];
    a = _mm256_xor_si256(a, _mm256_srli_epi64(a, 47));
    a = _mm256_xor_si256(a,
                         _mm256_loadu_si256((const __m256i*)(s + 32 * i)));
    __m256i lo = _mm256_mul_epu32(a, prime);
    __m256i hi = _mm256_mul_epu32(_mm256_srli_epi64(a, 32), prime);
    acc[i] = _mm256_add_epi64(lo, _mm256_slli_epi64(hi, 32));
  }
}
__attribute__((target("avx2"))) static void hashlong_loop_avx2(
    uint64_t* acc64, const uint8_t* in, size_t len) {
  __m256i acc[2];
  memcpy(acc, acc64, 64);
  const size_t nbStripesPerBlock = (192 - 64) / 8; /* 16 */
  const size_t block_len = 64 * nbStripesPerBlock; /* 1024 */
  const size_t nb_blocks = (len - 1) / block_len;
  for (size_t n = 0; n < nb_blocks; n++) {
    for (size_t st = 0; st < nbStripesPerBlock; st++)
      acc512_avx2(acc, in + n * block_len + st * 64, kSecret + st * 8);
    scramble_avx2(acc, kSecret + 192 - 64);
  }
  size_t nbStripes = ((len - 1) - block_len * nb_blocks) / 64;
  for (size_t st = 0; st < nbStripes; st++)
    acc512_avx2(acc, in + nb_blocks * block_len + st * 64, kSecret + st * 8);
  acc512_avx2(acc, in + len - 64, kSecret + 192 - 64 - 7);
  memcpy(acc64, acc, 64);
}
static int g_have_avx2 = -1;
#endif

/* util/xxhash.h:5123 XXH3_hashLong_internal_loop (scalar form) */
static void hashlong_loop_scalar(uint64_t* acc, const uint8_t* in, size_t len) {
  const size_t nbStripesPerBlock = (192 - 64) / 8;
  const size_t block_len = 64 * nbStripesPerBlock;
  const size_t nb_blocks = (len - 1) / block_len;
  for (size_t n = 0; n < nb_blocks; n++) {
    for (size_t st = 0; st < nbStripesPerBlock; st++)
      acc512_scalar(acc, in + n * block_len + st * 64, kSecret + st * 8);
    scramble_scalar(acc, kSecret + 192 - 64);
  }
  size_t nbStripes = ((len - 1) - block_len * nb_blocks) / 64;
  for (size_t st = 0; st < nbStripes; st++)
    acc512_scalar(acc, in + nb_blocks * block_len + st * 64, kSecret + st * 8);
  /* last stripe, XXH_SECRET_LASTACC_START = 7 */
  acc512_scalar(acc, in + len - 64, kSecret + 192 - 64 - 7);
}

/* util/xxhash.h:5164 XXH3_mergeAccs + :5194 XXH3_hashLong_64b_internal */
static uint64_t xxh3_hashlong(const uint8_t* in, size_t len, int fast) {
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
#ifdef OR_HAVE_X86
  if (g_have_avx2 < 0) g_have_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
  if (fast && g_have_avx2)
    hashlong_loop_avx2(acc, in, len);
  else
#endif
    hashlong_loop_scalar(acc, in, len);
  (void)fast;
  const uint8_t* s = kSecret + 11; /* XXH_SECRET_MERGEACCS_START */
  uint64_t r = (uint64_t)len * P64_1;
  for (int i = 0; i < 4; i++)
    r += mul128_fold64(acc[2 * i] ^ ld64(s + 16 * i),
                       acc[2 * i + 1] ^ ld64(s + 16 * i + 8));
  return xxh3_avalanche(r);
}

static uint64_t xxh3_64_impl(const void* p, size_t n, int fast) {
  const uint8_t* in = (const uint8_t*)p;
  if (n <= 16) return xxh3_len_0to16(in, n);
  if (n <= 128) return xxh3_len_17to128(in, n);
  if (n <= 240) return xxh3_len_129to240(in, n);
  return xxh3_hashlong(in, n, fast);
}
/* util/xxhash.h:5311 XXH3_64bits (seed 0, default secret) */
uint64_t oracle_xxh3_64(const void* p, size_t n) { return xxh3_64_impl(p, n, 0); }
static uint64_t oracle_xxh3_64_fast(const void* p, size_t n) {
  return xxh3_64_impl(p, n, 1);
}

/* util/xxhash.h XXH32 (~:2400-2560) */
static inline uint32_t xxh32_round(uint32_t acc, uint32_t in) {
  acc += in * P32_2;
  acc = rotl32(acc, 13);
  return acc * P32_1;
}
uint32_t oracle_xxh32(const void* p, size_t len, uint32_t seed) {
  const uint8_t* in = (const uint8_t*)p;
  const uint8_t* end = in + len;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P32_1 + P32_2, v2 = seed + P32_2, v3 = seed,
             v4 = seed - P32_1;
    const uint8_t* limit = end - 15;
    do {
      v1 = xxh32_round(v1, ld32(in));
      v2 = xxh32_round(v2, ld32(in + 4));
      v3 = xxh32_round(v3, ld32(in + 8));
      v4 = xxh32_round(v4, ld32(in + 12));
      in += 16;
    } while (in < limit);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + P32_5;
  }
  h += (uint32_t)len;
  len &= 15;
  while (len >= 4) {
    h += ld32(in) * P32_3;
    h = rotl32(h, 17) * P32_4;
    in += 4;
    len -= 4;
  }
  while (len > 0) {
    h += (*in++) * P32_5;
    h = rotl32(h, 11) * P32_1;
    len--;
  }
  h ^= h >> 15;
  h *= P32_2;
  h ^= h >> 13;
  h *= P32_3;
  h ^= h >> 16;
  return h;
}

/* util/xxhash.h XXH64 (~:2750-2990) */
static inline uint64_t xxh64_round(uint64_t acc, uint64_t in) {
  acc += in * P64_2;
  acc = rotl64(acc, 31);
  return acc * P64_1;
}
static inline uint64_t xxh64_merge(uint64_t acc, uint64_t v) {
  acc ^= xxh64_round(0, v);
  return acc * P64_1 + P64_4;
}
uint64_t oracle_xxh64(const void* p, size_t len, uint64_t seed) {
  const uint8_t* in = (const uint8_t*)p;
  const uint8_t* end = in + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed,
             v4 = seed - P64_1;
    const uint8_t* limit = end - 31;
    do {
      v1 = xxh64_round(v1, ld64(in));
      v2 = xxh64_round(v2, ld64(in + 8));
      v3 = xxh64_round(v3, ld64(in + 16));
      v4 = xxh64_round(v4, ld64(in + 24));
      in += 32;
    } while (in < limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh64_merge(h, v1);
    h = xxh64_merge(h, v2);
    h = xxh64_merge(h, v3);
    h = xxh64_merge(h, v4);
  } else {
    h = seed + P64_5;
  }
  h += (uint64_t)len;
  len &= 31;
  while (len >= 8) {
    h ^= xxh64_round(0, ld64(in));
    h = rotl64(h, 27) * P64_1 + P64_4;
    in += 8;
    len -= 8;
  }
  if (len >= 4) {
    h ^= (uint64_t)ld32(in) * P64_1;
    h = rotl64(h, 23) * P64_2 + P64_3;
    in += 4;
    len -= 4;
  }
  while (len > 0) {
    h ^= (*in++) * P64_5;
    h = rotl64(h, 11) * P64_1;
    len--;
  }
  return xxh64_avalanche(h);
}

/* ======================================================================== */
/* XXPH3 (xxHash 0.7.2 preview, util/xxph3.h) -- Hash64 / NPHash64          */
/* (util/hash.cc:81-88, util/hash.h:45-62), the per-KV protection hash of    */
/* db/kv_checksum.h.  Same default secret as XXH3 0.8.1 (xxph3.h:920).       */
/* ======================================================================== */

/* xxph3.h:1069 XXPH3_avalanche (PRIME64_3, unlike 0.8.1's PRIME_MX1) */
static inline uint64_t xxph3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}

/* xxph3.h:1082-1140 XXPH3_len_{1to3,4to8,9to16}_64b + RocksDB's empty rule */
static uint64_t xxph3_len_0to16(const uint8_t* in, size_t len, uint64_t seed) {
  const uint8_t* s = kSecret;
  if (len > 8) {
    const uint64_t lo = ld64(in) ^ (ld64(s) + seed);
    const uint64_t hi = ld64(in + len - 8) ^ (ld64(s + 8) - seed);
    return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
  }
  if (len >= 4) {
    const uint64_t in64 = (uint64_t)ld32(in) | ((uint64_t)ld32(in + len - 4) << 32);
    const uint64_t keyed = in64 ^ (ld64(s) + seed);
    const uint64_t mix64 = len + ((keyed ^ (keyed >> 51)) * P32_1);
    return xxph3_avalanche((mix64 ^ (mix64 >> 47)) * P64_2);
  }
  if (len) {
    const uint32_t combined = (uint32_t)in[0] | ((uint32_t)in[len >> 1] << 8) |
                              ((uint32_t)in[len - 1] << 16) | ((uint32_t)len << 24);
    const uint64_t keyed = (uint64_t)combined ^ ((uint64_t)ld32(s) + seed);
    return xxph3_avalanche(keyed * P64_1);
  }
  return mul128_fold64(seed + ld64(s), P64_2); /* xxph3.h:1133-1138 */
}

/* xxph3.h:1640 XXPH3_mix16B */
static inline uint64_t xxph3_mix16B(const uint8_t* in, const uint8_t* s, uint64_t seed) {
  return mul128_fold64(ld64(in) ^ (ld64(s) + seed), ld64(in + 8) ^ (ld64(s + 8) - seed));
}

/* xxph3.h:1651 XXPH3_len_17to128_64b */
static uint64_t xxph3_len_17to128(const uint8_t* in, size_t len, uint64_t seed) {
  const uint8_t* s = kSecret;
  uint64_t acc = len * P64_1;
  if (len > 32) {
    if (len > 64) {
      if (len > 96) {
        acc += xxph3_mix16B(in + 48, s + 96, seed);
        acc += xxph3_mix16B(in + len - 64, s + 112, seed);
      }
      acc += xxph3_mix16B(in + 32, s + 64, seed);
      acc += xxph3_mix16B(in + len - 48, s + 80, seed);
    }
    acc += xxph3_mix16B(in + 16, s + 32, seed);
    acc += xxph3_mix16B(in + len - 32, s + 48, seed);
  }
  acc += xxph3_mix16B(in, s, seed);
  acc += xxph3_mix16B(in + len - 16, s + 16, seed);
  return xxph3_avalanche(acc);
}

/* xxph3.h:1681 XXPH3_len_129to240_64b */
static uint64_t xxph3_len_129to240(const uint8_t* in, size_t len, uint64_t seed) {
  const uint8_t* s = kSecret;
  uint64_t acc = len * P64_1;
  const int nb_rounds = (int)len / 16;
  for (int i = 0; i < 8; i++) acc += xxph3_mix16B(in + 16 * i, s + 16 * i, seed);
  acc = xxph3_avalanche(acc);
  for (int i = 8; i < nb_rounds; i++) acc += xxph3_mix16B(in + 16 * i, s + 16 * (i - 8) + 3, seed);
  acc += xxph3_mix16B(in + len - 16, s + 136 - 17, seed);
  return xxph3_avalanche(acc);
}

/* xxph3.h:1322-1339 XXPH3_accumulate_512, XXPH3_acc_64bits (no lane swap) */
static inline void xxph3_acc512(uint64_t* acc, const uint8_t* in, const uint8_t* s) {
  for (int i = 0; i < 8; i++) {
    const uint64_t d = ld64(in + 8 * i);
    const uint64_t dk = d ^ ld64(s + 8 * i);
    acc[i] += d;
    acc[i] += (dk & 0xFFFFFFFFull) * (dk >> 32);
  }
}

/* xxph3.h:1514-1583 hashLong: 16 stripes per 1 KiB block (nb_blocks =
 * len / 1024, NOT (len-1)/1024), scramble after each full block, last stripe
 * only if len % 64 != 0, merge from secret+11 with start len*PRIME64_1.
 * The seeded secret is kSecret with +seed / -seed on alternating 8-byte words
 * (xxph3.h:1609-1620). */
static uint64_t xxph3_hashlong(const uint8_t* in, size_t len, uint64_t seed) {
  uint8_t sec[192];
  for (int i = 0; i < 12; i++) {
    const uint64_t a = ld64(kSecret + 16 * i) + seed;
    const uint64_t b = ld64(kSecret + 16 * i + 8) - seed;
    memcpy(sec + 16 * i, &a, 8);
    memcpy(sec + 16 * i + 8, &b, 8);
  }
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const size_t nb_blocks = len / 1024;
  for (size_t n = 0; n < nb_blocks; n++) {
    for (int st = 0; st < 16; st++) xxph3_acc512(acc, in + 1024 * n + 64 * st, sec + 8 * st);
    for (int i = 0; i < 8; i++) { /* xxph3.h:1464-1477 scramble */
      uint64_t a = acc[i];
      a ^= a >> 47;
      a ^= ld64(sec + 128 + 8 * i);
      acc[i] = a * P32_1;
    }
  }
  const size_t nb_stripes = (len - 1024 * nb_blocks) / 64;
  for (size_t st = 0; st < nb_stripes; st++)
    xxph3_acc512(acc, in + 1024 * nb_blocks + 64 * st, sec + 8 * st);
  if (len & 63) xxph3_acc512(acc, in + len - 64, sec + 192 - 64 - 7);
  uint64_t r = len * P64_1;
  for (int i = 0; i < 4; i++)
    r += mul128_fold64(acc[2 * i] ^ ld64(sec + 11 + 16 * i),
                       acc[2 * i + 1] ^ ld64(sec + 11 + 16 * i + 8));
  return xxph3_avalanche(r);
}

/* xxph3.h:1733 XXPH3_64bits_withSeed == util/hash.cc:81 Hash64(data, n, seed) */
uint64_t oracle_hash64(const void* p, size_t n, uint64_t seed) {
  const uint8_t* in = (const uint8_t*)p;
  if (n <= 16) return xxph3_len_0to16(in, n, seed);
  if (n <= 128) return xxph3_len_17to128(in, n, seed);
  if (n <= 240) return xxph3_len_129to240(in, n, seed);
  return xxph3_hashlong(in, n, seed);
}

/* db/kv_checksum.h:84-88 field seeds */
#define KV_SEED_K 0ull
#define KV_SEED_V 0xD28AAD72F49BD50Bull
#define KV_SEED_O 0xA5155AE5E937AA16ull
#define KV_SEED_S 0x77A00858DDD37F21ull
#define KV_SEED_C 0x4A2AB5CBD26F542Cull

/* ProtectionInfo64().ProtectKV / ProtectKVO [.ProtectS] [.ProtectC]
 * (db/kv_checksum.h:296-332, :420-460): XOR of NPHash64 of each field with its
 * seed; op/seq/cf are hashed as their native (little-endian) bytes. */
uint64_t oracle_kv_protect(const void* key, size_t klen, const void* value, size_t vlen,
                           int op_type, int has_seq, uint64_t seq, int has_cf, uint32_t cf) {
  uint64_t v = oracle_hash64(key, klen, KV_SEED_K) ^ oracle_hash64(value, vlen, KV_SEED_V);
  if (op_type >= 0) {
    const uint8_t op = (uint8_t)op_type;
    v ^= oracle_hash64(&op, 1, KV_SEED_O);
  }
  if (has_seq) v ^= oracle_hash64(&seq, 8, KV_SEED_S);
  if (has_cf) v ^= oracle_hash64(&cf, 4, KV_SEED_C);
  return v;
}

void oracle_hash64_batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         const uint64_t* seeds, uint64_t seed, uint64_t* out, size_t n) {
  for (size_t i = 0; i < n; i++)
    out[i] = oracle_hash64(base + offsets[i], lengths[i], seeds ? seeds[i] : seed);
}

void oracle_kv_protect_batch(const uint8_t* base, const uint64_t* key_offsets,
                             const uint32_t* key_sizes, const uint64_t* value_offsets,
                             const uint32_t* value_sizes, const uint8_t* op_types,
                             const uint64_t* seqnos, const uint32_t* cf_ids, uint64_t* out,
                             size_t n) {
  for (size_t i = 0; i < n; i++)
    out[i] = oracle_kv_protect(base + key_offsets[i], key_sizes[i], base + value_offsets[i],
                               value_sizes[i], op_types ? op_types[i] : -1, seqnos != NULL,
                               seqnos ? seqnos[i] : 0, cf_ids != NULL, cf_ids ? cf_ids[i] : 0);
}

/* ProtectionInfo<T>::Verify (kv_checksum.h:117-133): the low `len` bytes of
 * the protection value against the LE bytes at `stored`. */
int oracle_kv_verify(uint64_t prot, uint32_t len, const void* stored) {
  uint64_t s = 0;
  memcpy(&s, stored, len);
  const uint64_t mask = len >= 8 ? ~0ull : ((1ull << (8 * len)) - 1);
  return ((s ^ prot) & mask) == 0;
}

/* util/coding.h:109 GetVarint32Ptr(p, limit) (+ coding.cc
 * GetVarint32PtrFallback): bytes consumed, 0 on failure.  `avail` bounds the
 * read (the reference reads up to limit regardless); -1 when it cuts in. */
static int varint32_ptr(const uint8_t* p, size_t avail, size_t limit, uint32_t* v) {
  uint32_t r = 0;
  for (size_t j = 0; j < 5 && j < limit; j++) {
    if (j >= avail) return -1;
    const uint32_t b = p[j];
    r |= (b & 127u) << (7 * j);
    if (!(b & 128u)) {
      *v = r;
      return (int)j + 1;
    }
  }
  return 0;
}

/* MemTable::VerifyEntryChecksum (db/memtable.cc:273-307) on the entry at p
 * with `avail` readable bytes: 0 OK, 1 "Unable to parse internal key length",
 * 2 "... internal key length too short.", 3 "Unable to parse internal key
 * value", 4 checksum mismatch, 5 the entry runs past avail (the engine's
 * report; the reference would read on).  *computed = the protection value
 * ProtectKVO(user_key, value, type).ProtectS(seq) (0 unless parsed). */
int oracle_memtable_verify(const uint8_t* p, size_t avail, uint32_t prot_bytes,
                           uint64_t* computed) {
  *computed = 0;
  uint32_t ikl = 0, vl = 0;
  const int n1 = varint32_ptr(p, avail, 5, &ikl);
  if (n1 < 0) return 5;
  if (n1 == 0) return 1;
  if (ikl < 8) return 2;
  const size_t ko = (size_t)n1, kl = ikl - 8;
  if (ko + kl + 8 > avail) return 5;
  uint64_t tag;
  memcpy(&tag, p + ko + kl, 8);
  const size_t vp = ko + kl + 8;
  const int n2 = varint32_ptr(p + vp, avail - vp, 5, &vl);
  if (n2 < 0) return 5;
  if (n2 == 0) return 3;
  const size_t vo = vp + (size_t)n2;
  if (vo + vl + prot_bytes > avail) return 5;
  /* UnPackSequenceAndType (dbformat.h): seq = tag >> 8, type = tag & 0xff */
  *computed = oracle_kv_protect(p + ko, kl, p + vo, vl, (int)(tag & 0xff), 1, tag >> 8, 0, 0);
  return oracle_kv_verify(*computed, prot_bytes, p + vo + vl) ? 0 : 4;
}

void oracle_memtable_verify_batch(const uint8_t* base, size_t base_len, const uint64_t* offsets,
                                  size_t n, uint32_t prot_bytes, uint64_t* computed,
                                  uint8_t* status) {
  for (size_t i = 0; i < n; i++) {
    const size_t o = offsets[i];
    status[i] = (uint8_t)(o > base_len ? 5
                                       : oracle_memtable_verify(base + o, base_len - o, prot_bytes,
                                                                &computed[i]));
    if (o > base_len) computed[i] = 0;
  }
}

/* ======================================================================== */
/* Block checksum dispatcher (table/format.cc, table/format.h)               */
/* ======================================================================== */

/* table/format.cc:559 ModifyChecksumForLastByte */
static inline uint32_t modify_for_last_byte(uint32_t v, uint8_t last) {
  return v ^ ((uint32_t)last * 0x6b9083d9u);
}

static uint32_t compute_builtin(int type, const uint8_t* p, size_t n,
                                int fast) {
  switch (type) {
    case OR_kCRC32c: /* Mask(crc32c::Value(data, n)) */
      return oracle_crc32c_mask(fast ? oracle_crc32c_extend_fast(0, p, n)
                                     : oracle_crc32c_extend(0, p, n));
    case OR_kxxHash:
      return oracle_xxh32(p, n, 0);
    case OR_kxxHash64:
      return (uint32_t)oracle_xxh64(p, n, 0);
    case OR_kXXH3:
      if (n == 0) return 0;
      return modify_for_last_byte(
          (uint32_t)(fast ? oracle_xxh3_64_fast(p, n - 1)
                          : oracle_xxh3_64(p, n - 1)),
          p[n - 1]);
    default: /* kNoChecksum and unknown */
      return 0;
  }
}

/* table/format.cc:568 ComputeBuiltinChecksum */
uint32_t oracle_compute_builtin_checksum(int type, const void* p, size_t n) {
  return compute_builtin(type, (const uint8_t*)p, n, 0);
}

static uint32_t compute_with_last(int type, const uint8_t* p, size_t n,
                                  uint8_t last, int fast) {
  switch (type) {
    case OR_kCRC32c: {
      uint32_t c = fast ? oracle_crc32c_extend_fast(0, p, n)
                        : oracle_crc32c_extend(0, p, n);
      c = oracle_crc32c_extend(c, &last, 1);
      return oracle_crc32c_mask(c);
    }
    case OR_kxxHash:
    case OR_kxxHash64: {
      /* streaming over data || last (format.cc:603-622): identical to the
       * one-shot hash of the concatenation. */
      uint8_t* tmp = (uint8_t*)malloc(n + 1);
      if (n) memcpy(tmp, p, n);
      tmp[n] = last;
      uint32_t v = type == OR_kxxHash ? oracle_xxh32(tmp, n + 1, 0)
                                      : (uint32_t)oracle_xxh64(tmp, n + 1, 0);
      free(tmp);
      return v;
    }
    case OR_kXXH3:
      return modify_for_last_byte(
          (uint32_t)(fast ? oracle_xxh3_64_fast(p, n) : oracle_xxh3_64(p, n)),
          last);
    default:
      return 0;
  }
}

/* table/format.cc:594 ComputeBuiltinChecksumWithLastByte */
uint32_t oracle_compute_builtin_checksum_with_last_byte(int type, const void* p,
                                                        size_t n,
                                                        uint8_t last) {
  return compute_with_last(type, (const uint8_t*)p, n, last, 0);
}

/* table/format.h:119 ChecksumModifierForContext */
uint32_t oracle_checksum_modifier_for_context(uint32_t base, uint64_t offset) {
  uint32_t all_or_nothing = 0u - (uint32_t)(base != 0);
  uint32_t modifier = base ^ ((uint32_t)offset + (uint32_t)(offset >> 32));
  return modifier & all_or_nothing;
}

/* table/block_based/reader_common.cc:26 VerifyBlockChecksum */
static int verify_block(int type, const uint8_t* data, size_t block_size,
                        uint32_t modifier, uint32_t* computed_out,
                        uint32_t* stored_out, uint32_t* trailer_domain,
                        int fast) {
  size_t len = block_size + 1;
  uint32_t stored = ld32(data + len);
  uint32_t computed = compute_builtin(type, data, len, fast);
  if (trailer_domain) *trailer_domain = computed;
  stored -= modifier;
  int ok = stored == computed;
  if (!ok && type == OR_kCRC32c) {
    stored = oracle_crc32c_unmask(stored);
    computed = oracle_crc32c_unmask(computed);
  }
  if (computed_out) *computed_out = computed;
  if (stored_out) *stored_out = stored;
  return ok;
}
int oracle_verify_block_checksum(int type, const void* data, size_t block_size,
                                 uint32_t modifier, uint32_t* computed,
                                 uint32_t* stored) {
  return verify_block(type, (const uint8_t*)data, block_size, modifier,
                      computed, stored, NULL, 0);
}

/* ======================================================================== */
/* Threaded batch helpers (static contiguous partition per thread)           */
/* ======================================================================== */

typedef struct {
  int kind;
  int type;
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* sizes;
  const uint8_t* last_bytes;
  const uint32_t* modifiers;
  uint32_t* out32;
  uint64_t* out64;
  uint8_t* ok;
  size_t lo, hi;
  uint64_t bad;
  /* kind 4 (logical WAL records): first physical record of each of the
   * n_all records, n_phys physical records with hs-byte headers */
  const uint64_t* first;
  uint64_t n_phys;
  size_t n_all;
  uint32_t hs;
} batch_job;

/* kind 4: XXH3_64bits of each logical record's payload, its fragments
 * gathered back to back (log::Reader::ReadRecord's record checksum,
 * db/log_reader.cc:95-165, over the scratch it assembles at :129-156) */
static void logical_xxh3_range(batch_job* j) {
  size_t cap = (size_t)1 << 16;
  uint8_t* buf = (uint8_t*)malloc(cap);
  for (size_t i = j->lo; i < j->hi; i++) {
    const uint64_t b = j->first[i];
    const uint64_t e = i + 1 < j->n_all ? j->first[i + 1] : j->n_phys;
    size_t len = 0;
    for (uint64_t q = b; q < e; q++) len += j->sizes[q];
    if (len > cap) {
      while (cap < len) cap *= 2;
      buf = (uint8_t*)realloc(buf, cap);
    }
    size_t at = 0;
    for (uint64_t q = b; q < e; q++) {
      memcpy(buf + at, j->base + j->offsets[q] + j->hs, j->sizes[q]);
      at += j->sizes[q];
    }
    j->out64[i] = oracle_xxh3_64_fast(buf, len);
  }
  free(buf);
}

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  uint64_t bad = 0;
  if (j->kind == 4) {
    logical_xxh3_range(j);
    return NULL;
  }
  for (size_t i = j->lo; i < j->hi; i++) {
    const uint8_t* p = j->base + j->offsets[i];
    uint32_t m = j->modifiers ? j->modifiers[i] : 0;
    switch (j->kind) {
      case 0: { /* compute */
        uint8_t last = j->last_bytes ? j->last_bytes[i] : p[j->sizes[i]];
        j->out32[i] = compute_with_last(j->type, p, j->sizes[i], last, 1) + m;
        break;
      }
      case 1: { /* verify */
        uint32_t c, s, td;
        int ok = verify_block(j->type, p, j->sizes[i], m, &c, &s, &td, 1);
        /* report the trailer-domain computed value (before unmasking) */
        if (j->out32) j->out32[i] = td;
        if (j->ok) j->ok[i] = (uint8_t)ok;
        bad += !ok;
        break;
      }
      case 2:
        j->out32[i] = oracle_crc32c_extend_fast(0, p, j->sizes[i]);
        break;
      case 3:
        j->out64[i] = oracle_xxh3_64_fast(p, j->sizes[i]);
        break;
    }
  }
  j->bad = bad;
  return NULL;
}

static uint64_t run_batch(batch_job proto, size_t n, int nthreads) {
  crc_once();
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
  batch_job* jobs = (batch_job*)calloc((size_t)nthreads, sizeof(batch_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = proto;
    jobs[t].lo = n * (size_t)t / (size_t)nthreads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)nthreads;
  }
  for (int t = 1; t < nthreads; t++)
    pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  batch_worker(&jobs[0]);
  uint64_t bad = jobs[0].bad;
  for (int t = 1; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    bad += jobs[t].bad;
  }
  free(jobs);
  free(th);
  return bad;
}

void oracle_block_checksum_batch(int type, const uint8_t* base,
                                 const uint64_t* offsets, const uint32_t* sizes,
                                 const uint8_t* last_bytes,
                                 const uint32_t* modifiers, uint32_t* out,
                                 size_t n, int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 0;
  j.type = type;
  j.base = base;
  j.offsets = offsets;
  j.sizes = sizes;
  j.last_bytes = last_bytes;
  j.modifiers = modifiers;
  j.out32 = out;
  run_batch(j, n, nthreads);
}

uint64_t oracle_block_verify_batch(int type, const uint8_t* base,
                                   const uint64_t* offsets,
                                   const uint32_t* sizes,
                                   const uint32_t* modifiers,
                                   uint32_t* computed, uint8_t* ok, size_t n,
                                   int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 1;
  j.type = type;
  j.base = base;
  j.offsets = offsets;
  j.sizes = sizes;
  j.modifiers = modifiers;
  j.out32 = computed;
  j.ok = ok;
  return run_batch(j, n, nthreads);
}

void oracle_crc32c_batch(const uint8_t* base, const uint64_t* offsets,
                         const uint32_t* lengths, uint32_t* out, size_t n,
                         int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 2;
  j.base = base;
  j.offsets = offsets;
  j.sizes = lengths;
  j.out32 = out;
  run_batch(j, n, nthreads);
}

void oracle_xxh3_batch(const uint8_t* base, const uint64_t* offsets,
                       const uint32_t* lengths, uint64_t* out, size_t n,
                       int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 3;
  j.base = base;
  j.offsets = offsets;
  j.sizes = lengths;
  j.out64 = out;
  run_batch(j, n, nthreads);
}

void oracle_wal_record_xxh3_batch(const uint8_t* log, const uint64_t* phys_offsets,
                                  const uint32_t* phys_lengths, uint64_t n_phys, uint32_t hs,
                                  const uint64_t* first, uint64_t* out, size_t n, int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 4;
  j.base = log;
  j.offsets = phys_offsets;
  j.sizes = phys_lengths;
  j.n_phys = n_phys;
  j.hs = hs;
  j.first = first;
  j.n_all = n;
  j.out64 = out;
  run_batch(j, n, nthreads);
}

/* ======================================================================== */
/* WAL (db/log_format.h, db/log_writer.cc, db/log_reader.cc)                 */
/* ======================================================================== */

#define LOG_BLOCK 32768u  /* db/log_format.h:45 kBlockSize */
#define LOG_HDR 7u        /* db/log_format.h:48 kHeaderSize */
#define LOG_RHDR 11u      /* db/log_format.h:52 kRecyclableHeaderSize */

enum { kZeroType = 0, kFullType = 1, kFirstType = 2, kMiddleType = 3,
       kLastType = 4, kRecyclableFullType = 5, kRecyclableFirstType = 6,
       kRecyclableMiddleType = 7, kRecyclableLastType = 8,
       kSetCompressionType = 9, kUserDefinedTimestampSizeType = 10,
       kRecyclableUserDefinedTimestampSizeType = 11 };

/* db/log_writer.cc:228-263 EmitPhysicalRecord CRC:
 *   crc = type_crc_[t]  (= crc32c::Value(&t, 1), log_writer.cc:33-36)
 *   if recyclable: crc = Extend(crc, LE32(log_number), 4)
 *   crc = Crc32cCombine(crc, Value(payload, n), n); Mask(crc)
 * which equals Mask(Value(header[6 .. hdr) || payload)). */
uint32_t oracle_wal_record_crc(int type, uint32_t log_number,
                               const void* payload, size_t n) {
  uint8_t t = (uint8_t)type;
  uint32_t crc = oracle_crc32c_value(&t, 1);
  int recyclable = !(type < kRecyclableFullType || type == kSetCompressionType ||
                     type == kUserDefinedTimestampSizeType);
  if (recyclable) {
    uint8_t ln[4];
    memcpy(ln, &log_number, 4);
    crc = oracle_crc32c_extend(crc, ln, 4);
  }
  uint32_t payload_crc = oracle_crc32c_value(payload, n);
  crc = oracle_crc32c_combine(crc, payload_crc, n);
  return oracle_crc32c_mask(crc);
}

/* Sizing pass for the framing below (same walk, no writes). */
uint64_t oracle_wal_framed_size(const uint32_t* lengths, size_t n,
                                int recyclable) {
  const uint32_t hs = recyclable ? LOG_RHDR : LOG_HDR;
  uint64_t off = 0;
  uint32_t bo = 0; /* block_offset_ */
  for (size_t r = 0; r < n; r++) {
    uint64_t left = lengths[r];
    int begin = 1;
    do {
      uint32_t leftover = LOG_BLOCK - bo;
      if (leftover < hs) {
        off += leftover;
        bo = 0;
      }
      uint32_t avail = LOG_BLOCK - bo - hs;
      uint64_t frag = left < avail ? left : avail;
      off += hs + frag;
      bo += hs + (uint32_t)frag;
      left -= frag;
      begin = 0;
    } while (left > 0);
    (void)begin;
  }
  return off;
}

/* db/log_writer.cc:65-160 Writer::AddRecord (no compression) */
uint64_t oracle_wal_frame(const uint8_t* payloads, const uint32_t* lengths,
                          size_t n, int recyclable, uint32_t log_number,
                          uint8_t* dst, uint64_t* rec_offsets,
                          uint32_t* rec_lengths, uint64_t* n_phys) {
  crc_once();
  const uint32_t hs = recyclable ? LOG_RHDR : LOG_HDR;
  uint64_t off = 0, np = 0;
  uint32_t bo = 0;
  const uint8_t* src = payloads;
  for (size_t r = 0; r < n; r++) {
    uint64_t left = lengths[r];
    const uint8_t* ptr = src;
    int begin = 1;
    do {
      uint32_t leftover = LOG_BLOCK - bo;
      if (leftover < hs) {
        memset(dst + off, 0, leftover); /* zero trailer (log_writer.cc:88) */
        off += leftover;
        bo = 0;
      }
      uint32_t avail = LOG_BLOCK - bo - hs;
      uint64_t frag = left < avail ? left : avail;
      int end = left == frag;
      int type;
      if (begin && end)
        type = recyclable ? kRecyclableFullType : kFullType;
      else if (begin)
        type = recyclable ? kRecyclableFirstType : kFirstType;
      else if (end)
        type = recyclable ? kRecyclableLastType : kLastType;
      else
        type = recyclable ? kRecyclableMiddleType : kMiddleType;
      uint8_t* h = dst + off;
      h[4] = (uint8_t)(frag & 0xff);
      h[5] = (uint8_t)(frag >> 8);
      h[6] = (uint8_t)type;
      if (recyclable) memcpy(h + 7, &log_number, 4);
      uint32_t crc = oracle_wal_record_crc(type, log_number, ptr, frag);
      memcpy(h, &crc, 4);
      memcpy(h + hs, ptr, frag);
      if (rec_offsets) rec_offsets[np] = off;
      if (rec_lengths) rec_lengths[np] = (uint32_t)frag;
      np++;
      off += hs + frag;
      bo += hs + (uint32_t)frag;
      ptr += frag;
      left -= frag;
      begin = 0;
    } while (left > 0);
    src += lengths[r];
  }
  if (n_phys) *n_phys = np;
  return off;
}

/* db/log_reader.cc:450-531 ReadPhysicalRecord, CRC check branch, applied to
 * each 32 KiB log block independently (records never straddle blocks,
 * log_writer.cc:86-102).  A CRC failure drops the rest of the block
 * (log_reader.cc:523-530) -- later records of that block are not reported. */
typedef struct {
  const uint8_t* buf;
  uint64_t nbytes;
  uint64_t blo, bhi;
  uint64_t nrec, bad;
  /* per-block outputs (oracle_wal_verify_blocks; NULL for the totals form):
   * status (0 ok, 1 checksum, 2 length, 3 zero record, 4 old record),
   * records verified before the first failure, offset in the block of the
   * failing header or of the end of parsing; log_number for recyclable
   * headers (log_reader.cc:497-503) */
  uint8_t* status;
  uint32_t* nrec_out;
  uint32_t* fail_out;
  uint32_t log_number;
  int check_log;  /* compare recyclable headers' log number (the per-block form) */
} wal_job;

static void* wal_worker(void* arg) {
  wal_job* j = (wal_job*)arg;
  uint64_t nrec = 0, bad = 0;
  for (uint64_t b = j->blo; b < j->bhi; b++) {
    uint64_t start = b * LOG_BLOCK;
    uint64_t end = start + LOG_BLOCK;
    if (end > j->nbytes) end = j->nbytes;
    uint64_t pos = start;
    uint32_t blk_ok = 0;
    uint8_t st = 0;
    while (end - pos >= LOG_HDR) {
      const uint8_t* h = j->buf + pos;
      uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
      unsigned type = h[6];
      uint32_t hs = LOG_HDR;
      int recyc = (type >= kRecyclableFullType && type <= kRecyclableLastType) ||
                  type == kRecyclableUserDefinedTimestampSizeType;
      if (recyc) hs = LOG_RHDR;
      if (end - pos < hs) break;
      if (hs + length > end - pos) { bad++; st = 2; break; } /* kBadRecordLen */
      if (j->check_log && recyc && ld32(h + 7) != j->log_number) { st = 4; break; } /* kOldRecord */
      if (type == kZeroType && length == 0) { st = 3; break; } /* preallocated */
      uint32_t expected = oracle_crc32c_unmask(ld32(h));
      uint32_t actual = ~crc_raw_update_fast(~0u, h + 6, length + hs - 6);
      nrec++;
      if (actual != expected) { bad++; st = 1; break; }
      blk_ok++;
      pos += hs + length;
    }
    if (j->status) j->status[b] = st;
    if (j->nrec_out) j->nrec_out[b] = blk_ok;
    if (j->fail_out) j->fail_out[b] = (uint32_t)(pos - start);
  }
  j->nrec = nrec;
  j->bad = bad;
  return NULL;
}

/* per log block: status / verified records / failing offset (see wal_job) */
void oracle_wal_verify_blocks(const uint8_t* buf, uint64_t nbytes, uint32_t log_number,
                              uint8_t* status, uint32_t* nrec, uint32_t* fail_off, int nthreads) {
  crc_once();
  uint64_t nblocks = (nbytes + LOG_BLOCK - 1) / LOG_BLOCK;
  if (nthreads < 1) nthreads = 1;
  wal_job* jobs = (wal_job*)calloc((size_t)nthreads, sizeof(wal_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t].buf = buf;
    jobs[t].nbytes = nbytes;
    jobs[t].blo = nblocks * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].bhi = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
    jobs[t].status = status;
    jobs[t].nrec_out = nrec;
    jobs[t].fail_out = fail_off;
    jobs[t].log_number = log_number;
    jobs[t].check_log = 1;
  }
  for (int t = 1; t < nthreads; t++)
    pthread_create(&th[t], NULL, wal_worker, &jobs[t]);
  wal_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
}

uint64_t oracle_wal_verify(const uint8_t* buf, uint64_t nbytes, uint8_t* ok,
                           uint64_t ok_cap, uint64_t* bad, int nthreads) {
  crc_once();
  (void)ok;
  (void)ok_cap;
  uint64_t nblocks = (nbytes + LOG_BLOCK - 1) / LOG_BLOCK;
  if (nthreads < 1) nthreads = 1;
  wal_job* jobs = (wal_job*)calloc((size_t)nthreads, sizeof(wal_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t].buf = buf;
    jobs[t].nbytes = nbytes;
    jobs[t].blo = nblocks * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].bhi = nblocks * (uint64_t)(t + 1) / (uint64_t)nthreads;
  }
  for (int t = 1; t < nthreads; t++)
    pthread_create(&th[t], NULL, wal_worker, &jobs[t]);
  wal_worker(&jobs[0]);
  uint64_t nrec = jobs[0].nrec, nbad = jobs[0].bad;
  for (int t = 1; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    nrec += jobs[t].nrec;
    nbad += jobs[t].bad;
  }
  free(jobs);
  free(th);
  if (bad) *bad = nbad;
  return nrec;
}

/* ======================================================================== */
/* Synthetic data (splitmix64 per config)                     */
/* ======================================================================== */

#define SM_GAMMA 0x9E3779B97F4A7C15ull
uint64_t oracle_splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void oracle_fill_stream(uint8_t* dst, uint64_t start, uint64_t nbytes,
                        uint64_t seed) {
  for (uint64_t i = 0; i < nbytes; i++) {
    uint64_t g = start + i;
    uint64_t w = oracle_splitmix64(seed + ((g >> 3) + 1) * SM_GAMMA);
    dst[i] = (uint8_t)(w >> (8 * (g & 7)));
  }
}
