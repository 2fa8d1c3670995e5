// forst_amd/csrc/device_common.h -- gfx950 device helpers shared by the kernels.
#pragma once
// register budget of a kernel as resident waves per SIMD (the SIMT emulator,
// tests/emu, defines it away)
#ifndef FORST_WAVES_PER_EU
#define FORST_WAVES_PER_EU(n) __attribute__((amdgpu_waves_per_eu(n)))
#endif
#include <hip/hip_runtime.h>

#include <cstdint>

namespace forst {

// Wave-uniform value (forces an SGPR; the compiler cannot prove that
// threadIdx.x >> 6 is uniform on its own -- cdna_hip_programming.md T20).
__device__ __forceinline__ uint32_t uniform(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// a kernel's register budget for n waves per SIMD (the compiler spills
// rather than exceed it); nothing in the host emulation (tests/emu)
#ifdef FORST_HOST_EMULATION
#define FORST_WAVES_PER_EU(n)
#else
#define FORST_WAVES_PER_EU(n) __attribute__((amdgpu_waves_per_eu(n)))
#endif

// 16-byte vector with only 4-byte alignment: lowers to one global_load_dwordx4
// on gfx950 (dword-aligned multi-dword loads are legal), so lane segments that
// start at any dword boundary are read with one instruction.
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // 16-byte aligned (LDS)

// Opaque per-lane zero.  Adding it to a wave-uniform data address forces a
// VECTOR (global_load) access: hipcc otherwise turns uniform loads it proves
// unclobbered into scalar s_load_dword, whose SBASE low bits are ignored --
// wrong for the byte-granular, unaligned-start addresses of SST blocks --
// and which read through the scalar cache.  Descriptor arrays may still use
// SMEM; block bytes never do.
__device__ __forceinline__ uint32_t vzero() {
  uint32_t z;
#ifndef FORST_HOST_EMULATION  // tests/emu compiles these sources as host C++
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#else
  z = 0;
#endif
  return z;
}

// Copy through an opaque v_mov: the load that produced `v` is waited for HERE
// and the result is no longer a load destination.  Used on rarely taken
// branches whose loaded values merge into a hot path, where hipcc would
// otherwise place a draining s_waitcnt vmcnt(0) after the join.
__device__ __forceinline__ uint32_t retire(uint32_t v) {
  uint32_t r;
#ifndef FORST_HOST_EMULATION
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
#else
  r = v;
#endif
  return r;
}

// A value the compiler may not hoist: a lane constant recomputed where it is
// used, inside a loop, rather than kept live across it (at high register
// pressure such constants are spilled, and a spill reload in a streaming
// loop is a vmcnt(0) wait on the loads in flight).
__device__ __forceinline__ uint32_t fresh(uint32_t v) {
#ifndef FORST_HOST_EMULATION
  asm volatile("" : "+v"(v));
#endif
  return v;
}

// Orders a wave's LDS stores before its later LDS loads of other lanes'
// words (a wave's LDS operations complete in order on the GPU; the fences
// keep the compiler from moving them across; the emulator's threads meet).
__device__ __forceinline__ void wave_lds_sync() {
#ifdef FORST_HOST_EMULATION
  (void)__ballot(1);
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

#ifdef FORST_DEBUG_BOUNDS
// Diagnostics build only (make DEBUG_BOUNDS=1 -> lib/libforst_checksum_dbg.so):
// every block-data load is checked against the launch's buffer bounds; the
// first violation (source line, offset, width) is recorded and the access is
// skipped instead of faulting the GPU.
struct DbgState {
  uint64_t lo, hi;
  unsigned long long rec[4];  // line, offset from lo, width, count
};
static __device__ DbgState g_forst_dbg;
__device__ __forceinline__ bool dbg_ok(const void* p, uint32_t n, uint32_t line) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  if (a >= g_forst_dbg.lo && a + n <= g_forst_dbg.hi) return true;
  if (atomicCAS(&g_forst_dbg.rec[0], 0ull, static_cast<unsigned long long>(line)) == 0ull) {
    g_forst_dbg.rec[1] = a - g_forst_dbg.lo;
    g_forst_dbg.rec[2] = n;
  }
  atomicAdd(&g_forst_dbg.rec[3], 1ull);
  return false;
}
#define FORST_DBG_OK(p, n) ::forst::dbg_ok((p), (n), __LINE__)
#else
#define FORST_DBG_OK(p, n) true
#endif

__device__ __forceinline__ u32x4a4 ld16_a4(const uint8_t* p) {
  if (!FORST_DBG_OK(p, 16)) return u32x4a4{0u, 0u, 0u, 0u};
  return *reinterpret_cast<const u32x4a4*>(p);
}
__device__ __forceinline__ uint32_t ld4_a4(const uint8_t* p) {
  if (!FORST_DBG_OK(p, 4)) return 0u;
  return *reinterpret_cast<const uint32_t*>(p);
}

// Little-endian 32/64-bit read at any byte address, touching only the
// dword-aligned words that overlap [p, p+4) / [p, p+8) (never a word that lies
// entirely outside the requested bytes, so it cannot fault past a buffer end).
// (Pointers are always derived from the kernel's buffer argument by pointer
// arithmetic -- never rebuilt from integers -- so the compiler keeps them in
// the global address space and emits global_load, not flat_load.)
__device__ __forceinline__ uint32_t ldu32(const uint8_t* p) {
  const uint32_t m = reinterpret_cast<uint64_t>(p) & 3;
  const uint8_t* q = p - m + vzero();
  const uint32_t lo = ld4_a4(q);
  if (m == 0) return lo;
  const uint32_t hi = ld4_a4(q + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, m);
}
__device__ __forceinline__ uint64_t ldu64(const uint8_t* p) {
  const uint32_t m = reinterpret_cast<uint64_t>(p) & 3;
  const uint8_t* q = p - m + vzero();
  const uint32_t w0 = ld4_a4(q), w1 = ld4_a4(q + 4);
  if (m == 0) return (static_cast<uint64_t>(w1) << 32) | w0;
  const uint32_t w2 = ld4_a4(q + 8);
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, m);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, m);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ uint32_t ldu8(const uint8_t* p) {
  if (!FORST_DBG_OK(p, 1)) return 0u;
  return *(p + vzero());
}
// dword-aligned single dword, vector path
__device__ __forceinline__ uint32_t ld4v(const uint8_t* p) { return ld4_a4(p + vzero()); }

// little-endian 32-bit store at any alignment with the fewest naturally
// aligned stores: 1 (p % 4 == 0), 2 (p % 2 == 0) or 3 (odd: byte, short, byte)
// -- the writer's in-place CRCs land at arbitrary header offsets, and each
// store is a scattered partial-line write
__device__ __forceinline__ void st_le32(uint8_t* p, uint32_t v) {
  const uintptr_t m = reinterpret_cast<uintptr_t>(p) & 3;
  if (m == 0) {
    *reinterpret_cast<uint32_t*>(p) = v;
  } else if (m == 2) {
    reinterpret_cast<uint16_t*>(p)[0] = static_cast<uint16_t>(v);
    reinterpret_cast<uint16_t*>(p)[1] = static_cast<uint16_t>(v >> 16);
  } else {
    p[0] = static_cast<uint8_t>(v);
    *reinterpret_cast<uint16_t*>(p + 1) = static_cast<uint16_t>(v >> 8);
    p[3] = static_cast<uint8_t>(v >> 24);
  }
}

// A WAL physical-record header [crc:4 len:2 type:1 (lognum:4)] at byte pos
// (db/log_format.h, any alignment): one dword-aligned 16-byte load covers all
// 11 bytes.  The walks chase one header after another per lane at scattered
// addresses, so the header read is their cost: one load request instead of
// 7-11 byte loads.  Within 16 bytes of the buffer end, byte loads (bytes at
// or past log_len read as 0; callers check the room they need first).
struct WalHdr {
  uint32_t crc;     // masked, as stored
  uint32_t length;  // payload bytes
  uint32_t type;    // the type byte
  uint32_t lognum;  // recyclable headers' log number
};
__device__ __forceinline__ WalHdr load_wal_header(const uint8_t* log, uint64_t log_len,
                                                  uint64_t pos) {
  WalHdr r;
  const uint64_t q = pos & ~3ull;
  if (q + 16 <= log_len) {
    const u32x4a4 v = ld16_a4(log + q + vzero());
    const uint32_t o = static_cast<uint32_t>(pos & 3);
    const uint32_t d0 = __builtin_amdgcn_alignbyte(v.y, v.x, o);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(v.z, v.y, o);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(v.w, v.z, o);
    r.crc = d0;
    r.length = d1 & 0xffffu;
    r.type = (d1 >> 16) & 0xffu;
    r.lognum = (d1 >> 24) | (d2 << 8);
  } else {
    uint32_t b[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) b[k] = pos + k < log_len ? log[pos + k] : 0u;
    r.crc = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
    r.length = b[4] | (b[5] << 8);
    r.type = b[6];
    r.lognum = b[7] | (b[8] << 8) | (b[9] << 16) | (b[10] << 24);
  }
  return r;
}

// util/crc32c.h:44-53
__device__ __forceinline__ uint32_t crc_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}
__device__ __forceinline__ uint32_t crc_unmask(uint32_t m) {
  const uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}
// table/format.cc:559 ModifyChecksumForLastByte
__device__ __forceinline__ uint32_t modify_for_last_byte(uint32_t v,
                                                         uint32_t last) {
  return v ^ ((last & 0xffu) * 0x6b9083d9u);
}

// Byte stores of a little-endian u32 at any address (trailer / WAL header).
__device__ __forceinline__ void stu32_bytes(uint8_t* p, uint32_t v) {
  p[0] = static_cast<uint8_t>(v);
  p[1] = static_cast<uint8_t>(v >> 8);
  p[2] = static_cast<uint8_t>(v >> 16);
  p[3] = static_cast<uint8_t>(v >> 24);
}

}  // namespace forst
