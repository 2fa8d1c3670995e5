// tests/emu/hip/hip_runtime.h -- TEST INFRASTRUCTURE ONLY.
//
// A tiny SIMT emulator that lets the UNMODIFIED kernel sources in
// forst_amd/csrc/*.hip compile as host C++ (clang) and run on the CPU: every
// workgroup is run with one std::thread per work-item, waves of 64 threads
// exchange values through a per-wave barrier (__shfl_xor, readfirstlane) and
// __syncthreads is a workgroup barrier.  It shadows <hip/hip_runtime.h> only
// when tests/emu is first on the include path (tests/emu/build_emu.sh); the
// product build never sees it.  Used to debug kernel index math / lane logic
// without a GPU and to run the oracle parity tests on the CPU.
#pragma once

#include <atomic>
#include <barrier>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __constant__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define FORST_WAVES_PER_EU(n)
#define __shared__ static

struct dim3 {
  uint32_t x, y, z;
  constexpr dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};

typedef int hipError_t;
typedef void* hipStream_t;
constexpr hipError_t hipSuccess = 0;
constexpr hipError_t hipErrorUnknown = 999;
struct hipDeviceProp_t {
  char gcnArchName[256];
  int multiProcessorCount;
};
inline const char* hipGetErrorString(hipError_t) { return "emu"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipGetDevice(int* d) {
  *d = 0;
  return hipSuccess;
}
inline hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int) {
  std::memset(p, 0, sizeof(*p));
  std::strcpy(p->gcnArchName, "gfx950:sramecc+:xnack-");
  const char* cus = std::getenv("FORST_EMU_CUS");
  p->multiProcessorCount = cus ? std::atoi(cus) : 2;
  return hipSuccess;
}

namespace emu {
struct Wave {
  uint32_t slot[64];
  std::unique_ptr<std::barrier<>> bar;
};
struct Group {
  std::unique_ptr<std::barrier<>> bar;
  std::vector<Wave> waves;
};
extern thread_local dim3 tl_tid;
extern thread_local dim3 tl_bid;
extern thread_local Group* tl_group;
extern dim3 g_grid, g_block;

inline uint32_t exchange(uint32_t v, uint32_t src_lane) {
  Wave& w = tl_group->waves[tl_tid.x >> 6];
  const uint32_t lane = tl_tid.x & 63;
  w.slot[lane] = v;
  w.bar->arrive_and_wait();
  const uint32_t r = w.slot[src_lane & 63];
  w.bar->arrive_and_wait();
  return r;
}

template <typename K, typename... Args>
void launch(K kernel, dim3 grid, dim3 block, Args... args) {
  g_grid = grid;
  g_block = block;
  const uint32_t nthreads = block.x;
  for (uint32_t b = 0; b < grid.x; ++b) {
    Group g;
    g.bar = std::make_unique<std::barrier<>>(nthreads);
    g.waves.resize((nthreads + 63) / 64);
    for (uint32_t w = 0; w < g.waves.size(); ++w)
      g.waves[w].bar = std::make_unique<std::barrier<>>(std::min<uint32_t>(64, nthreads - 64 * w));
    std::vector<std::thread> th;
    th.reserve(nthreads);
    for (uint32_t t = 0; t < nthreads; ++t) {
      th.emplace_back([&, t, b] {
        tl_tid = dim3(t);
        tl_bid = dim3(b);
        tl_group = &g;
        kernel(args...);
      });
    }
    for (auto& x : th) x.join();
  }
}
}  // namespace emu

#define threadIdx (::emu::tl_tid)
#define blockIdx (::emu::tl_bid)
#define gridDim (::emu::g_grid)
#define blockDim (::emu::g_block)

inline void __syncthreads() { emu::tl_group->bar->arrive_and_wait(); }
// the lanes of a wave run in lockstep on the hardware: LDS written by one lane
// before this point is visible to the others after it
inline void __builtin_amdgcn_wave_barrier() {
  emu::tl_group->waves[emu::tl_tid.x >> 6].bar->arrive_and_wait();
}
inline uint32_t __shfl_xor(uint32_t v, int mask) {
  return emu::exchange(v, (emu::tl_tid.x & 63) ^ static_cast<uint32_t>(mask));
}
inline uint32_t __shfl(uint32_t v, int src) {
  return emu::exchange(v, static_cast<uint32_t>(src));
}
// the real builtins return int (sign-extends when widened): mirror that
inline int __builtin_amdgcn_readfirstlane(int v) {
  return static_cast<int>(emu::exchange(static_cast<uint32_t>(v), 0));
}
inline uint32_t __builtin_amdgcn_alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
  return static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | lo) >> (8 * (s & 3)));
}
// v_perm_b32: byte n of the result = byte sel_n of {S0:S1} (0-3 -> S1, 4-7 -> S0),
// 12 -> 0x00, >= 13 -> 0xff (8-11, sign replication, unused here)
inline uint32_t __builtin_amdgcn_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t v = (static_cast<uint64_t>(s0) << 32) | s1;
  uint32_t r = 0;
  for (int n = 0; n < 4; ++n) {
    const uint32_t b = (sel >> (8 * n)) & 0xffu;
    const uint32_t byte = b < 8 ? static_cast<uint32_t>(v >> (8 * b)) & 0xffu : b == 12 ? 0u : 0xffu;
    r |= byte << (8 * n);
  }
  return r;
}
// v_bitop3_b32: bit i of the result = bit ((a_i << 2) | (b_i << 1) | c_i) of imm
inline uint32_t __builtin_amdgcn_bitop3_b32(uint32_t a, uint32_t b, uint32_t c, uint32_t imm) {
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) {
    const uint32_t idx = (((a >> i) & 1u) << 2) | (((b >> i) & 1u) << 1) | ((c >> i) & 1u);
    r |= ((imm >> idx) & 1u) << i;
  }
  return r;
}
inline int __builtin_amdgcn_readlane(int v, int l) {
  return static_cast<int>(emu::exchange(static_cast<uint32_t>(v), static_cast<uint32_t>(l)));
}
inline unsigned long long __ballot(int pred) {
  emu::Wave& w = emu::tl_group->waves[emu::tl_tid.x >> 6];
  const uint32_t lane = emu::tl_tid.x & 63;
  w.slot[lane] = pred ? 1u : 0u;
  w.bar->arrive_and_wait();
  unsigned long long m = 0;
  for (uint32_t l = 0; l < 64; ++l) m |= static_cast<unsigned long long>(w.slot[l] & 1u) << l;
  w.bar->arrive_and_wait();
  return m;
}
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline int __ffsll(long long v) { return __builtin_ffsll(v); }
// v_mbcnt_lo / hi: acc + the bits of mask below this lane (lo: lanes 0..31 of
// the mask, hi: lanes 32..63)
inline uint32_t __builtin_amdgcn_mbcnt_lo(uint32_t m, uint32_t acc) {
  const uint32_t lane = emu::tl_tid.x & 63;
  return acc + static_cast<uint32_t>(__builtin_popcount(lane >= 32 ? m : m & ((1u << lane) - 1u)));
}
inline uint32_t __builtin_amdgcn_mbcnt_hi(uint32_t m, uint32_t acc) {
  const uint32_t lane = emu::tl_tid.x & 63;
  return acc + (lane < 32 ? 0u : static_cast<uint32_t>(__builtin_popcount(m & ((1u << (lane - 32)) - 1u))));
}
// ds_bpermute_b32 (pull): this lane reads lane (addr / 4) % 64's data
inline int __builtin_amdgcn_ds_bpermute(int addr, int data) {
  return static_cast<int>(emu::exchange(static_cast<uint32_t>(data),
                                        (static_cast<uint32_t>(addr) >> 2) & 63u));
}
// ds_permute_b32 (push): lane (addr / 4) % 64 receives this lane's data; a
// lane nobody writes gets 0 (callers here always form a permutation)
inline int __builtin_amdgcn_ds_permute(int addr, int data) {
  emu::Wave& w = emu::tl_group->waves[emu::tl_tid.x >> 6];
  const uint32_t lane = emu::tl_tid.x & 63;
  const uint32_t n = std::min<uint32_t>(64, emu::g_block.x - 64 * (emu::tl_tid.x >> 6));
  w.slot[lane] = (static_cast<uint32_t>(addr) >> 2) & 63u;
  w.bar->arrive_and_wait();
  uint32_t src = 64;
  for (uint32_t l = 0; l < n; ++l)
    if (w.slot[l] == lane) src = l;
  w.bar->arrive_and_wait();
  const uint32_t v = emu::exchange(static_cast<uint32_t>(data), src < 64 ? src : lane);
  return static_cast<int>(src < 64 ? v : 0u);
}
// DPP: row_shr:n (0x111..0x11f; lane i <- lane i-n in its row, else `old`)
// and row_ror:n (0x121..0x12f; lane i <- lane (i-n) mod 16 of its row)
inline uint32_t __builtin_amdgcn_update_dpp(uint32_t old, uint32_t src, int ctrl, int, int, bool) {
  const uint32_t lane = emu::tl_tid.x & 63;
  if (ctrl >= 0 && ctrl < 0x100) {  // quad_perm:[s0,s1,s2,s3] (lane i <- lane sel_{i%4} of its quad)
    const uint32_t sel = (static_cast<uint32_t>(ctrl) >> (2 * (lane & 3u))) & 3u;
    return emu::exchange(src, (lane & ~3u) | sel);
  }
  if (ctrl > 0x110 && ctrl < 0x120) {
    const uint32_t n = static_cast<uint32_t>(ctrl - 0x110);
    const uint32_t v = emu::exchange(src, (lane & 15u) >= n ? lane - n : lane);
    return (lane & 15u) >= n ? v : old;
  }
  const uint32_t n = static_cast<uint32_t>(ctrl - 0x120) & 15;
  return emu::exchange(src, (lane & ~15u) | ((lane - n) & 15u));
}
// v_mov_b32_dpp with bound_ctrl: lanes without a source lane get 0
inline uint32_t __builtin_amdgcn_mov_dpp(uint32_t src, int ctrl, int rm, int bm, bool) {
  return __builtin_amdgcn_update_dpp(0u, src, ctrl, rm, bm, true);
}
typedef uint32_t emu_u32x2 __attribute__((ext_vector_type(2)));
// v_permlane16_swap / v_permlane32_swap: swap odd 16-lane rows (upper 32-lane
// half) of `old` with even rows (lower half) of `src`; returns {old', src'}
inline emu_u32x2 __builtin_amdgcn_permlane16_swap(uint32_t old, uint32_t src, bool, bool) {
  const uint32_t lane = emu::tl_tid.x & 63;
  const uint32_t o_partner = emu::exchange(old, lane ^ 16);
  const uint32_t s_partner = emu::exchange(src, lane ^ 16);
  const bool odd = (lane >> 4) & 1;
  emu_u32x2 r;
  r[0] = odd ? s_partner : old;  // odd rows of old <- even rows of src
  r[1] = odd ? src : o_partner;  // even rows of src <- odd rows of old
  return r;
}
inline emu_u32x2 __builtin_amdgcn_permlane32_swap(uint32_t old, uint32_t src, bool, bool) {
  const uint32_t lane = emu::tl_tid.x & 63;
  const uint32_t o_partner = emu::exchange(old, lane ^ 32);
  const uint32_t s_partner = emu::exchange(src, lane ^ 32);
  const bool hi = (lane >> 5) & 1;
  emu_u32x2 r;
  r[0] = hi ? s_partner : old;
  r[1] = hi ? src : o_partner;
  return r;
}
// scoped atomics (the scan's look-back words: clang's __hip_atomic_* builtins
// also compile for the host) and the wave sleep hint
#ifndef __HIP_MEMORY_SCOPE_AGENT
#define __HIP_MEMORY_SCOPE_AGENT 3
#endif
inline void __builtin_amdgcn_s_sleep(int) { std::this_thread::yield(); }
inline uint32_t atomicXor(uint32_t* p, uint32_t v) { return __atomic_fetch_xor(p, v, __ATOMIC_RELAXED); }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
}
inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { return __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }
inline uint32_t atomicOr(uint32_t* p, uint32_t v) { return __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
inline unsigned long long atomicMin(unsigned long long* p, unsigned long long v) {
  unsigned long long cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED)) {
  }
  return cur;
}

inline uint32_t atomicMin(uint32_t* p, uint32_t v) {
  uint32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED)) {
  }
  return cur;
}

// stream-ordered allocation / copies: host memory, everything synchronous
typedef void* hipMemPool_t;
constexpr hipError_t hipErrorInvalidDevice = 101;
constexpr hipError_t hipErrorInvalidValue = 1;
enum hipMemcpyKind { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2, hipMemcpyDeviceToDevice = 3 };
enum { hipMemAllocationTypePinned = 1, hipMemLocationTypeDevice = 1,
       hipMemPoolAttrReleaseThreshold = 4, hipMemPoolReuseAllowOpportunistic = 2,
       hipMemPoolReuseAllowInternalDependencies = 3 };
typedef int hipMemPoolAttr;
struct hipMemPoolProps {
  int allocType;
  int handleTypes;
  struct { int type; int id; } location;
  void* win32SecurityAttributes;
  size_t maxSize;
  unsigned char reserved[56];
};
inline hipError_t hipMemPoolCreate(hipMemPool_t* p, const hipMemPoolProps*) {
  *p = reinterpret_cast<hipMemPool_t>(1);
  return hipSuccess;
}
inline hipError_t hipMemPoolSetAttribute(hipMemPool_t, int, void*) { return hipSuccess; }
inline hipError_t hipMallocFromPoolAsync(void** p, size_t n, hipMemPool_t, hipStream_t) {
  *p = std::aligned_alloc(256, (n + 255) & ~size_t(255));
  return *p ? hipSuccess : 2;
}
inline hipError_t hipFreeAsync(void* p, hipStream_t) {
  std::free(p);
  return hipSuccess;
}
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
  std::memcpy(d, s, n);
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
// streams and events: launches run to completion in order, so these are no-ops
typedef void* hipEvent_t;
constexpr unsigned hipStreamNonBlocking = 1, hipEventDisableTiming = 2;
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
  static int dummy;
  *s = &dummy;
  return hipSuccess;
}
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  static int dummy;
  *e = &dummy;
  return hipSuccess;
}
inline hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
inline hipError_t hipStreamGetDevice(hipStream_t, int* d) {
  *d = 0;
  return hipSuccess;
}
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
inline hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
inline hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) {
  std::memset(d, v, n);
  return hipSuccess;
}

#define hipLaunchKernelGGL(K, G, B, SH, ST, ...) ::emu::launch(K, G, B, __VA_ARGS__)
template <typename K>
inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* n, K, int, size_t) {
  *n = 2;
  return hipSuccess;
}
