// tests/emu/emu_globals.cc -- TEST INFRASTRUCTURE ONLY (SIMT emulator state).
#include "hip/hip_runtime.h"

namespace emu {
thread_local dim3 tl_tid;
thread_local dim3 tl_bid;
thread_local Group* tl_group = nullptr;
dim3 g_grid, g_block;
}  // namespace emu
