#!/bin/bash
# tests/emu/build_emu.sh <out.so> -- TEST INFRASTRUCTURE ONLY.
# Compiles the unmodified kernel sources as host C++ against the SIMT emulator
# header (tests/emu/hip/hip_runtime.h) into a CPU-only library exposing the
# same C ABI as forst_amd/lib/libforst_checksum.so.
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT=${1:-/tmp/libforst_emu.so}
CXX=${CXX_EMU:-/opt/rocm/llvm/bin/clang++}
# EMU_DEFINES: extra -D options (the kernels' build knobs, e.g. -DFORST_FRAG_K=8)
# EMU_SANITIZE=1: build under -fsanitize=address,undefined (tools/asan_cpu.sh)
SAN=""
if [ -n "${EMU_SANITIZE:-}" ]; then
  SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libasan"
fi
"$CXX" -std=c++20 -O1 -g -fPIC -shared -w $SAN -I"$HERE" -I"$ROOT/include" -include hip/hip_runtime.h -DFORST_HOST_EMULATION ${EMU_DEFINES:-} \
  -x c++ "$ROOT/forst_amd/csrc/crc32c.hip" "$ROOT/forst_amd/csrc/xxh3.hip" "$ROOT/forst_amd/csrc/xxhash_legacy.hip" "$ROOT/forst_amd/csrc/kv_protect.hip" "$ROOT/forst_amd/csrc/kv_sites.hip" "$ROOT/forst_amd/csrc/wal.hip" "$ROOT/forst_amd/csrc/wal_recover.hip" "$ROOT/forst_amd/csrc/crc_combine.hip" \
  "$ROOT/forst_amd/csrc/capi.hip" "$HERE/emu_globals.cc" -o "$OUT" -lpthread
echo "$OUT"
