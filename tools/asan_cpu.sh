#!/bin/bash
# tools/asan_cpu.sh -- the host C++ under AddressSanitizer + UndefinedBehavior-
# Sanitizer, on the CPU (no GPU sanitizer exists here, and none is needed: the
# parsers of untrusted file bytes are host code):
#   1. lib/libforst_checksum_asan.so (make -C forst_amd/csrc asan: sst_host.cc,
#      block_codecs.cc, wal_host.cc, table_writer.cc, host_batch.cc and both
#      shims built with -fsanitize=address,undefined) runs the CPU tests of
#      those files and the corrupted-input corpus (tests/test_host_corpus.py);
#   2. the SIMT emulator (tests/emu, the kernel sources compiled as host C++)
#      built with EMU_SANITIZE=1 runs the emulator kernel tests.
# Any sanitizer report aborts the run (halt_on_error, -fno-sanitize-recover).
set -eo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-/tmp/forst_asan}
mkdir -p "$OUT"
make -s -C forst_amd/csrc asan
ASAN_RT=$(g++ -print-file-name=libasan.so)
UBSAN_RT=$(g++ -print-file-name=libubsan.so)
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
FORST_TEST_LIB=$PWD/forst_amd/lib/libforst_checksum_asan.so LD_PRELOAD="$ASAN_RT $UBSAN_RT" \
  python -m pytest -x -q -p no:cacheprovider -m "not gpu" \
  tests/test_sst.py tests/test_block_codecs.py tests/test_table_writer.py tests/test_capi_cpu.py \
  tests/test_host_corpus.py tests/test_sst_pinned.py > "$OUT/host.log" 2>&1 \
  || { tail -60 "$OUT/host.log"; exit 1; }
tail -1 "$OUT/host.log"
CLANG_RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so 2>/dev/null | head -1)
EMU_SANITIZE=1 LD_PRELOAD="$CLANG_RT" python -m pytest -x -q -p no:cacheprovider \
  tests/test_emu_kernels.py > "$OUT/emu.log" 2>&1 || { tail -60 "$OUT/emu.log"; exit 1; }
tail -1 "$OUT/emu.log"
