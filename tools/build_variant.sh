#!/bin/bash
# A/B builds: forst_amd/lib/libforst_checksum_<name>.so = the current build with
# the given HIP sources recompiled under extra -D flags.
#   tools/build_variant.sh <name> "<src.hip> ..." -DFOO=1 ...
set -eo pipefail
cd "$(dirname "$0")/../forst_amd/csrc"
NAME=$1; SRCS=$2; shift 2
make -s -j8
D=build/v_$NAME
mkdir -p "$D"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics -fgpu-flush-denormals-to-zero"
OBJS=""
for o in build/*.o; do
  b=$(basename "$o" .o)
  if [[ " $SRCS " == *" $b.hip "* ]]; then
    /opt/rocm/bin/hipcc $FLAGS "$@" -c "$b.hip" -o "$D/$b.o"
    OBJS="$OBJS $D/$b.o"
  else
    OBJS="$OBJS $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libforst_checksum_$NAME.so $OBJS -lpthread -lz -ldl
echo "../lib/libforst_checksum_$NAME.so"
