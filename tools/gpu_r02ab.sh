#!/bin/bash
# parity (GPU suite: crc / wal / shim) at the current build, then an A/B of the
# product build against a baseline build (LIB_B, default the previous HEAD's
# lib/libforst_checksum_old.so), alternating processes on one box
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r02ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_wal_recover.py} -m gpu > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
bash tools/ab_libs.sh $TAG forst_amd/lib/libforst_checksum_old.so forst_amd/lib/libforst_checksum.so ${CFGS:-C2 NS16 C5}
