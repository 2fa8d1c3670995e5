#!/bin/bash
# fragment-aware record XXH3: a14 + recovery parity on the GPU, then the C5
# WAL line and its kernel trace
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02d
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "record_xxh3 or full_size" tests/test_wal_recover.py -m gpu > "$OUT/tests.log" 2>&1 \
  || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 300 python -u tools/prof_wal.py > "$OUT/wal.json" 2> "$OUT/wal.err" || { tail -20 "$OUT/wal.err"; exit 1; }
cat "$OUT/wal.json"
bash profiles/profile.sh r02d C5 || { tail -30 gpurun_out/prof_r02d_C5/*.log; exit 1; }
