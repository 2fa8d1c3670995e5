#!/bin/bash
# a14 / recovery with the compact gathered batch: parity + C5 timing + kernel trace
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02n
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wal or record" tests/test_wal_recover.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u tools/prof_wal.py > "$OUT/wal.json" 2> "$OUT/wal.err" || { tail -20 "$OUT/wal.err"; exit 1; }
cat "$OUT/wal.json"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 tools/prof_wal.py > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
echo done
