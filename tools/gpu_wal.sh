#!/bin/bash
# WAL recovery on the GPU: its parity tests, the C5 WAL line (bench.run_wal), a kernel trace
# and the HBM PMC passes of tools/prof_wal.py
# usage: tools/gpu_wal.sh <tag> [pytest-k]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-x}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_wal_golden.py tests/test_wal_recover.py ${K:+-k "$K"} > "$OUT/pytest_wal.log" 2>&1 \
  || { tail -30 "$OUT/pytest_wal.log"; exit 1; }
tail -2 "$OUT/pytest_wal.log"
timeout -k 10 300 python -u tools/prof_wal.py > "$OUT/wal_C5.log" 2>&1 || { tail -20 "$OUT/wal_C5.log"; exit 1; }
tail -1 "$OUT/wal_C5.log"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
  -- python3 tools/prof_wal.py > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv \
  -- python3 tools/prof_wal.py > "$OUT/pmc_fetch.log" 2>&1 || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv \
  -- python3 tools/prof_wal.py > "$OUT/pmc_write.log" 2>&1 || { tail -20 "$OUT/pmc_write.log"; exit 1; }
echo done
