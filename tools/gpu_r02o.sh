#!/bin/bash
# CRC rows kernel with the head as a chain reset and immediate-offset loads:
# parity, then C2 / NS16 / C5 and the SQ counters of C2 and C5
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02o
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_recover.py tests/test_table_writer.py tests/test_sst.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u tools/prof_wal.py > "$OUT/wal.json" 2> "$OUT/wal.err" || { tail -20 "$OUT/wal.err"; exit 1; }
cat "$OUT/wal.json"
bash tools/gpu_bench_cfgs.sh r02o C2 NS16
bash tools/gpu_sq.sh r02o_sq C5
