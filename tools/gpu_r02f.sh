#!/bin/bash
# SQ counters (issue / wait breakdown) for the C5 WAL kernels
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02f
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -o "SQ_[A-Z_]*" "$OUT/counters.txt" | sort -u > "$OUT/sq_names.txt" || true
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU \
  -d "$OUT/sq" -o sq --output-format csv -- python3 tools/prof_wal.py > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
echo done
