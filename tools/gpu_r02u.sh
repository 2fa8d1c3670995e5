#!/bin/bash
# C5 kernel trace + SQ counters at the current build (frag kernel issue rewrite)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02u
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 tools/prof_wal.py > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 1; }
bash tools/gpu_sq.sh r02u C5
