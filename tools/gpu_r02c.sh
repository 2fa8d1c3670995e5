#!/bin/bash
# default bench line (with host-memory + recovery extras), then rocprofv3
# evidence for C2 and C5
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02c
mkdir -p "$OUT"
timeout -k 10 700 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
for c in C2 C5; do
  bash profiles/profile.sh r02c $c || { tail -30 gpurun_out/prof_r02c_$c/*.log; exit 1; }
done
