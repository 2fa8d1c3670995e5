#!/bin/bash
# profiles/profile.sh -- rocprofv3 evidence for bench.py (run on the GPU box):
#   1. --kernel-trace --stats          per-kernel durations (must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE                 HBM read traffic   (separate pass, guide §HBM)
#   3. --pmc WRITE_SIZE                 HBM write traffic  (separate pass)
# Usage: bash profiles/profile.sh <tag> [bench args...]
# Writes raw output under gpurun_out/prof_<tag>/; summarise with
#   python profiles/summarize.py <tag>
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
shift || true
ARGS=${*:---steps 5 --warmup 2 --no-cpu-baseline --no-extras}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv \
  -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv \
  -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv \
  -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
echo "profile $TAG done"
