#!/bin/bash
# kernel trace of the C5 a14 + recovery calls alone (tools/prof_a14.py)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-tr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 tools/prof_a14.py > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 1; }
grep a14_ms "$OUT/kt.log"
