#!/bin/bash
# A/B: fragment-aware XXH3 register budget (2 vs 3 waves per SIMD) on C5
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02e
mkdir -p "$OUT"
timeout -k 10 600 python -u tools/wal_ab.py FORST_FRAG_WPE=2 FORST_FRAG_WPE=3 > "$OUT/ab.log" 2>&1 || { tail -30 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
