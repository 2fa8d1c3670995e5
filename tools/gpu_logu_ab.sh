#!/bin/bash
# tools/gpu_logu_ab.sh <tag>: CRC verify on SST-packed blocks with the C5
# record size mix (log-uniform 32 B..32 KiB), and with the small tail cut
# (>= 64 B: no serial short path; >= 1 KiB), rows vs v2
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-logu}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/ab_bench.py --config LOGU --config LOGU64 --config LOGU1K --rounds 3 \
  --var FORST_CRC_VARIANT= --var FORST_CRC_VARIANT=rows --var FORST_CRC_VARIANT=v2 > "$OUT/ab.log" 2>&1 \
  || { tail -20 "$OUT/ab.log"; exit 1; }
python3 tools/abfmt.py "$OUT/ab.log"
