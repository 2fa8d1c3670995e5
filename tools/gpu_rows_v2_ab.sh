#!/bin/bash
# tools/gpu_rows_v2_ab.sh <tag>: CRC rows vs v2 kernel on large / mixed blocks
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-rowsv2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/ab_bench.py --config NS16 --config C64 --config C3CRC --config C2 \
  --var FORST_CRC_VARIANT=rows --var FORST_CRC_VARIANT=v2 > "$OUT/ab.log" 2>&1 \
  || { tail -20 "$OUT/ab.log"; exit 1; }
python3 tools/abfmt.py "$OUT/ab.log"
