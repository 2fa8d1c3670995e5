#!/bin/bash
# tools/gpu_c4_ab.sh <tag>: C4 (512 K x 16 KiB: two 64-block chunks per wave)
# rows vs v2 / v1, and NS16 for reference
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --config NS16 --var FORST_CRC_VARIANT=rows \
  --var FORST_CRC_VARIANT=v2 > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
timeout -k 10 300 python -u tools/ab_bench.py --config C4X --var FORST_XXH3_VARIANT= \
  --var FORST_XXH3_VARIANT=v1 > "$OUT/abx.log" 2>&1 || { tail -20 "$OUT/abx.log"; exit 1; }
python3 tools/abfmt.py "$OUT/ab.log" "$OUT/abx.log"
