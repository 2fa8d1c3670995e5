#!/bin/bash
# tools/gpu_x_ab.sh <tag>: XXH3 rows vs v1 kernel across block sizes
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-xab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/ab_bench.py --config X64 --config C3 --config NS16X --config X4 \
  --var FORST_XXH3_VARIANT= --var FORST_XXH3_VARIANT=v1 > "$OUT/ab.log" 2>&1 \
  || { tail -20 "$OUT/ab.log"; exit 1; }
python3 tools/abfmt.py "$OUT/ab.log"
