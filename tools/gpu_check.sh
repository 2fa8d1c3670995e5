#!/bin/bash
# tools/gpu_check.sh -- one gpurun call: GPU parity tests, smoke, bench, A/B.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   gpurun --timeout 1100 -- bash tools/gpu_check.sh [tag]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
echo "== pytest -m gpu"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "== smoke"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
echo "== A/B stream vs simple"
timeout -k 10 240 python -u tools/ab_bench.py --config C2 --config NS16 --config NS16X --config C3 \
  --var FORST_CRC_VARIANT=,FORST_XXH3_VARIANT= \
  --var FORST_CRC_VARIANT=simple,FORST_XXH3_VARIANT=simple > "$OUT/ab.log" 2>&1 \
  || { tail -20 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
echo "done $TAG"
