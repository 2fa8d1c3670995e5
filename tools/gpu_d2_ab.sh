#!/bin/bash
# tools/gpu_d2_ab.sh <tag>: CRC rows kernel with two steps in flight (rows_d2)
# vs the default: GPU parity under the variant, then A/B verify / compute.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-d2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
FORST_CRC_VARIANT=rows_d2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for m in verify compute; do
  timeout -k 10 300 python -u tools/ab_bench.py --config C2 --config NS16 --config C3CRC --mode $m \
    --var FORST_CRC_VARIANT= --var FORST_CRC_VARIANT=rows_d2 > "$OUT/ab_$m.log" 2>&1 \
    || { tail -20 "$OUT/ab_$m.log"; exit 1; }
  echo "== $m"
  python3 tools/abfmt.py "$OUT/ab_$m.log"
done
