#!/bin/bash
# tools/gpu_slide_ab.sh <tag>: GPU parity + verify / compute rates after a
# rows-kernel change (compare against the previous round of logs)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-slide}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for m in verify compute; do
  timeout -k 10 300 python -u tools/ab_bench.py --config C2 --config NS16 --config X4 --config NS16X \
    --config C3 --mode $m --var FORST_CRC_VARIANT= --var FORST_CRC_VARIANT=rows_probe_load \
    > "$OUT/ab_$m.log" 2>&1 || { tail -20 "$OUT/ab_$m.log"; exit 1; }
  echo "== $m"
  python3 tools/abfmt.py "$OUT/ab_$m.log"
done
