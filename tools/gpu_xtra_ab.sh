#!/bin/bash
# tools/gpu_xtra_ab.sh <tag>: GPU parity, then C2 / X4 A/B of the default CRC
# path against its load-only probe and the v2 kernel (verify and trailer).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-xtra}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --config X4 --var FORST_CRC_VARIANT= \
  --var FORST_CRC_VARIANT=rows_probe_load --var FORST_CRC_VARIANT=v2 > "$OUT/ab.log" 2>&1 \
  || { tail -20 "$OUT/ab.log"; exit 1; }
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --mode trailer --var FORST_CRC_VARIANT= \
  --var FORST_CRC_VARIANT=v2 > "$OUT/ab_tr.log" 2>&1 || { tail -20 "$OUT/ab_tr.log"; exit 1; }
python3 tools/abfmt.py "$OUT/ab.log" "$OUT/ab_tr.log"
