#!/bin/bash
# tools/gpu_feed_ab.sh <tag>: GPU parity, then A/B of the rows kernels' work
# feed (dynamic chunks vs one static share per wave) on uniform and mixed
# block sizes, CRC rows vs v2 on mixed sizes, and the C5 WAL pipeline.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-feed}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --config NS16X --config C3 --config X4 \
  --var FORST_FEED= --var FORST_FEED=static > "$OUT/ab_feed.log" 2>&1 || { tail -20 "$OUT/ab_feed.log"; exit 1; }
cat "$OUT/ab_feed.log"
timeout -k 10 300 python -u tools/ab_bench.py --config C3CRC --config NS16 --config C64 \
  --var FORST_CRC_VARIANT= --var FORST_CRC_VARIANT=rows --var FORST_CRC_VARIANT=rows,FORST_FEED=static \
  > "$OUT/ab_crc.log" 2>&1 || { tail -20 "$OUT/ab_crc.log"; exit 1; }
cat "$OUT/ab_crc.log"
timeout -k 10 300 python -u tools/wal_ab.py FORST_FEED= FORST_FEED=static > "$OUT/wal.log" 2>&1 \
  || { tail -20 "$OUT/wal.log"; exit 1; }
cat "$OUT/wal.log"
