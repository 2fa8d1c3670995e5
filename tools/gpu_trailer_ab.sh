#!/bin/bash
# tools/gpu_trailer_ab.sh <tag>: where the write-side (trailer) kernel loses
# time against verify: compute with last_bytes[] (trailer minus stores),
# compute with the type byte from memory, trailer, verify -- rows vs v2.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-trailer}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for m in trailer; do
  timeout -k 10 200 python -u tools/ab_bench.py --config C2 --mode $m --var FORST_CRC_VARIANT=,FORST_TRAILER=fused \
    --var FORST_CRC_VARIANT=,FORST_TRAILER=,FORST_SCATTER= --var FORST_CRC_VARIANT=,FORST_TRAILER=,FORST_SCATTER=rmw > "$OUT/ab_$m.log" 2>&1 || { tail -20 "$OUT/ab_$m.log"; exit 1; }
  echo "== $m"
  python3 tools/abfmt.py "$OUT/ab_$m.log"
done
