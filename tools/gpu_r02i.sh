#!/bin/bash
# A/B of the CRC kernel variants after gating the per-step descriptor work
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02i
mkdir -p "$OUT"
for c in C2 NS16 C4; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $c --var FORST_CRC_VARIANT=rows --var FORST_CRC_VARIANT=rows_d2 --var FORST_CRC_VARIANT=v2 --var FORST_CRC_VARIANT=rows_probe_load > "$OUT/ab_$c.log" 2>&1 || { tail -20 "$OUT/ab_$c.log"; exit 1; }
  tail -6 "$OUT/ab_$c.log"
done
