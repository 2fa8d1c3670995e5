#!/bin/bash
# memory-side ceilings of the rows CRC kernel: one vs two steps of loads in flight
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02k
mkdir -p "$OUT"
for c in C2 NS16; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $c --var FORST_CRC_VARIANT=rows_probe_load --var FORST_CRC_VARIANT=rows_probe_contig --var FORST_CRC_VARIANT=probe_load > "$OUT/ab_$c.log" 2>&1 || { tail -20 "$OUT/ab_$c.log"; exit 1; }
done
echo ok
