#!/bin/bash
# SQ issue / wait counters for the C2 and C4 block kernels
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02g
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in C2 C4; do
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
  -d "$OUT/sq_$c" -o sq --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/sq_$c.log" 2>&1 || { tail -20 "$OUT/sq_$c.log"; exit 1; }
done
echo done
