#!/bin/bash
# SQ issue / wait counters for bench configs and the C5 WAL set
# usage: tools/gpu_sq.sh <tag> [configs...]   (C5 = tools/prof_wal.py, KV = the a15_kv extra)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sq}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${*:-C2}; do
  if [ "$c" = C5 ]; then PROG="tools/prof_wal.py"; elif [ "$c" = KV ]; then PROG="bench.py --extra a15_kv --steps 5 --warmup 2"; else PROG="bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-extras"; fi
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
    -d "$OUT/sq_$c" -o sq --output-format csv -- python3 $PROG > "$OUT/sq_$c.log" 2>&1 || { tail -20 "$OUT/sq_$c.log"; exit 1; }
done
echo done
