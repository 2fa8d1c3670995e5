#!/bin/bash
# Issue / memory-pipeline counters (two --pmc passes, each within the per-block
# limits) for bench configs and the C5 WAL set.
# usage: tools/gpu_pmc2.sh <tag> [configs...]   (C5 = tools/prof_wal.py)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pmc2}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ"
for c in ${*:-C2}; do
  if [ "$c" = C5 ]; then PROG="tools/prof_wal.py"; else PROG="bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-extras"; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P -d "$OUT/p${i}_$c" -o p --output-format csv -- python3 $PROG > "$OUT/p${i}_$c.log" 2>&1 || { tail -20 "$OUT/p${i}_$c.log"; exit 1; }
  done
done
echo done
