#!/bin/bash
# tools/pmc_sq.sh <tag> <config> [variant env] -- SQ counter passes (one run
# each, rocprofv3 --pmc) over tools/ab_bench.py (verify kernel).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; CFG=$2; VAR=${3:-}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD"
P3="SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INSTS_WAVE32"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 tools/ab_bench.py --config $CFG --rounds 1 --reps 3 ${VAR:+--var $VAR} > "$OUT/p$i.log" 2>&1 \
    || { tail -20 "$OUT/p$i.log"; exit 1; }
done
echo "pmc $TAG done"
