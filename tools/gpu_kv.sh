#!/bin/bash
# tools/gpu_kv.sh -- a15 iteration on the GPU box: the kv / hash64 parity tests,
# the a15_kv bench extra, its kernel trace + FETCH/WRITE (profiles/profile.sh KV)
# and, with SQ=1, the SQ counter passes of the same program.  TAG names the run.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06kv}
OUT=gpurun_out/kv_$TAG
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "kv or hash64" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
timeout -k 10 200 python -u bench.py --extra a15_kv --steps 20 --warmup 3 > "$OUT/bench.log" 2>&1 \
  || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
if [ -z "$NOPROF" ]; then
  bash profiles/profile.sh $TAG KV
fi
if [ -n "$SQ" ]; then
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD"
  P3="SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INSTS_WAVE32"
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P -d "gpurun_out/pmc_$TAG/p$i" -o p$i --output-format csv -- \
      python3 bench.py --extra a15_kv --steps 5 --warmup 1 > "$OUT/sq$i.log" 2>&1 \
      || { tail -20 "$OUT/sq$i.log"; exit 1; }
  done
  python3 tools/pmc_summary.py $TAG "kv_kernel<protect>" 1048576 > "$OUT/sq_protect.txt"
  python3 tools/pmc_summary.py $TAG "kv_kernel<verify>" 1048576 > "$OUT/sq_verify.txt"
  cat "$OUT/sq_protect.txt"
fi
echo "kv $TAG done"
