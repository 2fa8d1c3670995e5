#!/bin/bash
# bench.py lines for the block configurations (no extras) + SQ counters for C2
# usage: tools/gpu_bench_cfgs.sh <tag> [configs...]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-x}; shift || true
CFGS=${*:-C2 NS16 C4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-extras > "$OUT/bench_$c.log" 2>&1 || { tail -20 "$OUT/bench_$c.log"; exit 1; }
  tail -1 "$OUT/bench_$c.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['unit'], {k: (v['name'][:22], v['avg_ms'], v['frac']) for k, v in d['kernels'].items()})" || tail -2 "$OUT/bench_$c.log"
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
  -d "$OUT/sq_C2" -o sq --output-format csv -- python3 bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/sq_C2.log" 2>&1 || { tail -20 "$OUT/sq_C2.log"; exit 1; }
echo done
