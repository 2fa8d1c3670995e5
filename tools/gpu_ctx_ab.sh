#!/bin/bash
# tools/gpu_ctx_ab.sh <tag>: verify-kernel time on C2 in different contexts
# (verify only, + computed[] stores, after a trailer pass as in bench.py)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-ctx}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for m in "--mode verify" "--mode verify --computed" "--mode pair" "--mode pair --computed" "--mode trailer"; do
  echo "== $m"
  timeout -k 10 200 python -u tools/ab_bench.py --config C2 --config NS16X $m > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
  python3 -c "
import json,sys; t=open('$OUT/ab.log').read(); j=json.loads(t[t.index('{'):])
for k,v in j.items(): print(f\"{k:30s} {v['median_ms']:8.3f} ms frac {v['roofline_frac_median']}\")"
done
