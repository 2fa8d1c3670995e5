#!/bin/bash
# round-end evidence at the current build: the whole -m gpu suite and smoke,
# rocprofv3 kernel trace + FETCH/WRITE passes for every config, then the full
# default bench line.  TAG names the profiles (profiles/pmc_<TAG>_*.json sort
# after the previous ones, so bench.py reads these).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r02z2}
OUT=gpurun_out/final_$TAG
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
if [ -z "$NOPROF" ]; then
  bash tools/gpu_prof_all.sh $TAG ${CFGS:-C2 NS16 NS16X C3 C4 C5}
fi
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
