#!/bin/bash
# evidence at the current build: the whole -m gpu suite and smoke,
# rocprofv3 kernel trace + FETCH/WRITE passes for the configs (C5 split by
# call site), then the default bench line.  TAG names the profiles.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06z}
OUT=gpurun_out/final_$TAG
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=30 > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
if [ -z "$NOPROF" ]; then
  for c in ${CFGS:-C2 NS16 NS16X C3 C3S C4 C5A14 C5REC C5VER C5WRI KV NS16H32 NS16H64}; do
    bash profiles/profile.sh $TAG $c || { tail -30 gpurun_out/prof_${TAG}_$c/*.log; exit 1; }
  done
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 900 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log"
fi
