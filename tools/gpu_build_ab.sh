#!/bin/bash
# tools/gpu_build_ab.sh <tag> <other.so>: A/B of two builds of the library
# (in-tree vs FORST_LIB_PATH=<other.so>), alternating processes, 3 rounds
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
TAG=${1:-buildab}
OTHER=${2:-forst_amd/lib_ab/libforst_checksum_prev.so}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CFG="--config C2 --config NS16 --config X4 --config C3 --rounds 3 --reps 5"
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_bench.py $CFG > "$OUT/new_$r.log" 2>&1 || { tail -20 "$OUT/new_$r.log"; exit 1; }
  FORST_LIB_PATH=$OTHER timeout -k 10 300 python -u tools/ab_bench.py $CFG > "$OUT/old_$r.log" 2>&1 \
    || { tail -20 "$OUT/old_$r.log"; exit 1; }
done
for r in 1 2 3; do echo "== round $r new"; python3 tools/abfmt.py "$OUT/new_$r.log"; echo "== round $r prev"; python3 tools/abfmt.py "$OUT/old_$r.log"; done
