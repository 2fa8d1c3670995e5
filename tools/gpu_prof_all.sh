#!/bin/bash
# rocprofv3 evidence for every configuration at the current build:
# kernel trace + FETCH_SIZE + WRITE_SIZE passes (profiles/profile.sh)
#   tools/gpu_prof_all.sh <tag> [configs...]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02}; shift || true
for c in ${*:-C2 NS16 NS16X C3 C4 C5}; do
  bash profiles/profile.sh $TAG $c || { tail -30 gpurun_out/prof_${TAG}_$c/*.log; exit 1; }
done
