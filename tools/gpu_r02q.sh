#!/bin/bash
# rocprofv3 evidence for every configuration at the current build:
# kernel trace + FETCH_SIZE + WRITE_SIZE passes (profiles/profile.sh)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in C2 NS16 NS16X C3 C4 C5; do
  bash profiles/profile.sh r02q $c || { tail -30 gpurun_out/prof_r02q_$c/*.log; exit 1; }
done
