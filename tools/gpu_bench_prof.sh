#!/bin/bash
# tools/gpu_bench_prof.sh <tag>: rocprofv3 evidence (kernel trace + FETCH/WRITE
# passes) for the default bench config, then the full default bench line.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
bash profiles/profile.sh "$TAG"
mkdir -p gpurun_out/bench_$TAG
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG/bench.log 2>&1 || { tail -20 gpurun_out/bench_$TAG/bench.log; exit 1; }
tail -1 gpurun_out/bench_$TAG/bench.log
