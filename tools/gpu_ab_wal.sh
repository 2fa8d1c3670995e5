#!/bin/bash
# WAL GPU parity (record XXH3, recovery vs the reference fixtures, full-size
# C5 properties) then a C5 A/B of two library builds
#   tools/gpu_ab_wal.sh <tag> <lib A> <lib B>
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; A=$2; B=$3
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wal_golden.py tests/test_wal_recover.py tests/test_gpu_parity.py -k "wal or xxh3 or frag or recover or C5" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/ab_multi.sh $TAG C5 $A $B
