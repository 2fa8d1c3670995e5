#!/bin/bash
# WAL suites at the current build, then A/B of recovery against a base build
#   tools/gpu_ab_rec.sh <base.so>
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab_rec
timeout -k 10 400 python -u -m pytest tests/test_wal_recover.py tests/test_wal_golden.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_rec/pytest.log 2>&1 || { tail -30 gpurun_out/ab_rec/pytest.log; exit 1; }
tail -1 gpurun_out/ab_rec/pytest.log
bash tools/ab_multi.sh ab_rec C5 "$1" forst_amd/lib/libforst_checksum.so
bash tools/ab_multi.sh ab_rec SW "$1" forst_amd/lib/libforst_checksum.so
