#!/bin/bash
# new-component GPU tests: table writer, host-memory multi-device path,
# threaded shim, SST verify changes
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02b
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_table_writer.py tests/test_gpu_hostpath.py \
  tests/test_gpu_shim.py tests/test_sst.py tests/test_wal_recover.py -m gpu -x -v -s --timeout 240 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -5 "$OUT/pytest.log"
