#!/bin/bash
# reference-pinned SST files on the GPU: verify, corruption text, writer rewrite, fv6 footers
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02s
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sst_pinned.py tests/test_sst.py tests/test_table_writer.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
