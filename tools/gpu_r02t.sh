#!/bin/bash
# frag-kernel issue rewrite: XXH3/WAL parity on the GPU, then C5 A/B of the
# frag kernel's register target (diag build)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r02t}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_recover.py -m gpu -k "xxh3 or wal or frag or short or recover or XXH3" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 600 python -u tools/wal_ab.py ${AB:-FORST_FRAG_WPE=3 FORST_FRAG_WPE=2 FORST_FRAG_WPE=3} > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
