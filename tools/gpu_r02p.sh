#!/bin/bash
# XXH3 finishing loads unconditional again; fragment kernel 2 vs 3 waves/SIMD
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02p
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_recover.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 600 python -u tools/wal_ab.py FORST_FRAG_WPE=2 FORST_FRAG_WPE=3 > "$OUT/ab.log" 2>&1 || { tail -30 "$OUT/ab.log"; exit 1; }
cat "$OUT/ab.log"
bash tools/gpu_bench_cfgs.sh r02p C3 NS16X
