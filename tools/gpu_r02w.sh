#!/bin/bash
# loop restructure (both step copies issue on every path): parity, then bench
# lines for every block config and the C5 WAL set
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r02w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_recover.py tests/test_gpu_shim.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_bench_cfgs.sh ${TAG:-r02w} C2 NS16 NS16X C3 C4
timeout -k 10 300 python -u tools/prof_wal.py > "$OUT/wal.log" 2>&1 || { tail -20 "$OUT/wal.log"; exit 1; }
tail -1 "$OUT/wal.log"
