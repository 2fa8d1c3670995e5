#!/bin/bash
# guided chunk sizes in the work feed: parity, tail profile, A/B vs the
# previous product build (lib/libforst_checksum_old.so)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02gss}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_wal_recover.py tests/test_gpu_shim.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 300 python -u tools/wave_tail.py --config C2 --config NS16 > "$OUT/tail.log" 2>&1 || { tail -20 "$OUT/tail.log"; exit 1; }
grep '^{"' "$OUT/tail.log" | cut -c1-400
bash tools/ab_libs.sh ${TAG:-r02gss} forst_amd/lib/libforst_checksum_old.so forst_amd/lib/libforst_checksum.so ${CFGS:-C2 NS16 NS16X C3 C5}
