#!/bin/bash
# tools/gpu_kv_ab.sh -- a15 parity (kv + call-site tests) on the product build,
# then the a15_kv bench through each A/B library given in $LIBS.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/kvab_${TAG:-x}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_kv_sites.py tests/test_gpu_parity.py -k "kv or hash64 or memtable or write_batch or block_kv" \
  -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  for L in ${LIBS:-}; do
    timeout -k 10 120 python -u tools/ab_kv.py forst_amd/lib/libforst_checksum_$L.so $L >> "$OUT/ab.jsonl" 2> "$OUT/ab_$L.err" || { tail -20 "$OUT/ab_$L.err"; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    r = json.loads(l); print(r['lib'], r['protect_ms'], r['verify_ms'], r['protect_roofline_frac'], r['verify_roofline_frac'])
"
