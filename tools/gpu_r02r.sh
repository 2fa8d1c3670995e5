#!/bin/bash
# the default bench line with every extra (host paths, configs, C5), as the driver runs it
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02r
mkdir -p "$OUT"
timeout -k 10 900 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']); print(json.dumps(d['extras'])[:3000])"
