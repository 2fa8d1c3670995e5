#!/bin/bash
# tools/gpu_wal_prof.sh <tag>: C5 WAL A/B (pipeline vs CRC kernel variants vs
# the per-block wave kernel) and a rocprofv3 kernel trace of the default path.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-wal}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
[ -n "$NO_AB" ] || timeout -k 10 400 python -u tools/wal_ab.py FORST_WAL_VARIANT= FORST_CRC_VARIANT=v2 \
  FORST_CRC_VARIANT=rows FORST_WAL_VARIANT=wave > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
[ -n "$NO_AB" ] || cat "$OUT/ab.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 -c "import sys; sys.path.insert(0, '.'); import bench; from forst_amd import engine; engine.init_device(); print(bench.run_wal(5, 1))" \
  > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
PY
