#!/bin/bash
# tools/gpu_a14_prof.sh <tag>: rocprofv3 kernel trace of the C5 logical-record
# XXH3 path (forst_wal_record_xxh3_batch)
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-a14}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 -c "
import sys; sys.path.insert(0, '.')
import numpy as np, torch
from forst_amd import engine, workload
engine.init_device()
w = workload.make_wal_batch(10_000_000, workload.SEEDS['C5'])
offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
for _ in range(3):
    h, f = engine.wal_record_xxh3_batch(w.log, offs)
torch.cuda.synchronize()
print('n', h.numel())
" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
PY
