#!/usr/bin/env python3
"""tools/prof_recover_shape.py <shape> -- forst_wal_recover_batch (PIT) on a
~44 GiB log of a given record-length shape, 5 timed calls after 2 untimed:
  c5        C5's log-uniform 32 B - 32 KiB lengths (bench.run_wal)
  u<L>      every record L bytes (same log size as C5)
  sorted    C5's lengths sorted (records of equal size next to each other)
Prints one JSON line (median ms, records, log bytes).  Run under rocprofv3
--kernel-trace --stats to split the time by kernel (measurement aid for the
fused recovery kernel's per-record finish cost)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
shape = sys.argv[1] if len(sys.argv) > 1 else "c5"
seed = workload.SEEDS["C5"]
c5 = workload.log_uniform_lengths(10_000_000, 32, 32768, seed)
total = int(c5.astype(np.int64).sum())
if shape == "c5":
    lens = c5
elif shape == "sorted":
    lens = np.sort(c5)
else:
    L = int(shape[1:])
    lens = np.full(total // L, L, dtype=np.uint32)
w = workload.make_wal_batch(0, seed, lengths=lens)
for _ in range(2):
    engine.wal_recover_batch(w.log, 0, engine.kPointInTimeRecovery,
                             record_capacity=len(lens) + 1024)
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rec, rep, res = engine.wal_recover_batch(w.log, 0, engine.kPointInTimeRecovery,
                                             record_capacity=len(lens) + 1024)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
assert res.n_records == len(lens) and res.n_reports == 0
print(json.dumps({"shape": shape, "records": len(lens), "physical": int(res.n_physical),
                  "log_bytes": w.total, "recover_ms": round(float(np.median(ts)) * 1e3, 3)}),
      flush=True)
