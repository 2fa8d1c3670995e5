#!/usr/bin/env python3
"""tools/prof_a14.py -- A/B timing of the C5 a14 record XXH3 and the fused
recovery alone (no result checks: timing-only kernel variants of the
diagnostics builds run through it).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
w = workload.make_wal_batch(10_000_000, workload.SEEDS["C5"])
offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 3)


a14 = timed(lambda: engine.wal_record_xxh3_batch(w.log, offs))
rec = timed(lambda: engine.wal_recover_batch(w.log, 0, engine.kPointInTimeRecovery,
                                             record_capacity=w.n_records + 1024))
print(json.dumps({"a14_ms": a14, "recover_ms": rec}), flush=True)
