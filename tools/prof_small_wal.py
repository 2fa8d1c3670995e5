#!/usr/bin/env python3
"""tools/prof_small_wal.py -- latency of small WAL writer-side CRC batches
(the raw rows kernel): logs of 1 K, 10 K and 100 K records log-uniform in
[32, 32768] B, HIP-event median of 50 calls each, no result checks (A/B of
builds through tools/with_lib.py).  Prints one JSON line: ms per batch."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
out = {}
for n in (1000, 10_000, 100_000):
    w = workload.make_wal_batch(n, workload.SEEDS["C5"])
    offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
    crc = torch.empty(len(w.rec_offsets), dtype=torch.uint32, device="cuda")
    for _ in range(3):
        engine.wal_record_crc_batch(w.log, offs, write_in_place=True, out=crc)
    ts = []
    for _ in range(50):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        engine.wal_record_crc_batch(w.log, offs, write_in_place=True, out=crc)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    out[f"write_{n}_ms"] = round(float(np.median(ts)), 4)
    out[f"kernel_{n}"] = engine.last_kernel()
print(json.dumps(out), flush=True)
