#!/usr/bin/env python3
"""tools/prof_wal_writer.py -- C5 writer-side record CRCs two ways on one
build, alternating: forst_wal_record_crc_batch (descriptors from a pass over
the headers, a finish pass masks and stores) and forst_wal_record_crc_lengths
(the rows kernel's WAL writer mode: descriptors from the writer's lengths,
CRCs masked and stored in place by the kernel).  HIP events, median of 9
each; prints one JSON line with ms and the writer roofline fraction
(bench.run_wal's algorithmic bytes)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
w = workload.make_wal_batch(10_000_000, workload.SEEDS["C5"])
offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
lens = torch.from_numpy(w.rec_lengths.astype(np.int32)).cuda()
crc = torch.empty(len(w.rec_offsets), dtype=torch.uint32, device="cuda")
alg = int(w.rec_lengths.astype(np.int64).sum()) + 7 * len(w.rec_offsets) + 16 * len(w.rec_offsets)
ref = w.log.clone()
ts = {"headers": [], "lengths": [], "lengths_no_store": [], "headers_no_store": []}
for k in range(20):
    for name in ts:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        engine.wal_record_crc_batch(w.log, offs, write_in_place="no_store" not in name, out=crc,
                                    payload_lengths=lens if name.startswith("lengths") else None)
        e1.record()
        torch.cuda.synchronize()
        if k >= 2:
            ts[name].append(e0.elapsed_time(e1))
assert torch.equal(w.log, ref)
out = {}
for name, v in ts.items():
    ms = float(np.median(v))
    out[name] = {"ms": round(ms, 4), "frac": round(alg / (ms / 1e3) / 1e9 / bench.HBM_PEAK_GBS, 4)}
print(json.dumps(out), flush=True)
