#!/usr/bin/env python3
"""tools/prof_c5_split.py -- what the C5 records of each size class cost the
raw CRC32C rows kernel (forst_crc32c_batch over the physical records'
header[6..] + payload, as the WAL verify / writer paths run it): all records,
then only the records of each class, HIP events, median of 9.  Prints one
JSON line.  (Measurement aid for the small-record path)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
w = workload.make_wal_batch(10_000_000, workload.SEEDS["C5"])
offs = w.rec_offsets.astype(np.int64) + 6   # the CRC covers header[6..7) + payload
lens = w.rec_lengths.astype(np.int64) + 1


def timed(sel, order=None):
    oo, nn = offs[sel], lens[sel]
    if order is not None:  # descriptors reordered (binning experiments)
        k = order(nn)
        oo, nn = oo[k], nn[k]
    o = torch.from_numpy(np.ascontiguousarray(oo)).cuda()
    n = torch.from_numpy(np.ascontiguousarray(nn).astype(np.int32)).cuda()
    out = torch.empty(len(o), dtype=torch.uint32, device="cuda")
    for _ in range(2):
        engine.crc32c_batch(w.log, o, n, out=out)
    ts = []
    for _ in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        engine.crc32c_batch(w.log, o, n, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return {"n": int(len(o)), "bytes": int(lens[sel].sum()), "ms": round(float(np.median(ts)), 4),
            "kernel": engine.last_kernel()}


res = {"all": timed(np.ones(len(offs), bool))}
for lo, hi in ((0, 64), (64, 128), (128, 256), (256, 512), (512, 1024), (1024, 1 << 20)):
    res[f"{lo}-{hi}"] = timed((lens > lo) & (lens <= hi))
everything = np.ones(len(offs), bool)
# descriptors grouped by 1 KiB round count (stable: log order within a group)
res["by_rounds"] = timed(everything, lambda nn: np.argsort((nn + 1023) // 1024, kind="stable"))
# ... and in groups of 64 descriptors sorted by round count (a local sort)
res["by_rounds_local64"] = timed(everything, lambda nn: np.argsort(
    (np.arange(len(nn)) // 64) * 64 + (nn + 1023) // 1024, kind="stable"))
res["by_rounds_desc"] = timed(everything, lambda nn: np.argsort(-((nn + 1023) // 1024),
                                                                kind="stable"))
res["by_len"] = timed(everything, lambda nn: np.argsort(nn, kind="stable"))
res["le512"] = timed(lens <= 512)
res["gt512"] = timed(lens > 512)
print(json.dumps(res), flush=True)
