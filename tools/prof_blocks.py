#!/usr/bin/env python3
"""tools/prof_blocks.py <config> -- A/B timing of one block config's write side
(trailer pass) and read side (verify pass) alone, with no result checks, so
timing-only kernel variants of the A/B builds can run through it.  Prints one
JSON line: HIP-event ms per pass and the verify fraction of 8 TB/s."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
sizes, ctype, desc, seed = bench.describe(cfg, 1)
b = workload.make_sst_batch(len(sizes), None, seed, ctype=ctype, sizes=sizes)
ok = torch.empty(b.n, dtype=torch.uint8, device="cuda")
comp = torch.empty(b.n, dtype=torch.uint32, device="cuda")
bad = torch.zeros(1, dtype=torch.int64, device="cuda")
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(23)]
for k, e in enumerate(evs):
    e[0].record()
    engine.block_trailer_batch(ctype, b.base, b.offsets, b.sizes, b.types)
    e[1].record()
    engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes, computed=comp, stored=None, ok=ok,
                              mismatches=bad)
    e[2].record()
torch.cuda.synchronize()
tw = float(np.mean([e[0].elapsed_time(e[1]) for e in evs[3:]]))
tv = float(np.mean([e[1].elapsed_time(e[2]) for e in evs[3:]]))
alg_v = int(np.asarray(sizes, dtype=np.int64).sum()) + 22 * len(sizes)
print(json.dumps({"config": cfg, "trailer_ms": round(tw, 4), "verify_ms": round(tv, 4),
                  "verify_frac": round(alg_v / (tv / 1e3) / 8e12, 4)}), flush=True)
