#!/usr/bin/env python3
"""tools/prof_e2e.py -- A/B timing of bench.py's PCIe-inclusive path alone
(pinned host -> HBM -> verify -> host results, two streams, C2 batch) and the
host-memory entry points.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from forst_amd import engine, workload  # noqa: E402

engine.init_device()
sizes, ctype, desc, seed = bench.describe("C2", 1)
b = workload.make_sst_batch(len(sizes), None, seed, ctype=ctype, sizes=sizes)
engine.block_trailer_batch(ctype, b.base, b.offsets, b.sizes, b.types)
r = [round(bench.end_to_end_pcie(b, ctype), 2) for _ in range(3)]
print(json.dumps({"e2e_GiBps": r}), flush=True)
