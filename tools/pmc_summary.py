#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh output: per-launch averages of the counters of
the kernels whose name contains the filter, and per-block figures."""
import collections
import csv
import glob
import sys

tag, filt = sys.argv[1], sys.argv[2]
nblocks = int(sys.argv[3]) if len(sys.argv) > 3 else 0
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
waves = avg.get("SQ_WAVES", 1)
for k, v in avg.items():
    extra = f"  per block {v / nblocks:10.1f}" if nblocks and k.startswith("SQ_INSTS") else ""
    print(f"{k:24s} {v:16.0f}{extra}")
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in avg:
            print(f"{k:24s} {100 * avg[k] / wc:6.1f}% of wave cycles")
